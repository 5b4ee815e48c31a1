from .vec_env import VecEnv
from .ppo import *  # noqa: F401,F403
