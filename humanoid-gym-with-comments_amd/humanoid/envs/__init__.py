"""Env registry (reference humanoid/envs/__init__.py:48-50; the missing D11/D12 envs are not
registered)."""
from humanoid import LEGGED_GYM_ROOT_DIR, LEGGED_GYM_ENVS_DIR  # noqa: F401
from .custom.humanoid_config import XBotLCfg, XBotLCfgPPO
from .custom.humanoid_env import XBotLFreeEnv
from humanoid.utils.task_registry import task_registry

task_registry.register("humanoid_ppo", XBotLFreeEnv, XBotLCfg(), XBotLCfgPPO())
