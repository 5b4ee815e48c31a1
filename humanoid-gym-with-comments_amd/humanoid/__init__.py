"""MI355X-native drop-in for the rollout + update path of humanoid-gym (XBot-L).

Package layout and public names mirror the reference's ``humanoid`` package
(humanoid/__init__.py:35-36) so scripts written against it import unchanged.
"""
import os

LEGGED_GYM_ROOT_DIR = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
LEGGED_GYM_ENVS_DIR = os.path.join(LEGGED_GYM_ROOT_DIR, "humanoid", "envs")
