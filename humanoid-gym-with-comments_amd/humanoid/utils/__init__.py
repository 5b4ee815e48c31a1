from .helpers import (class_to_dict, get_load_path, get_args, export_policy_as_jit, set_seed,  # noqa: F401
                      update_class_from_dict, parse_sim_params, SimParams)
from .task_registry import task_registry  # noqa: F401
from .math import *  # noqa: F401,F403
