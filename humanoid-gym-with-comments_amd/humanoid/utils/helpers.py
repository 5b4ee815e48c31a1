"""Config/seed/checkpoint plumbing (reference humanoid/utils/helpers.py).

Isaac Gym's argument parser and SimParams are replaced by argparse and a small dataclass;
names, flags and behaviour of the helpers the training path uses are kept.
"""
import argparse
import copy
import os
import random
from dataclasses import dataclass, field

import numpy as np
import torch


def class_to_dict(obj) -> dict:
    """Nested config object -> dict; keys in dir() order (alphabetical), helpers.py:43-58."""
    if not hasattr(obj, "__dict__"):
        return obj
    out = {}
    for key in dir(obj):
        if key.startswith("_"):
            continue
        val = getattr(obj, key)
        out[key] = [class_to_dict(v) for v in val] if isinstance(val, list) else class_to_dict(val)
    return out


def update_class_from_dict(obj, d):
    for key, val in d.items():
        attr = getattr(obj, key, None)
        if isinstance(attr, type):
            update_class_from_dict(attr, val)
        else:
            setattr(obj, key, val)


def set_seed(seed):
    if seed == -1:
        seed = np.random.randint(0, 10000)
    print("Setting seed: {}".format(seed))
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    torch.cuda.manual_seed_all(seed)


@dataclass
class SimParams:
    """Stand-in for gymapi.SimParams: the fields the env reads."""
    dt: float = 0.001
    substeps: int = 1
    gravity: tuple = (0.0, 0.0, -9.81)
    up_axis: int = 1
    use_gpu_pipeline: bool = True
    physx: dict = field(default_factory=dict)


def parse_sim_params(args, cfg):
    sp = SimParams()
    sim = cfg.get("sim", {}) if isinstance(cfg, dict) else {}
    for k in ("dt", "substeps", "up_axis"):
        if k in sim:
            setattr(sp, k, sim[k])
    if "gravity" in sim:
        sp.gravity = tuple(sim["gravity"])
    sp.physx = dict(sim.get("physx", {}))
    return sp


def get_load_path(root, load_run=-1, checkpoint=-1):
    try:
        runs = sorted(r for r in os.listdir(root) if r not in ("exported", "openloop_action"))  # play.py outputs
        last_run = os.path.join(root, runs[-1])
    except Exception:
        raise ValueError("No runs in this directory: " + root)
    load_run = last_run if load_run == -1 else os.path.join(root, load_run)
    if checkpoint == -1:
        models = sorted((f for f in os.listdir(load_run) if "model" in f), key=lambda m: "{0:0>15}".format(m))
        model = models[-1]
    else:
        model = "model_{}.pt".format(checkpoint)
    return os.path.join(load_run, model)


def update_cfg_from_args(env_cfg, cfg_train, args):
    if env_cfg is not None and getattr(args, "num_envs", None) is not None:
        env_cfg.env.num_envs = args.num_envs
    if cfg_train is not None:
        if getattr(args, "seed", None) is not None:
            cfg_train.seed = args.seed
        for a, k in (("max_iterations", "max_iterations"), ("experiment_name", "experiment_name"),
                     ("run_name", "run_name"), ("load_run", "load_run"), ("checkpoint", "checkpoint")):
            if getattr(args, a, None) is not None:
                setattr(cfg_train.runner, k, getattr(args, a))
        if getattr(args, "resume", False):
            cfg_train.runner.resume = True
    return env_cfg, cfg_train


def get_args(argv=None):
    """Same flags as the reference (helpers.py:161-239) minus Isaac Gym's pipeline flags."""
    p = argparse.ArgumentParser(description="RL Policy")
    p.add_argument("--task", type=str, default="humanoid_ppo")
    p.add_argument("--resume", action="store_true", default=False)
    p.add_argument("--experiment_name", type=str)
    p.add_argument("--run_name", type=str)
    p.add_argument("--load_run", type=str)
    p.add_argument("--checkpoint", type=int)
    p.add_argument("--headless", action="store_true", default=False)
    p.add_argument("--horovod", action="store_true", default=False)
    p.add_argument("--rl_device", type=str, default="cuda:0")
    p.add_argument("--sim_device", type=str, default="cuda:0")
    p.add_argument("--num_envs", type=int)
    p.add_argument("--seed", type=int)
    p.add_argument("--max_iterations", type=int)
    args = p.parse_args(argv)
    args.physics_engine = "hg_sim"
    return args


def export_policy_as_jit(actor_critic, path):
    """TorchScript export of the actor and the lin-vel estimator (helpers.py:242-254)."""
    os.makedirs(path, exist_ok=True)
    torch.jit.script(copy.deepcopy(actor_critic.actor).to("cpu")).save(os.path.join(path, "policy_1.pt"))
    torch.jit.script(copy.deepcopy(actor_critic.base_lin_vel).to("cpu")).save(os.path.join(path, "base_lin_vel.pt"))
