"""Evaluation loop (humanoid/scripts/play.py of the reference), headless.

    python -m humanoid.scripts.play --task humanoid_ppo --load_run <run> --resume [--steps 1000]

Loads the checkpoint, exports the actor (TorchScript policy_1.pt + base_lin_vel.pt, and ONNX
policy.onnx), runs the policy on a single environment with the reference's play settings and
writes the open-loop action trace (openloop_action.npz) plus per-step state logs (states.npz) and
the mean episode rewards.  There is no viewer or video: hg_sim has no renderer.

Reference defect fixed: play.py:77 sets ``train_cfg.runner.resume = True``, but
``make_alg_runner`` resets it to False before reading it (task_registry.py:137), so without an
explicit ``--resume`` the reference exports and plays the randomly initialised policy.  Here the
resume request travels in ``args``, which make_alg_runner honours: play always loads the
checkpoint (``--load_run`` / ``--checkpoint``, default the newest).
"""
import argparse
import os

import numpy as np
import torch

from humanoid import LEGGED_GYM_ROOT_DIR
from humanoid.envs import *  # noqa: F401,F403
from humanoid.utils import get_args, task_registry
from humanoid.utils.helpers import export_policy_as_jit
from humanoid.utils.onnx_io import export_policy_as_onnx

EXPORT_POLICY = True
FIX_COMMAND = True


def play(args, steps=100):
    env_cfg, train_cfg = task_registry.get_cfgs(name=args.task)
    env_cfg.env.num_envs = min(env_cfg.env.num_envs, 1)
    env_cfg.terrain.mesh_type = "plane"
    env_cfg.terrain.num_rows = 5
    env_cfg.terrain.num_cols = 5
    env_cfg.terrain.curriculum = False
    env_cfg.terrain.max_init_terrain_level = 5
    env_cfg.noise.add_noise = True
    env_cfg.domain_rand.push_robots = False
    env_cfg.noise.noise_level = 0.5
    train_cfg.seed = 123145
    env, _ = task_registry.make_env(name=args.task, args=args, env_cfg=env_cfg)
    obs = env.get_observations()
    train_cfg.runner.resume = True
    args.resume = True  # see the module docstring (task_registry.py:137 would drop the line above)
    runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args, train_cfg=train_cfg)
    policy = runner.get_inference_policy(device=env.device)
    root = os.path.join(LEGGED_GYM_ROOT_DIR, "logs", train_cfg.runner.experiment_name)
    if EXPORT_POLICY:
        path = os.path.join(root, "exported", "policies")
        export_policy_as_jit(runner.alg.actor_critic, path)
        export_policy_as_onnx(runner.alg.actor_critic, path)
        print("Exported policy (TorchScript + ONNX) to:", path)
    actions_log, states = [], {k: [] for k in ("dof_pos", "dof_vel", "dof_torque", "command_x", "base_vel_x",
                                               "base_vel_yaw", "contact_forces_z")}
    rew_sums, n_eps = {}, 0
    for _ in range(steps):
        with torch.no_grad():
            actions = policy(obs.detach())
        actions_log.append(actions[0].cpu().numpy())
        if FIX_COMMAND:
            env.commands[:, 0] = 0.5
            env.commands[:, 1:4] = 0.0
        obs, _, _, _, infos = env.step(actions.detach())
        states["dof_pos"].append(env.dof_pos[0].cpu().numpy())
        states["dof_vel"].append(env.dof_vel[0].cpu().numpy())
        states["dof_torque"].append(env.torques[0].cpu().numpy())
        states["command_x"].append(float(env.commands[0, 0]))
        states["base_vel_x"].append(float(env.base_lin_vel[0, 0]))
        states["base_vel_yaw"].append(float(env.base_ang_vel[0, 2]))
        states["contact_forces_z"].append(env.contact_forces[0, env.feet_indices, 2].cpu().numpy())
        k = int(env.reset_buf.sum().item())
        if k > 0:
            n_eps += k
            for name, v in infos["episode"].items():
                rew_sums[name] = rew_sums.get(name, 0.0) + float(v) * k
    out = os.path.join(root, "openloop_action")
    os.makedirs(out, exist_ok=True)
    np.savez(os.path.join(out, "openloop_action.npz"), action=np.array(actions_log))
    np.savez(os.path.join(out, "states.npz"), **{k: np.array(v) for k, v in states.items()})
    if n_eps:
        print(f"Average rewards per second over {n_eps} episodes:")
        for name, v in rew_sums.items():
            print(f" - {name}: {v / n_eps:.4f}")
    return np.array(actions_log)


if __name__ == "__main__":
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--steps", type=int, default=100)
    extra, rest = ap.parse_known_args()
    play(get_args(rest), steps=extra.steps)
