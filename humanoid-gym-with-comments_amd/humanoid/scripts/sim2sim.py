"""Sim-to-sim evaluation of an exported policy (humanoid/scripts/sim2sim.py of the reference), headless
and batched.

The reference loads ``policy_1.pt`` into MuJoCo (XBot-L.xml) and drives it at 100 Hz with a 1 kHz
PD loop, building the policy input itself from the simulator's raw state (sim2sim.py:79-90
``get_obs``, :186-207 the observation frame and its 15-frame history) with joystick commands and
a viewer.  MuJoCo is not installed here, so the second simulator is this build's own hg_sim run
with the robot's **MJCF parameter profile** instead of the Isaac Gym asset's — the differences a
policy trained on the URDF profile meets when it is transferred:

  * joint armature 0.01 kg m^2 (``leg_joint_param``, XBot-L.xml:37-39; the asset uses 0,
    humanoid_config.py:118);
  * joint frictionloss 0.01 N m on every leg joint, 0.05 N m on the ankles (:38, :426, :431, :476,
    :481; the URDF has 0.1 N m on the ankles only);
  * joint damping 0.01 N m s/rad (:38), added to the PD damping — a stated deviation: MuJoCo's
    passive damping is never clipped, while the folded term is clipped with the PD torque at the
    200 N m limit and loses its implicit integration on a saturated joint (0.01 against kd = 10:
    0.1 % of the damping, and only on saturated joints);
  * ground/foot friction 0.9 (the default geom friction, :14; MuJoCo's max-combine of two 0.9
    geoms), no friction randomisation;
  * 50 solver iterations (``<option iterations='50' solver='PGS'>``, :3) instead of 4 + 1;
  * the MJCF trunk: 0.951 kg lighter than the URDF's (tests/test_model_mjcf.py), applied as a
    base-mass offset (its 1-2 cm COM shift is not modelled);
  * the sim2sim PD loop's torque clip of 200 N m on every joint (sim2sim.py:309) instead of the
    env's effort x 0.85.

``--profile urdf`` runs the training profile instead (the same physics the policy was trained in).
Every env holds a fixed velocity command (a grid over --vx/--vy/--wz instead of the joystick);
domain randomisation, pushes, the env's action-delay blend and observation noise are off.  The
policy input is built here from the raw state exactly as sim2sim.py builds it — phase sin/cos, commands x obs
scales, q - q_default, dq x 0.05, last action, base angular velocity, roll/pitch/yaw (wrapped to
(-pi, pi]) — clipped to +-18 and stacked oldest-first over 15 frames; the env's own observation
pipeline (K_post) is not used as the policy input.  The gait phase uses the trained cycle time
(``rewards.cycle_time``, 0.64 s) where the reference script hard-codes its D11 robot's 0.85 s.

Outputs (``--out``): ``sim2sim.json`` with per-command tracking errors, fall counts and survival
time, and ``sim2sim_traces.npz`` (per-step base velocities, joint targets and positions of env 0).

    python -m humanoid.scripts.sim2sim --load_model <.../exported/policies/policy_1.pt> \
        [--profile mjcf|urdf] [--duration 20] [--vx -0.25 0.0 0.4] [--vy 0.0] [--wz 0.0]
"""
import argparse
import ctypes
import itertools
import json
import math
import os

import numpy as np
import torch

from humanoid import _native as N

MJCF_PROFILE = dict(
    armature=0.01,
    joint_friction={"joint": 0.01, "ankle": 0.05},
    joint_damping=0.01,
    friction=0.9,
    pgs_iterations=50,
    trunk_mass_delta=-0.951,
    tau_limit=200.0,
)


def make_cfg(profile, num_envs, duration, self_collisions=True):
    """XBotLCfg for a sim2sim run: fixed commands, no randomisation/noise/pushes, the profile's
    physics parameters (see the module docstring).  self_collisions=False drops every
    self-collision pair (asset.self_collisions = 1; ablation runs only)."""
    from humanoid.envs import XBotLCfg
    cfg = XBotLCfg()
    if not self_collisions:
        cfg.asset.self_collisions = 1
    cfg.env.num_envs = num_envs
    cfg.env.episode_length_s = duration + 1.0
    cfg.terrain.mesh_type = "plane"
    cfg.terrain.curriculum = False
    cfg.noise.add_noise = False
    cfg.domain_rand.randomize_friction = False
    cfg.domain_rand.randomize_base_mass = False
    cfg.domain_rand.push_robots = False
    cfg.domain_rand.dynamic_randomization = 0.0
    cfg.commands.heading_command = False
    cfg.commands.resampling_time = duration + 1.0
    if profile == "mjcf":
        p = MJCF_PROFILE
        cfg.sim.hg.armature = p["armature"]
        cfg.sim.hg.joint_friction = dict(p["joint_friction"])
        cfg.sim.hg.pgs_iterations = p["pgs_iterations"]
        cfg.terrain.static_friction = p["friction"]
        cfg.control.damping = {k: v + p["joint_damping"] for k, v in cfg.control.damping.items()}
    elif profile != "urdf":
        raise ValueError(f"profile must be 'mjcf' or 'urdf', got {profile!r}")
    return cfg


def make_env(profile, num_envs, duration, device="cuda:0", self_collisions=True):
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    cfg = make_cfg(profile, num_envs, duration, self_collisions)
    env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", device, True)
    if profile == "mjcf":
        p = MJCF_PROFILE
        env.env_frictions[:] = p["friction"]
        env.body_mass[:] = env.body_mass + p["trunk_mass_delta"]
        for j in range(env.num_actions):
            env._hgcfg.torque_limit[j] = p["tau_limit"]
        stream = ctypes.c_void_p(torch.cuda.current_stream(env.device).cuda_stream)
        N.check(env.hg.hg_update_cfg(env.sim, ctypes.byref(env._hgcfg), stream), env.sim)
    return env


def quat_to_euler(q):
    """sim2sim.py:53-76 ``quaternion_to_euler_array`` for [N, 4] (x, y, z, w) rows, wrapped as
    sim2sim.py:188 does (angles > pi shifted by -2 pi; atan2 / asin already lie in [-pi, pi])."""
    x, y, z, w = q.unbind(-1)
    roll = torch.atan2(2.0 * (w * x + y * z), 1.0 - 2.0 * (x * x + y * y))
    pitch = torch.asin(torch.clamp(2.0 * (w * y - z * x), -1.0, 1.0))
    yaw = torch.atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z))
    e = torch.stack([roll, pitch, yaw], dim=-1)
    return torch.where(e > math.pi, e - 2.0 * math.pi, e)


def quat_rotate_inverse(q, v):
    """v expressed in the frame of the (x, y, z, w) quaternion q (rows)."""
    qv, w = q[:, :3], q[:, 3:4]
    a = v * (2.0 * w * w - 1.0)
    b = torch.cross(qv, v, dim=-1) * w * 2.0
    c = qv * (qv * v).sum(-1, keepdim=True) * 2.0
    return a - b + c


def obs_frame(env, cmd, action, t):
    """One sim2sim observation frame (sim2sim.py:186-202) per env from the raw simulator state."""
    cfg = env.cfg
    sc = cfg.normalization.obs_scales
    rs = env.root_states
    quat = rs[:, 3:7]
    omega = quat_rotate_inverse(quat, rs[:, 10:13])
    n = env.num_envs
    ph = 2.0 * math.pi * t / cfg.rewards.cycle_time
    frame = torch.empty(n, cfg.env.num_single_obs, dtype=torch.float32, device=env.device)
    frame[:, 0] = math.sin(ph)
    frame[:, 1] = math.cos(ph)
    frame[:, 2] = cmd[:, 0] * sc.lin_vel
    frame[:, 3] = cmd[:, 1] * sc.lin_vel
    frame[:, 4] = cmd[:, 2] * sc.ang_vel
    frame[:, 5:17] = (env.dof_pos - env.default_dof_pos) * sc.dof_pos
    frame[:, 17:29] = env.dof_vel * sc.dof_vel
    frame[:, 29:41] = action
    frame[:, 41:44] = omega
    frame[:, 44:47] = quat_to_euler(quat)
    clip = cfg.normalization.clip_observations
    return torch.clamp(frame, -clip, clip)


def step_direct(env, action):
    """env.step(action) with the policy output applied as sim2sim.py applies it.  The env's step
    prologue blends the new action with the previous one by a random delay (humanoid_env.py:624-626,
    always on in the reference's env); presetting the previous action to the new one makes that
    blend the identity (to one rounding), as in the reference script's PD loop."""
    env.actions[:] = action
    return env.step(action)


def command_grid(vx, vy, wz):
    return np.array(list(itertools.product(vx, vy, wz)), dtype=np.float32)


def load_policy(path, device="cuda:0"):
    """The actor to drive: a TorchScript export (policy_1.pt), an ONNX actor (Gemm/Elu chain, e.g.
    the reference's humanoid/OnnxTest.onnx) or a weights npz (W0, b0, ..., W3, b3 in nn.Linear
    layout; tests/golden/onnx_actor.npz).  ONNX and npz files are read as numbers only."""
    if path.endswith(".onnx"):
        from humanoid.utils.onnx_io import load_onnx_mlp
        return load_onnx_mlp(path).to(device).eval()
    if path.endswith(".npz"):
        return mlp_from_weights(np.load(path, allow_pickle=False)).to(device).eval()
    return torch.jit.load(path, map_location=device)


def mlp_from_weights(w):
    """nn.Sequential(Linear, ELU, ..., Linear) from a W0, b0, W1, b1, ... dict."""
    import torch.nn as nn
    layers, k = [], 0
    while f"W{k}" in w:
        W, b = np.asarray(w[f"W{k}"], np.float32), np.asarray(w[f"b{k}"], np.float32)
        lin = nn.Linear(W.shape[1], W.shape[0])
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy(W))
            lin.bias.copy_(torch.from_numpy(b))
        if layers:
            layers.append(nn.ELU())
        layers.append(lin)
        k += 1
    return nn.Sequential(*layers)


def run(policy, profile="mjcf", commands=((0.4, 0.0, 0.0),), duration=10.0, envs_per_command=4,
        device="cuda:0", trace_env=0, env=None, record_q=False):
    """Drive ``policy`` (TorchScript or any callable [N, 705] -> [N, 12]) in the sim2sim loop.
    ``env``: an env made by make_env(profile, len(commands) * envs_per_command, duration) whose
    initial state the caller has read (the oracle comparison starts from it).  ``record_q``: keep
    every env's joint positions per step (traces["q_all"], [steps, N, 12]).
    Returns (summary dict, traces dict)."""
    cmds = np.asarray(commands, dtype=np.float32).reshape(-1, 3)
    n = len(cmds) * envs_per_command
    if env is None:
        env = make_env(profile, n, duration, device)
    assert env.num_envs == n
    cmd = torch.tensor(np.repeat(cmds, envs_per_command, axis=0), device=env.device)
    cfg = env.cfg
    stack, nso = cfg.env.frame_stack, cfg.env.num_single_obs
    hist = torch.zeros(n, stack * nso, dtype=torch.float32, device=env.device)
    action = torch.zeros(n, env.num_actions, dtype=torch.float32, device=env.device)
    steps = int(round(duration / env.dt))
    clip_a = cfg.normalization.clip_actions
    err_v = torch.zeros(n, dtype=torch.float64, device=env.device)
    err_w = torch.zeros(n, dtype=torch.float64, device=env.device)
    alive_steps = torch.zeros(n, dtype=torch.float64, device=env.device)
    falls = torch.zeros(n, dtype=torch.int64, device=env.device)
    fall_step = torch.full((n,), -1, dtype=torch.int64, device=env.device)
    alive = torch.ones(n, dtype=torch.bool, device=env.device)
    tr = {k: [] for k in ("base_vel", "base_wz", "target_q", "q", "height")}
    q_all = []
    env.rows_dropped.zero_()  # the counter is cumulative over the sim's life (include/hgsim.h)
    with torch.no_grad():
        for k in range(steps):
            env.commands[:, :3] = cmd
            frame = obs_frame(env, cmd, action, k * env.dt)
            hist = torch.cat([hist[:, nso:], frame], dim=1)   # oldest first (sim2sim.py:204-206)
            action = torch.clamp(policy(hist).float(), -clip_a, clip_a)
            _, _, _, reset, _ = step_direct(env, action)
            vb = env.base_lin_vel
            wz = env.base_ang_vel[:, 2]
            fell = reset.bool()
            falls += fell.long()
            fall_step = torch.where(fell & alive, torch.full_like(fall_step, k + 1), fall_step)
            alive &= ~fell
            if record_q:
                q_all.append(env.dof_pos.clone())
            live = alive.double()
            err_v += live * torch.linalg.vector_norm(vb[:, :2] - cmd[:, :2], dim=1).double()
            err_w += live * (wz - cmd[:, 2]).abs().double()
            alive_steps += live
            if trace_env is not None:
                tr["base_vel"].append(vb[trace_env, :2].cpu().numpy())
                tr["base_wz"].append(float(wz[trace_env]))
                tr["target_q"].append((action[trace_env] * cfg.control.action_scale
                                       + env.default_dof_pos[0]).cpu().numpy())
                tr["q"].append(env.dof_pos[trace_env].cpu().numpy())
                tr["height"].append(float(env.root_states[trace_env, 2]))
            if fell.any():
                hist[fell] = 0.0
                action[fell] = 0.0
    torch.cuda.synchronize(env.device)
    per = []
    for c in range(len(cmds)):
        s = slice(c * envs_per_command, (c + 1) * envs_per_command)
        a = alive_steps[s].clamp(min=1.0)
        per.append(dict(command=[float(x) for x in cmds[c]],
                        lin_vel_error=float((err_v[s] / a).mean()), yaw_rate_error=float((err_w[s] / a).mean()),
                        falls=int(falls[s].sum()), survival_s=float(alive_steps[s].mean() * env.dt)))
    summary = dict(profile=profile, duration_s=duration, envs=n, envs_per_command=envs_per_command,
                   policy_dt=env.dt, sim_dt=env.sim_dt, pgs_iterations=int(env._hgcfg.pgs_iterations),
                   commands=per, falls=int(falls.sum()),
                   survived_fraction=float((falls == 0).double().mean()),
                   fall_step=fall_step.cpu().tolist(), rows_dropped=int(env.rows_dropped.sum()))
    traces = {k: np.asarray(v) for k, v in tr.items()}
    if record_q:
        traces["q_all"] = torch.stack(q_all).cpu().numpy()
    return summary, traces


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--load_model", required=True,
                    help="TorchScript actor (exported policy_1.pt), ONNX actor (.onnx) or weights (.npz)")
    ap.add_argument("--profile", default="mjcf", choices=["mjcf", "urdf"])
    ap.add_argument("--duration", type=float, default=20.0, help="seconds of simulated time")
    ap.add_argument("--vx", type=float, nargs="+", default=[-0.25, 0.0, 0.4])
    ap.add_argument("--vy", type=float, nargs="+", default=[0.0])
    ap.add_argument("--wz", type=float, nargs="+", default=[0.0])
    ap.add_argument("--envs_per_command", type=int, default=16)
    ap.add_argument("--out", default=None, help="output directory (default: next to the policy)")
    a = ap.parse_args(argv)
    policy = load_policy(a.load_model)
    summary, traces = run(policy, a.profile, command_grid(a.vx, a.vy, a.wz), a.duration, a.envs_per_command)
    out = a.out or os.path.join(os.path.dirname(os.path.abspath(a.load_model)), f"sim2sim_{a.profile}")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "sim2sim.json"), "w") as f:
        json.dump(summary, f, indent=1)
    np.savez(os.path.join(out, "sim2sim_traces.npz"), **traces)
    for c in summary["commands"]:
        print(f"cmd {c['command']}: |v_xy - cmd| {c['lin_vel_error']:.3f} m/s  |wz - cmd| {c['yaw_rate_error']:.3f} "
              f"rad/s  falls {c['falls']}  survival {c['survival_s']:.1f} s")
    print(f"profile {a.profile}: survived {summary['survived_fraction'] * 100:.0f} % of {summary['envs']} envs -> {out}")
    return summary


if __name__ == "__main__":
    main()
