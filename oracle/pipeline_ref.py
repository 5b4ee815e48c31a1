"""Full env-step oracle at the 12-DOF profile — TEST INFRASTRUCTURE ONLY.

Composes oracle/physics_ref.c (physics), oracle/envlogic_ref.py (reference arithmetic) and
oracle/rng_ref.py (the Philox draw schedule) into the exact sequence hg_step + hg_post run:
  prologue  humanoid_env.py:620-635   (delay blend, multiplicative noise, clip)
  physics   humanoid_env.py:639-649   (decimation x PD + simulate)
  post      humanoid_env.py:770-809   (derived state, callback, termination, reward, reset, obs)
State is a dict of numpy arrays in the reference's AoS shapes ([N,13] root, [N,13,3] contact...).
"""
import numpy as np

import envlogic_ref as E
import rng_ref as R

f32 = np.float32
L12 = E.LAYOUT12


class Cfg:
    """The subset of hg_cfg the pipeline needs, built from an HgCfg ctypes struct."""

    def __init__(self, c):
        self.c = c
        self.seed = int(c.seed)
        self.n = int(c.num_envs)
        self.P = E.Params(dt=c.dt, cycle_time=c.cycle_time, target_joint_pos_scale=c.target_joint_pos_scale,
                          target_feet_height=c.target_feet_height, base_height_target=c.base_height_target,
                          min_dist=c.min_dist, max_dist=c.max_dist, tracking_sigma=c.tracking_sigma,
                          max_contact_force=c.max_contact_force, max_episode_length=c.max_episode_length,
                          only_positive_rewards=bool(c.only_positive_rewards),
                          obs_scales=dict(lin_vel=c.obs_lin_vel, ang_vel=c.obs_ang_vel, dof_pos=c.obs_dof_pos,
                                          dof_vel=c.obs_dof_vel, quat=c.obs_quat),
                          noise_scales=dict(dof_pos=c.noise_dof_pos, dof_vel=c.noise_dof_vel, ang_vel=c.noise_ang_vel,
                                            quat=c.noise_quat),
                          noise_level=c.noise_level, clip_obs=c.clip_observations)
        self.default = np.array(c.default_dof_pos[:12], f32)
        self.scales = {n: float(c.reward_scale[k]) for k, n in enumerate(E.REWARD_NAMES)}
        self.L = E.Layout(D=12, ref_idx=tuple(c.ref_idx), yaw_roll=tuple(c.yaw_roll_idx),
                          feet=tuple(c.feet_body), knees=tuple(c.knee_body), base=0)


def preprocess_actions(cfg, actions_in, prev_actions, step):
    """k_step prologue (humanoid_env.py:624-635) with the Philox draws of hg_common.h."""
    c = cfg.c
    env = np.arange(cfg.n)
    delay = R.u01(R.rng4(cfg.seed, env, step, 0, R.ACT_DELAY)[0])[:, None]
    z = R.normals(cfg.seed, env, step, R.ACT_NOISE, 12)
    a = (f32(1.0) - delay) * actions_in.astype(f32) + delay * prev_actions
    a = a + f32(c.dynamic_randomization) * z * a
    return np.clip(a, -c.clip_actions, c.clip_actions).astype(f32)


def _resample(cfg, S, ids, step, salt):
    c = cfg.c
    if len(ids) == 0:
        return
    r = R.rng4(cfg.seed, ids, step, salt, R.CMD)
    cx = f32(c.cmd_lin_x[1] - c.cmd_lin_x[0]) * R.u01(r[0]) + f32(c.cmd_lin_x[0])
    cy = f32(c.cmd_lin_y[1] - c.cmd_lin_y[0]) * R.u01(r[1]) + f32(c.cmd_lin_y[0])
    if c.heading_command:
        S["commands"][ids, 3] = f32(c.cmd_heading[1] - c.cmd_heading[0]) * R.u01(r[2]) + f32(c.cmd_heading[0])
    else:
        S["commands"][ids, 2] = f32(c.cmd_ang_yaw[1] - c.cmd_ang_yaw[0]) * R.u01(r[2]) + f32(c.cmd_ang_yaw[0])
    keep = (np.sqrt(cx * cx + cy * cy) > 0.2).astype(f32)
    S["commands"][ids, 0] = cx * keep
    S["commands"][ids, 1] = cy * keep


def reset_envs(cfg, S, rid, counter):
    """reset_idx (humanoid_env.py:1109-1163) for env ids rid, Philox draws as k_post."""
    c = cfg.c
    if len(rid) == 0:
        return
    if c.curriculum and counter != 0:
        # _update_terrain_curriculum (humanoid_env.py:1075-1095); S["terrain_origins"] is the
        # host copy of the [rows, cols, 3] table
        d = S["root_states"][rid, :2] - S["env_origins"][rid, :2]
        dist = np.sqrt((d * d).sum(1, dtype=f32), dtype=f32)
        cmd = S["commands"][rid, :2]
        cn = np.sqrt((cmd * cmd).sum(1, dtype=f32), dtype=f32)
        up = dist > f32(c.terrain_env_length) / f32(2)
        down = (dist < cn * f32(c.max_episode_length_s) * f32(0.5)) & ~up
        lvl = S["terrain_levels"][rid].astype(np.int64) + up.astype(np.int64) - down.astype(np.int64)
        maxl = int(c.terrain_rows)
        rnd = np.minimum((R.u01(R.rng4(cfg.seed, rid, counter, 0, R.TERRAIN)[0]) * f32(maxl)).astype(np.int64), maxl - 1)
        lvl = np.where(lvl >= maxl, rnd, np.maximum(lvl, 0))
        S["terrain_levels"][rid] = lvl
        S["env_origins"][rid] = S["terrain_origins"][lvl, S["terrain_types"][rid]]
    u = np.concatenate([np.stack(R.rng4(cfg.seed, rid, counter, b, R.RESET_DOF), 1) for b in range(3)], 1)
    S["dof_pos"][rid] = cfg.default[None, :] + f32(0.2) * R.u01(u) + f32(-0.1)
    S["dof_vel"][rid] = 0
    root = np.zeros((len(rid), 13), f32)
    root[:, 0:3] = np.array(c.init_pos[:3], f32) + S["env_origins"][rid]
    root[:, 3:7] = np.array(c.init_rot[:4], f32)
    root[:, 7:10] = np.array(c.init_lin_vel[:3], f32)
    root[:, 10:13] = np.array(c.init_ang_vel[:3], f32)
    if c.terrain_type != 0:
        rr = R.rng4(cfg.seed, rid, counter, 0, R.RESET_ROOT)
        root[:, 0] += f32(2) * R.u01(rr[0]) - f32(1)
        root[:, 1] += f32(2) * R.u01(rr[1]) - f32(1)
    if c.fix_base_link:
        root[:, 7:13] = 0
        root[:, 2] += f32(1.8)
    S["root_states"][rid] = root
    S["lambda"][rid] = 0
    _resample(cfg, S, rid, counter, 1)
    for k in ("last_last_actions", "actions", "last_actions", "last_dof_vel", "feet_air_time"):
        S[k][rid] = 0
    S["episode_length_buf"][rid] = 0
    for name in S["episode_sums"]:
        S["episode_sums"][name][rid] = 0
    S["projected_gravity"][rid] = E.quat_rotate_inverse(root[:, 3:7], np.tile(np.array([0, 0, -1], f32), (len(rid), 1)))


def initial_state(cfg, env_origins, body_mass, frictions):
    """hg_create's k_init followed by hg_reset_masked(all) (humanoid_env.py:176-178); returns
    (S, obs_stack, priv_stack)."""
    c, n = cfg.c, cfg.n
    S = dict(root_states=np.zeros((n, 13), f32), dof_pos=np.tile(cfg.default, (n, 1)), dof_vel=np.zeros((n, 12), f32),
             contact_forces=np.zeros((n, 13, 3), f32), rigid_state=np.zeros((n, 13, 13), f32),
             torques=np.zeros((n, 12), f32), actions=np.zeros((n, 12), f32), last_actions=np.zeros((n, 12), f32),
             last_last_actions=np.zeros((n, 12), f32), last_dof_vel=np.zeros((n, 12), f32),
             last_root_vel=np.zeros((n, 6), f32), commands=np.zeros((n, 4), f32),
             episode_length_buf=np.zeros(n, np.int64), feet_air_time=np.zeros((n, 2), f32),
             last_contacts=np.zeros((n, 2), bool), feet_height=np.zeros((n, 2), f32),
             last_feet_z=np.full((n, 2), 0.05, f32), env_frictions=np.asarray(frictions, f32).reshape(n, 1),
             body_mass=np.asarray(body_mass, f32).reshape(n, 1), rand_push_force=np.zeros((n, 3), f32),
             rand_push_torque=np.zeros((n, 3), f32), ref_dof_pos=np.zeros((n, 12), f32),
             env_origins=np.asarray(env_origins, f32), lambda_=None, base_lin_vel=np.zeros((n, 3), f32),
             base_ang_vel=np.zeros((n, 3), f32), projected_gravity=np.tile(np.array([0, 0, -1], f32), (n, 1)))
    S.pop("lambda_")
    S["lambda"] = np.zeros((n, 60), f32)
    S["default_dof_pos"] = cfg.default[None, :]
    S["episode_sums"] = {name: np.zeros(n, f32) for name in E.REWARD_NAMES}
    reset_envs(cfg, S, np.arange(n), 0)
    S["base_euler_xyz"] = E.euler_xyz(S["root_states"][:, 3:7])
    noise = R.normals(cfg.seed, np.arange(n), 0, R.OBS_NOISE, 47) if c.add_noise else None
    o, p, ref = E.obs_frames(S, cfg.L, cfg.P, noise=noise)
    clip = f32(c.clip_observations)
    S["ref_dof_pos"] = ref
    obs = E.stack(np.zeros((n, c.frame_stack * 47), f32), np.clip(o, -clip, clip))
    priv = E.stack(np.zeros((n, c.c_frame_stack * 73), f32), np.clip(p, -clip, clip))
    return S, obs, priv


def post(cfg, S, counter, hist_obs, hist_priv):
    """One hg_post (mode 0).  Mutates S; returns (obs_stack, priv_stack, rew, reset, timeout, terms)."""
    c, P, L = cfg.c, cfg.P, cfg.L
    n = cfg.n
    env = np.arange(n)
    S["episode_length_buf"] = S["episode_length_buf"] + 1
    q = S["root_states"][:, 3:7]
    S["base_lin_vel"] = E.quat_rotate_inverse(q, S["root_states"][:, 7:10])
    S["base_ang_vel"] = E.quat_rotate_inverse(q, S["root_states"][:, 10:13])
    S["projected_gravity"] = E.quat_rotate_inverse(q, np.tile(np.array([0, 0, -1], f32), (n, 1)))
    S["base_euler_xyz"] = E.euler_xyz(q)
    ids = np.nonzero(S["episode_length_buf"] % c.resample_interval == 0)[0]
    _resample(cfg, S, ids, counter, 0)
    if c.heading_command:
        fwd = E.quat_apply(q, np.tile(np.array([1, 0, 0], f32), (n, 1)))
        heading = np.arctan2(fwd[:, 1], fwd[:, 0]).astype(f32)
        S["commands"][:, 2] = np.clip(f32(0.5) * E.wrap_to_pi(S["commands"][:, 3] - heading), -1.0, 1.0)
    if c.push_robots and counter % c.push_interval == 0:
        r0, r1 = R.rng4(cfg.seed, env, counter, 0, R.PUSH), R.rng4(cfg.seed, env, counter, 1, R.PUSH)
        mv, ma = f32(c.max_push_vel_xy), f32(c.max_push_ang_vel)
        S["rand_push_force"][:, 0] = f32(2) * mv * R.u01(r0[0]) - mv
        S["rand_push_force"][:, 1] = f32(2) * mv * R.u01(r0[1]) - mv
        S["root_states"][:, 7:9] = S["rand_push_force"][:, :2]
        for k, u in enumerate((r0[2], r0[3], r1[0])):
            S["rand_push_torque"][:, k] = f32(2) * ma * R.u01(u) - ma
        S["root_states"][:, 10:13] = S["rand_push_torque"]
    reset, timeout = E.termination(S["contact_forces"], S["episode_length_buf"], L, P)
    S["default_dof_pos"] = cfg.default[None, :]
    terms = E.rewards(S, L, P)
    rew = E.total_reward(terms, cfg.scales, S["episode_sums"], P)
    reset_envs(cfg, S, np.nonzero(reset)[0], counter)
    S["base_euler_xyz"] = E.euler_xyz(S["root_states"][:, 3:7])
    noise = R.normals(cfg.seed, env, counter, R.OBS_NOISE, 47) if c.add_noise else None
    o, p, ref = E.obs_frames(S, L, P, noise=noise)
    clip = f32(c.clip_observations)
    o, p = np.clip(o, -clip, clip), np.clip(p, -clip, clip)
    S["ref_dof_pos"] = ref
    obs = E.stack(hist_obs, o, reset)
    priv = E.stack(hist_priv, p, reset)
    S["last_last_actions"] = S["last_actions"].copy()
    S["last_actions"] = S["actions"].copy()
    S["last_dof_vel"] = S["dof_vel"].copy()
    S["last_root_vel"] = S["root_states"][:, 7:13].copy()
    return obs, priv, rew, reset, timeout, terms
