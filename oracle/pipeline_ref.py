"""Full env-step oracle — TEST INFRASTRUCTURE ONLY.

Composes oracle/physics_ref.c (physics), oracle/envlogic_ref.py (reference arithmetic) and a draw
source into the exact sequence hg_step + hg_post run:
  prologue  humanoid_env.py:616-635   (delay blend, multiplicative noise, clip)
  physics   humanoid_env.py:639-649   (decimation x PD + simulate)
  post      humanoid_env.py:770-809   (derived state, callback, termination, reward, reset, obs)
  obs clip  humanoid_env.py:654-657
State is a dict of numpy arrays in the reference's AoS shapes ([N,13] root, [N,13,3] contact...).
Every function is DOF-layout generic (width from the state arrays, index maps from
``cfg.L``), so the same code runs at the 12-DOF XBot-L profile the kernels implement and at the
fork's native 18-DOF layout, where it is pinned against the reference itself.

Random draws.  The reference draws from torch's global generator (humanoid_env.py:624-631,
:868, :1018-1032, :665-681, :1038-1066, :1090-1092); the kernels draw counter-based Philox
(csrc/hg_common.h).  Both are behind one interface:
  * ``PhiloxDraws`` — the kernels' draw schedule, bit for bit (oracle/rng_ref.py);
  * ``InjectedDraws`` — the raw uniforms / normals / integers recorded while the reference's own
    methods ran with torch's RNG calls intercepted (tests/golden/gen_goldens.py, pipeline18.npz):
    with these the oracle must reproduce the reference's outputs (tests/test_oracle_pipeline.py).
The arithmetic that turns draws into state (ranges, association order) is shared, so pinning the
injected path pins the Philox path's arithmetic too.
"""
import numpy as np

import envlogic_ref as E
import rng_ref as R

f32 = np.float32
L12 = E.LAYOUT12


class Cfg:
    """The subset of hg_cfg the pipeline needs, from an HgCfg ctypes struct or any object with the
    same field names (tests build an 18-DOF one from the reference's config).  ``L`` (Layout) and
    ``default`` may be overridden for layouts other than the 12-DOF profile."""

    def __init__(self, c, L=None, default=None):
        self.c = c
        self.seed = int(c.seed)
        self.n = int(c.num_envs)
        self.offset = int(getattr(c, "env_offset", 0))   # the shard's first global env id
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
        self.default = np.asarray(c.default_dof_pos[:12] if default is None else default, f32)
        self.scales = {n: float(c.reward_scale[k]) for k, n in enumerate(E.REWARD_NAMES)}
        self.L = L if L is not None else E.Layout(D=12, ref_idx=tuple(c.ref_idx), yaw_roll=tuple(c.yaw_roll_idx),
                                                  feet=tuple(c.feet_body), knees=tuple(c.knee_body), base=0)


# ------------------------------------------------------------------------------------------ draws
class PhiloxDraws:
    """The kernels' draw schedule (csrc/hg_common.h rng4 + csrc/hg_envlogic.hip / hg_physics.hip)."""

    def __init__(self, seed, n, offset=0):
        # offset: the shard's first GLOBAL env id (data parallel): every stream is keyed
        # by the global id, as the kernels key theirs (cfg.env_offset + local index)
        self.seed, self.n, self.off = seed, n, int(offset)

    def _all(self):
        return np.arange(self.n) + self.off

    def act_delay(self, step):                       # torch.rand((N, 1))           :624
        return R.u01(R.rng4(self.seed, self._all(), step, 0, R.ACT_DELAY)[0])[:, None]

    def act_noise(self, step, D):                    # torch.randn_like(actions)     :631
        return R.normals(self.seed, self._all(), step, R.ACT_NOISE, D)

    def cmd(self, ids, step, salt):                  # 3 x torch_rand_float         :1024-1030
        r = R.rng4(self.seed, np.asarray(ids) + self.off, step, salt, R.CMD)
        return R.u01(r[0]), R.u01(r[1]), R.u01(r[2])

    def push(self, step):                            # torch_rand_float (N,2), (N,3) :672-677
        r0, r1 = R.rng4(self.seed, self._all(), step, 0, R.PUSH), R.rng4(self.seed, self._all(), step, 1, R.PUSH)
        return np.stack([R.u01(r0[0]), R.u01(r0[1])], 1), np.stack([R.u01(r0[2]), R.u01(r0[3]), R.u01(r1[0])], 1)

    def reset_dof(self, rid, counter, D):            # torch_rand_float (n, D)       :1044
        blocks = (D + 3) // 4
        g = np.asarray(rid) + self.off
        u = np.concatenate([np.stack(R.rng4(self.seed, g, counter, b, R.RESET_DOF), 1) for b in range(blocks)], 1)
        return R.u01(u[:, :D])

    def reset_root(self, rid, counter):              # torch_rand_float (n, 2)       :1062
        rr = R.rng4(self.seed, np.asarray(rid) + self.off, counter, 0, R.RESET_ROOT)
        return np.stack([R.u01(rr[0]), R.u01(rr[1])], 1)

    def terrain_level(self, rid, counter, maxl):     # torch.randint_like(levels, maxl) :1091
        u = R.u01(R.rng4(self.seed, np.asarray(rid) + self.off, counter, 0, R.TERRAIN)[0])
        return np.minimum((u * f32(maxl)).astype(np.int64), maxl - 1)

    def obs_noise(self, step, width):                # torch.randn_like(obs_now)     :868
        return R.normals(self.seed, self._all(), step, R.OBS_NOISE, width)


class InjectedDraws:
    """Draws recorded from the reference (tests/golden/gen_goldens.py): a dict purpose -> list of
    arrays in call order.  Each request pops the next recorded array of its purpose and checks
    its shape, so a call-order or shape mismatch with the reference fails loudly."""

    def __init__(self, recorded):
        self.q = {k: list(v) for k, v in recorded.items()}

    def _pop(self, key, shape):
        if not self.q.get(key):
            raise AssertionError(f"no recorded draw left for {key}")
        a = np.asarray(self.q[key].pop(0))
        if tuple(a.shape) != tuple(shape):
            raise AssertionError(f"draw {key}: recorded shape {a.shape}, requested {shape}")
        return a

    def act_delay(self, step):
        return self._pop("step:rand", (self._n, 1)).astype(f32)

    def act_noise(self, step, D):
        return self._pop("step:randn_like", (self._n, D)).astype(f32)

    def cmd(self, ids, step, salt):
        key = "callback:cmd" if salt == 0 else "reset:cmd"
        n = len(ids)
        return tuple(self._pop(key, (n, 1))[:, 0].astype(f32) for _ in range(3))

    def push(self, step):
        return self._pop("push", (self._n, 2)).astype(f32), self._pop("push", (self._n, 3)).astype(f32)

    def reset_dof(self, rid, counter, D):
        return self._pop("reset:dof", (len(rid), D)).astype(f32)

    def reset_root(self, rid, counter):
        return self._pop("reset:root", (len(rid), 2)).astype(f32)

    def terrain_level(self, rid, counter, maxl):
        return self._pop("curriculum:randint", (len(rid),)).astype(np.int64)

    def obs_noise(self, step, width):
        return self._pop("obs:randn_like", (self._n, width)).astype(f32)

    def bind(self, n):
        self._n = n
        return self


def _draws(cfg, draws):
    return PhiloxDraws(cfg.seed, cfg.n, cfg.offset) if draws is None else draws


def _rand_float(lo, hi, u):
    """isaacgym.torch_utils.torch_rand_float: (upper - lower) * u + lower, float32."""
    return (f32(hi - lo) * u + f32(lo)).astype(f32)


# ------------------------------------------------------------------------------------------ pieces
def preprocess_actions(cfg, actions_in, prev_actions, step, draws=None):
    """step() prologue (humanoid_env.py:624-635): delay blend, multiplicative noise, clip."""
    c = cfg.c
    d = _draws(cfg, draws)
    D = actions_in.shape[1]
    delay = d.act_delay(step)
    z = d.act_noise(step, D)
    a = (f32(1.0) - delay) * actions_in.astype(f32) + delay * prev_actions
    a = a + f32(c.dynamic_randomization) * z * a
    return np.clip(a, -c.clip_actions, c.clip_actions).astype(f32)


def _resample(cfg, S, ids, step, salt, draws=None):
    """_resample_commands (humanoid_env.py:1018-1032)."""
    c = cfg.c
    if len(ids) == 0:
        return
    ux, uy, uh = _draws(cfg, draws).cmd(ids, step, salt)
    cx = _rand_float(c.cmd_lin_x[0], c.cmd_lin_x[1], ux)
    cy = _rand_float(c.cmd_lin_y[0], c.cmd_lin_y[1], uy)
    if c.heading_command:
        S["commands"][ids, 3] = _rand_float(c.cmd_heading[0], c.cmd_heading[1], uh)
    else:
        S["commands"][ids, 2] = _rand_float(c.cmd_ang_yaw[0], c.cmd_ang_yaw[1], uh)
    keep = (np.sqrt(cx * cx + cy * cy) > 0.2).astype(f32)
    S["commands"][ids, 0] = cx * keep
    S["commands"][ids, 1] = cy * keep


def push_robots(cfg, S, counter, draws=None):
    """_push_robots (humanoid_env.py:665-681): every env's root velocity is overwritten."""
    c = cfg.c
    uf, ut = _draws(cfg, draws).push(counter)
    mv, ma = c.max_push_vel_xy, c.max_push_ang_vel
    S["rand_push_force"][:, :2] = _rand_float(-mv, mv, uf)
    S["root_states"][:, 7:9] = S["rand_push_force"][:, :2]
    S["rand_push_torque"] = _rand_float(-ma, ma, ut)
    S["root_states"][:, 10:13] = S["rand_push_torque"]


def terrain_curriculum(cfg, S, rid, counter, draws=None):
    """_update_terrain_curriculum (humanoid_env.py:1075-1095); S["terrain_origins"] is the host
    copy of the [rows, cols, 3] table.  The reference skips it before init_done (counter 0)."""
    c = cfg.c
    d = S["root_states"][rid, :2] - S["env_origins"][rid, :2]
    dist = np.sqrt((d * d).sum(1, dtype=f32), dtype=f32)
    cmd = S["commands"][rid, :2]
    cn = np.sqrt((cmd * cmd).sum(1, dtype=f32), dtype=f32)
    up = dist > f32(c.terrain_env_length) / f32(2)
    down = (dist < cn * f32(c.max_episode_length_s) * f32(0.5)) & ~up
    lvl = S["terrain_levels"][rid].astype(np.int64) + up.astype(np.int64) - down.astype(np.int64)
    maxl = int(c.terrain_rows)
    rnd = _draws(cfg, draws).terrain_level(rid, counter, maxl)
    lvl = np.where(lvl >= maxl, rnd, np.maximum(lvl, 0))
    S["terrain_levels"][rid] = lvl
    S["env_origins"][rid] = S["terrain_origins"][lvl, S["terrain_types"][rid]]


def reset_envs(cfg, S, rid, counter, draws=None):
    """reset_idx (humanoid_env.py:1109-1163) for env ids rid: curriculum, _reset_dofs,
    _reset_root_states, _resample_commands, buffer zeroing, extras["episode"] means, projected
    gravity.  Returns the episode reward means (rew_<name> of extras["episode"]) or None."""
    c = cfg.c
    if len(rid) == 0:
        return None
    d = _draws(cfg, draws)
    if c.curriculum and counter != 0:
        terrain_curriculum(cfg, S, rid, counter, d)
    D = S["dof_pos"].shape[1]
    u = d.reset_dof(rid, counter, D)
    # default + torch_rand_float(-0.1, 0.1, ...)
    S["dof_pos"][rid] = cfg.default[None, :] + _rand_float(-0.1, 0.1, u)
    S["dof_vel"][rid] = 0
    root = np.zeros((len(rid), 13), f32)
    root[:, 0:3] = np.array(c.init_pos[:3], f32) + S["env_origins"][rid]
    root[:, 3:7] = np.array(c.init_rot[:4], f32)
    root[:, 7:10] = np.array(c.init_lin_vel[:3], f32)
    root[:, 10:13] = np.array(c.init_ang_vel[:3], f32)
    if c.terrain_type != 0:  # custom origins: xy within 1 m of the centre
        root[:, 0:2] += _rand_float(-1.0, 1.0, d.reset_root(rid, counter))
    if c.fix_base_link:
        root[:, 7:13] = 0
        root[:, 2] += f32(1.8)
    S["root_states"][rid] = root
    if "lambda" in S:
        S["lambda"][rid] = 0  # solver warm start (no reference counterpart)
    _resample(cfg, S, rid, counter, 1, d)
    for k in ("last_last_actions", "actions", "last_actions", "last_dof_vel", "feet_air_time"):
        S[k][rid] = 0
    S["episode_length_buf"][rid] = 0
    means = {}
    for name in S["episode_sums"]:
        means[name] = f32(np.mean(S["episode_sums"][name][rid], dtype=f32) / f32(c.max_episode_length_s))
        S["episode_sums"][name][rid] = 0
    S["projected_gravity"][rid] = E.quat_rotate_inverse(root[:, 3:7], np.tile(np.array([0, 0, -1], f32), (len(rid), 1)))
    return means


def heights(cfg, root_states, points_xy, hf):
    """_get_heights (humanoid_env.py:949-985) on the heightfield hf [rows, cols] int16 with the
    base-frame sample grid points_xy [P, 2]: quat_apply_yaw (utils/math.py:39-43), + base
    position + border, / horizontal_scale truncated, clipped, min of 3 neighbours x vertical_scale."""
    c = cfg.c
    n, P = root_states.shape[0], points_xy.shape[0]
    q = root_states[:, 3:7].astype(f32)
    qy = np.zeros_like(q)
    qy[:, 2:4] = q[:, 2:4]
    qy = qy / np.maximum(np.linalg.norm(qy, axis=1, keepdims=True), f32(1e-9)).astype(f32)
    pts = np.concatenate([points_xy.astype(f32), np.zeros((P, 1), f32)], 1)
    p = E.quat_apply(np.repeat(qy, P, 0), np.tile(pts, (n, 1))).reshape(n, P, 3)
    p = p + root_states[:, None, :3].astype(f32)
    p = p + f32(c.hf_border)
    ij = (p / f32(c.hf_horizontal_scale)).astype(np.int64)  # .long() truncates toward zero
    px = np.clip(ij[:, :, 0].reshape(-1), 0, hf.shape[0] - 2)
    py = np.clip(ij[:, :, 1].reshape(-1), 0, hf.shape[1] - 2)
    h = np.minimum(np.minimum(hf[px, py], hf[px + 1, py]), hf[px, py + 1])
    return (h.reshape(n, P).astype(f32) * f32(c.hf_vertical_scale)).astype(f32)


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
             env_origins=np.asarray(env_origins, f32), base_lin_vel=np.zeros((n, 3), f32),
             base_ang_vel=np.zeros((n, 3), f32), projected_gravity=np.tile(np.array([0, 0, -1], f32), (n, 1)))
    S["lambda"] = np.zeros((n, LAMBDA_WIDTH), f32)
    S["default_dof_pos"] = cfg.default[None, :]
    S["episode_sums"] = {name: np.zeros(n, f32) for name in E.REWARD_NAMES}
    reset_envs(cfg, S, np.arange(n), 0)
    S["base_euler_xyz"] = E.euler_xyz(S["root_states"][:, 3:7])
    noise = PhiloxDraws(cfg.seed, n, cfg.offset).obs_noise(0, 47) if c.add_noise else None
    o, p, ref = E.obs_frames(S, cfg.L, cfg.P, noise=noise)
    clip = f32(c.clip_observations)
    S["ref_dof_pos"] = ref
    obs = E.stack(np.zeros((n, c.frame_stack * 47), f32), np.clip(o, -clip, clip))
    priv = E.stack(np.zeros((n, c.c_frame_stack * 73), f32), np.clip(p, -clip, clip))
    return S, obs, priv


LAMBDA_WIDTH = 24 * 3 + 16 * 3 + 2 * 12  # HG_LAMW (include/hgsim.h): solver warm-start slots per env; only their zeroing on reset matters here


def post(cfg, S, counter, hist_obs, hist_priv, draws=None, extras=None):
    """One hg_post (mode 0) = post_physics_step minus the refreshes (humanoid_env.py:780-806)
    plus the obs clip of step() (:654-657).  Mutates S; returns (obs_stack, priv_stack, rew,
    reset, timeout, terms).  ``extras`` (a dict) receives "episode" (reward means of the resetting
    envs, reset_idx :1145-1148) when some env resets."""
    c, P, L = cfg.c, cfg.P, cfg.L
    d = _draws(cfg, draws)
    n = S["root_states"].shape[0]
    S["episode_length_buf"] = S["episode_length_buf"] + 1
    q = S["root_states"][:, 3:7]
    S["base_lin_vel"] = E.quat_rotate_inverse(q, S["root_states"][:, 7:10])
    S["base_ang_vel"] = E.quat_rotate_inverse(q, S["root_states"][:, 10:13])
    S["projected_gravity"] = E.quat_rotate_inverse(q, np.tile(np.array([0, 0, -1], f32), (n, 1)))
    S["base_euler_xyz"] = E.euler_xyz(q)
    # _post_physics_step_callback (:1000-1016)
    ids = np.nonzero(S["episode_length_buf"] % c.resample_interval == 0)[0]
    _resample(cfg, S, ids, counter, 0, d)
    if c.heading_command:
        fwd = E.quat_apply(q, np.tile(np.array([1, 0, 0], f32), (n, 1)))
        heading = np.arctan2(fwd[:, 1], fwd[:, 0]).astype(f32)
        S["commands"][:, 2] = np.clip(f32(0.5) * E.wrap_to_pi(S["commands"][:, 3] - heading), -1.0, 1.0)
    if c.push_robots and counter % c.push_interval == 0:
        push_robots(cfg, S, counter, d)
    reset, timeout = E.termination(S["contact_forces"], S["episode_length_buf"], L, P)
    S["default_dof_pos"] = cfg.default[None, :]
    terms = E.rewards(S, L, P)
    rew = E.total_reward(terms, cfg.scales, S["episode_sums"], P)
    means = reset_envs(cfg, S, np.nonzero(reset)[0], counter, d)
    if extras is not None and means is not None:
        extras["episode"] = means
    S["base_euler_xyz"] = E.euler_xyz(S["root_states"][:, 3:7])
    width = 5 + 3 * S["dof_pos"].shape[1] + 6
    noise = d.obs_noise(counter, width) if c.add_noise else None
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


def step_without_physics(cfg, S, actions, counter, hist_obs, hist_priv, gains, draws=None, extras=None):
    """The reference's step() (humanoid_env.py:616-660) with gym.simulate a no-op: prologue,
    decimation x _compute_torques on the unchanged state, post, obs clip.  ``counter`` is the
    common_step_counter AFTER post_physics_step's increment (:781).  gains = (p_gains, d_gains,
    torque_limits, action_scale).  Used to pin the composition against the reference itself."""
    S["actions"] = preprocess_actions(cfg, actions, S["actions"], counter, draws)
    p, dg, tl, scale = gains
    S["torques"] = E.compute_torques(S["actions"], p, dg, S["default_dof_pos"], S["dof_pos"], S["dof_vel"], tl, scale)
    return post(cfg, S, counter, hist_obs, hist_priv, draws, extras)
