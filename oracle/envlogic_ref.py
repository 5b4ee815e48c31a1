"""CPU restatement (numpy) of the reference env arithmetic — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Each function
cites the reference lines it restates (humanoid/envs/custom/humanoid_env.py).  It is written for
any DOF layout: ``Layout`` carries the index maps, so the same code runs at the fork's native
18-DOF layout (pinned against tests/golden/env18.npz, generated from the reference itself) and
at the 12-DOF XBot-L profile the HIP kernels implement (SURVEY App. A index maps).

Arithmetic is float32 in the reference's operation order where it matters.
"""
from dataclasses import dataclass, field

import numpy as np

f32 = np.float32
PI_F = f32(np.pi)
TWO_PI_F = f32(2 * np.pi)

REWARD_NAMES = [
    "action_smoothness", "base_acc", "base_height", "collision", "default_joint_pos", "dof_acc", "dof_vel",
    "feet_air_time", "feet_clearance", "feet_contact_forces", "feet_contact_number", "feet_distance",
    "foot_slip", "joint_pos", "knee_distance", "low_speed", "orientation", "torques", "track_vel_hard",
    "tracking_ang_vel", "tracking_lin_vel", "vel_mismatch_exp",
]


@dataclass
class Layout:
    D: int
    ref_idx: tuple          # (l_pitch, l_knee, l_ankle, r_pitch, r_knee, r_ankle)
    yaw_roll: tuple         # (l0, l1, r0, r1)
    feet: tuple = (6, 12)
    knees: tuple = (4, 10)
    base: int = 0


LAYOUT18 = Layout(D=18, ref_idx=(8, 9, 10, 14, 15, 16), yaw_roll=(6, 7, 12, 13))   # humanoid_env.py:731-739,1265-1266
LAYOUT12 = Layout(D=12, ref_idx=(2, 3, 4, 8, 9, 10), yaw_roll=(0, 1, 6, 7))


@dataclass
class Params:
    dt: float = 0.01
    cycle_time: float = 0.64
    target_joint_pos_scale: float = 0.17
    target_feet_height: float = 0.1
    base_height_target: float = 0.94
    min_dist: float = 0.2
    max_dist: float = 0.5
    tracking_sigma: float = 5.0
    max_contact_force: float = 700.0
    max_episode_length: int = 2400
    only_positive_rewards: bool = True
    obs_scales: dict = field(default_factory=lambda: dict(lin_vel=2.0, ang_vel=1.0, dof_pos=1.0, dof_vel=0.05, quat=1.0))
    noise_scales: dict = field(default_factory=lambda: dict(dof_pos=0.05, dof_vel=0.5, ang_vel=0.1, quat=0.03))
    noise_level: float = 0.6
    clip_obs: float = 18.0


# ------------------------------------------------------------------------------------------ math
def quat_rotate_inverse(q, v):
    q = q.astype(f32)
    v = v.astype(f32)
    qw = q[:, 3:4]
    qv = q[:, :3]
    a = v * (f32(2.0) * qw ** 2 - f32(1.0))
    b = np.cross(qv, v) * qw * f32(2.0)
    c = qv * np.sum(qv * v, axis=1, keepdims=True) * f32(2.0)
    return (a - b + c).astype(f32)


def quat_apply(q, v):
    xyz = q[:, :3]
    t = np.cross(xyz, v) * f32(2)
    return (v + q[:, 3:] * t + np.cross(xyz, t)).astype(f32)


def _pymod(a, b):
    return (a - b * np.floor(a / b)).astype(f32)


def euler_xyz(q):
    """isaacgym get_euler_xyz + get_euler_xyz_tensor wrap (humanoid_env.py:51-56)."""
    x, y, z, w = [q[:, i].astype(f32) for i in range(4)]
    roll = np.arctan2(f32(2.0) * (w * x + y * z), w * w - x * x - y * y + z * z)
    sinp = f32(2.0) * (w * y - z * x)
    pitch = np.where(np.abs(sinp) >= 1, np.copysign(f32(np.pi / 2), sinp), np.arcsin(np.clip(sinp, -1, 1)))
    yaw = np.arctan2(f32(2.0) * (w * z + x * y), w * w + x * x - y * y - z * z)
    e = np.stack([_pymod(roll.astype(f32), TWO_PI_F), _pymod(pitch.astype(f32), TWO_PI_F),
                  _pymod(yaw.astype(f32), TWO_PI_F)], axis=1)
    e = np.where(e > PI_F, e - TWO_PI_F, e)
    return e.astype(f32)


def wrap_to_pi(a):
    a = _pymod(a, TWO_PI_F)
    return np.where(a > PI_F, a - TWO_PI_F, a).astype(f32)


# ------------------------------------------------------------------------------------------ pieces
def compute_torques(actions, p_gains, d_gains, default_dof_pos, dof_pos, dof_vel, torque_limits, action_scale):
    """_compute_torques (humanoid_env.py:910-925)."""
    a = actions.astype(f32) * f32(action_scale)
    t = p_gains * (a + default_dof_pos - dof_pos) - d_gains * dof_vel
    return np.clip(t, -torque_limits, torque_limits).astype(f32)


def phase(ep_len, P):
    """_get_phase (humanoid_env.py:683-686)."""
    return (ep_len.astype(f32) * f32(P.dt) / f32(P.cycle_time)).astype(f32)


def gait(ep_len, P):
    """_get_gait_phase (humanoid_env.py:688-703) -> (sin, cos, stance[N,2])."""
    ph = phase(ep_len, P)
    s = np.sin(f32(2 * np.pi) * ph).astype(f32)
    c = np.cos(f32(2 * np.pi) * ph).astype(f32)
    st = np.zeros((len(ep_len), 2), f32)
    st[:, 0] = s >= 0
    st[:, 1] = s < 0
    st[np.abs(s) < 0.1] = 1
    return s, c, st


def ref_state(ep_len, L: Layout, P):
    """compute_ref_state (humanoid_env.py:705-744)."""
    s, _, _ = gait(ep_len, P)
    ref = np.zeros((len(ep_len), L.D), f32)
    s1 = f32(P.target_joint_pos_scale)
    s2 = f32(2 * P.target_joint_pos_scale)
    sl = np.minimum(s, 0)
    sr = np.maximum(s, 0)
    i = L.ref_idx
    ref[:, i[0]] = sl * s1
    ref[:, i[1]] = sl * s2
    ref[:, i[2]] = sl * s1
    ref[:, i[3]] = sr * s1
    ref[:, i[4]] = sr * s2
    ref[:, i[5]] = sr * s1
    ref[np.abs(s) < 0.1] = 0
    return ref


def noise_vec(L: Layout, P):
    """_get_noise_scale_vec (humanoid_env.py:748-768), restated literally with the fork's shift
    k = D - 12 (the fork writes `17+6`, `29+6*2`, `41+6*2`, ...).  At the 18-DOF fork layout this
    reproduces a reference defect — the ang-vel / euler noise lands on action slots 53:59 and the
    real ang-vel / euler slots 59:65 get none (pinned by tests/golden/env18.npz); at the 12-DOF
    profile (k = 0) the same formula is the aligned upstream layout."""
    k = L.D - 12
    n = np.zeros(5 + 3 * L.D + 6, f32)
    n[5:17 + k] = P.noise_scales["dof_pos"] * P.obs_scales["dof_pos"]
    n[17 + k:29 + 2 * k] = P.noise_scales["dof_vel"] * P.obs_scales["dof_vel"]
    n[29 + 2 * k:41 + 2 * k] = 0.0
    n[41 + 2 * k:44 + 2 * k] = P.noise_scales["ang_vel"] * P.obs_scales["ang_vel"]
    n[44 + 2 * k:47 + 2 * k] = P.noise_scales["quat"] * P.obs_scales["quat"]
    return n


def termination(contact_forces, ep_len, L: Layout, P):
    """check_termination (humanoid_env.py:811-816)."""
    reset = np.linalg.norm(contact_forces[:, L.base, :], axis=-1) > 1.0
    timeout = ep_len > P.max_episode_length
    return reset | timeout, timeout


def rewards(S, L: Layout, P):
    """The 22 _reward_* terms (humanoid_env.py:1170-1437).  S: dict of state arrays; mutates
    S['feet_air_time'], S['last_contacts'], S['feet_height'], S['last_feet_z'] like the reference.
    Returns dict name -> term (unscaled)."""
    T = {}
    q, qd, a = S["dof_pos"], S["dof_vel"], S["actions"]
    la, lla = S["last_actions"], S["last_last_actions"]
    cf, rs, root = S["contact_forces"], S["rigid_state"], S["root_states"]
    blv, bav, pg, eul, cmd = S["base_lin_vel"], S["base_ang_vel"], S["projected_gravity"], S["base_euler_xyz"], S["commands"]
    fe, kn = list(L.feet), list(L.knees)
    _, _, stance = gait(S["episode_length_buf"], P)
    contact = cf[:, fe, 2] > 5.0
    T["action_smoothness"] = (np.sum(np.square(la - a), 1) + np.sum(np.square(a + lla - 2 * la), 1)
                              + f32(0.05) * np.sum(np.abs(a), 1))
    T["base_acc"] = np.exp(-np.linalg.norm(S["last_root_vel"] - root[:, 7:13], axis=1) * 3)
    mh = np.sum(rs[:, fe, 2] * stance, 1) / np.sum(stance, 1)
    T["base_height"] = np.exp(-np.abs(root[:, 2] - (mh - f32(0.05)) - f32(P.base_height_target)) * 100)
    T["collision"] = np.sum(1.0 * (np.linalg.norm(cf[:, [L.base], :], axis=-1) > 0.1), 1)
    jd = q - S["default_dof_pos"]
    y = L.yaw_roll
    yr = np.linalg.norm(jd[:, [y[0], y[1]]], axis=1) + np.linalg.norm(jd[:, [y[2], y[3]]], axis=1)
    yr = np.clip(yr - f32(0.1), 0, 50)
    T["default_joint_pos"] = np.exp(-yr * 100) - f32(0.01) * np.linalg.norm(jd, axis=1)
    T["dof_acc"] = np.sum(np.square((S["last_dof_vel"] - qd) / f32(P.dt)), 1)
    T["dof_vel"] = np.sum(np.square(qd), 1)
    # feet_air_time (mutates)
    filt = contact | (stance != 0) | S["last_contacts"]
    S["last_contacts"] = contact.copy()
    first = (S["feet_air_time"] > 0) * filt
    S["feet_air_time"] = S["feet_air_time"] + f32(P.dt)
    T["feet_air_time"] = np.sum(np.clip(S["feet_air_time"], 0, 0.5) * first, 1)
    S["feet_air_time"] = S["feet_air_time"] * ~filt
    # feet_clearance (mutates)
    fz = rs[:, fe, 2] - f32(0.05)
    S["feet_height"] = S["feet_height"] + (fz - S["last_feet_z"])
    S["last_feet_z"] = fz
    swing = 1 - stance
    rp = np.abs(S["feet_height"] - f32(P.target_feet_height)) < 0.01
    T["feet_clearance"] = np.sum(rp * swing, 1)
    S["feet_height"] = S["feet_height"] * ~contact
    T["feet_contact_forces"] = np.sum(np.clip(np.linalg.norm(cf[:, fe, :], axis=-1) - f32(P.max_contact_force), 0, 400), 1)
    T["feet_contact_number"] = np.mean(np.where(contact == stance, f32(1), f32(-0.3)), 1)

    def dist_rew(pos, mx):
        d = np.linalg.norm(pos[:, 0, :] - pos[:, 1, :], axis=1)
        dmin = np.clip(d - f32(P.min_dist), -0.5, 0)
        dmax = np.clip(d - f32(mx), 0, 0.5)
        return (np.exp(-np.abs(dmin) * 100) + np.exp(-np.abs(dmax) * 100)) / 2

    T["feet_distance"] = dist_rew(rs[:, fe, :2], P.max_dist)
    T["foot_slip"] = np.sum(np.sqrt(np.linalg.norm(rs[:, fe, 10:12], axis=2)) * contact, 1)
    diff = q - S["ref_dof_pos"]
    nd = np.linalg.norm(diff, axis=1)
    T["joint_pos"] = np.exp(-2 * nd) - f32(0.2) * np.clip(nd, 0, 0.5)
    T["knee_distance"] = dist_rew(rs[:, kn, :2], P.max_dist / 2)
    sp, cm = np.abs(blv[:, 0]), np.abs(cmd[:, 0])
    low, high = sp < 0.5 * cm, sp > 1.2 * cm
    des = ~(low | high)
    mis = np.sign(blv[:, 0]) != np.sign(cmd[:, 0])
    r = np.zeros(len(sp), f32)
    r[low] = -1.0
    r[high] = 0.0
    r[des] = 1.2
    r[mis] = -2.0
    T["low_speed"] = r * (np.abs(cmd[:, 0]) > 0.1)
    T["orientation"] = (np.exp(-np.sum(np.abs(eul[:, :2]), 1) * 10) + np.exp(-np.linalg.norm(pg[:, :2], axis=1) * 20)) / 2
    T["torques"] = np.sum(np.square(S["torques"]), 1)
    le = np.linalg.norm(cmd[:, :2] - blv[:, :2], axis=1)
    ae = np.abs(cmd[:, 2] - bav[:, 2])
    T["track_vel_hard"] = (np.exp(-le * 10) + np.exp(-ae * 10)) / 2 - f32(0.2) * (le + ae)
    T["tracking_ang_vel"] = np.exp(-np.square(cmd[:, 2] - bav[:, 2]) * f32(P.tracking_sigma))
    T["tracking_lin_vel"] = np.exp(-np.sum(np.square(cmd[:, :2] - blv[:, :2]), 1) * f32(P.tracking_sigma))
    T["vel_mismatch_exp"] = (np.exp(-np.square(blv[:, 2]) * 10) + np.exp(-np.linalg.norm(bav[:, :2], axis=1) * 5.0)) / 2
    return {k: np.asarray(v, dtype=f32) for k, v in T.items()}


def total_reward(terms, scales, sums, P):
    """compute_reward (humanoid_env.py:889-907): alphabetical sum, episode sums, clip >= 0."""
    rew = np.zeros_like(next(iter(terms.values())))
    for name in sorted(scales):
        r = (terms[name] * f32(scales[name])).astype(f32)
        rew = rew + r
        sums[name] = sums[name] + r
    if P.only_positive_rewards:
        rew = np.maximum(rew, 0)
    return rew.astype(f32)


def obs_frames(S, L: Layout, P, noise=None):
    """compute_observations frames (humanoid_env.py:818-869) -> (obs_frame [N,5+3D+6], priv_frame
    [N,5+4D+20]); noise: standard normals [N, obs width] or None (add_noise False)."""
    os_ = P.obs_scales
    s, c, stance = gait(S["episode_length_buf"], P)
    ref = ref_state(S["episode_length_buf"], L, P)
    contact = (S["contact_forces"][:, list(L.feet), 2] > 5.0).astype(f32)
    cmd = S["commands"][:, :3] * np.array([os_["lin_vel"], os_["lin_vel"], os_["ang_vel"]], f32)
    ci = np.concatenate([s[:, None], c[:, None], cmd], 1)
    q = (S["dof_pos"] - S["default_dof_pos"]) * f32(os_["dof_pos"])
    dq = S["dof_vel"] * f32(os_["dof_vel"])
    priv = np.concatenate([ci, q, dq, S["actions"], S["dof_pos"] - ref, S["base_lin_vel"] * f32(os_["lin_vel"]),
                           S["base_ang_vel"] * f32(os_["ang_vel"]), S["base_euler_xyz"] * f32(os_["quat"]),
                           S["rand_push_force"][:, :2], S["rand_push_torque"], S["env_frictions"],
                           S["body_mass"] / f32(30.0), stance, contact], 1).astype(f32)
    obs = np.concatenate([ci, q, dq, S["actions"], S["base_ang_vel"] * f32(os_["ang_vel"]),
                          S["base_euler_xyz"] * f32(os_["quat"])], 1).astype(f32)
    if noise is not None:
        obs = obs + noise * noise_vec(L, P) * f32(P.noise_level)
    return obs.astype(f32), priv.astype(f32), ref


def stack(history, frame, reset=None):
    """deque append + stack (humanoid_env.py:871-887) on a [N, F*W] history; reset envs'
    history zeroed first (reset_idx :1160-1163)."""
    W = frame.shape[1]
    h = history.copy()
    if reset is not None:
        h[reset] = 0
    return np.concatenate([h[:, W:], frame], 1)


# ------------------------------------------------------------------------------------------ GAE
def gae(rewards, dones, values, last_values, gamma, lam, normalize=True):
    """RolloutStorage.compute_returns (rollout_storage.py:122-143), float32 in the reference's
    op order.  rewards/dones/values [T,N], last_values [N] -> (returns, normalised advantages);
    normalize=False returns the raw advantages (returns - values)."""
    T = rewards.shape[0]
    g, l = f32(gamma), f32(lam)
    adv = np.zeros(rewards.shape[1], f32)
    ret = np.zeros_like(rewards, dtype=f32)
    for t in reversed(range(T)):
        nv = last_values.astype(f32) if t == T - 1 else values[t + 1]
        nnt = f32(1.0) - dones[t].astype(f32)
        delta = rewards[t] + (nnt * g) * nv - values[t]
        adv = delta + ((nnt * g) * l) * adv
        ret[t] = adv + values[t]
    a = (ret - values).astype(f32)
    if not normalize:
        return ret, a
    a64 = a.astype(np.float64)
    mean = a64.mean()
    std = a64.std(ddof=1)
    return ret, ((a - f32(mean)) / (f32(std) + f32(1e-8))).astype(f32)
