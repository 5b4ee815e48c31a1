"""Closed-loop sim2sim on the CPU reference physics — TEST INFRASTRUCTURE ONLY.

The reference's deployment loop (humanoid/scripts/sim2sim.py:185-280) restated in numpy around
oracle/physics_ref.c: every policy step (decimation = 10 substeps of 1 ms) the policy input is
built from the raw simulator state exactly as sim2sim.py builds it —
  frame = [sin, cos of 2 pi t / cycle_time, cmd_x * 2, cmd_y * 2, cmd_yaw * 1, q - q_default,
           0.05 qd, last action, base angular velocity (base frame), roll / pitch / yaw]
  (sim2sim.py:210-223; obs scales humanoid_config.py normalization.obs_scales), clipped to +-18
  (:225), stacked oldest-first over 15 frames (:227-232) —
the policy output is clipped to +-18 (:234) and becomes the PD target 0.25 a + q_default
(:236) held over the 10 substeps, with the env's PD law and torque clip (the physics oracle's
step, humanoid_env.py:910-925).  The policy is any callable [N, 705] float64 -> [N, 12]; `mlp`
builds the ELU MLP of a weights dict (tests/golden/onnx_actor.npz: the reference's trained
OnnxTest.onnx actor).

A fall is the env's termination criterion (humanoid_env.py:811-816: net contact force on the
base link > 1 N); a fallen env stops counting (its tracking errors are averaged over the steps it
was alive, as scripts/sim2sim.py does on the GPU).

This driver is the CPU leg of the PhysX-side evidence: the GPU leg is
humanoid/scripts/sim2sim.py on hg_sim; tests/test_onnx_closed_loop.py and
tests/test_gpu_parity.py::test_onnx_actor_closed_loop_gpu_vs_oracle compare them.
"""
import math

import numpy as np

import physics_ref as P


def elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))


def mlp(weights, dtype=np.float64):
    """ELU MLP y = W3 elu(W2 elu(W1 elu(W0 x + b0) + b1) + b2) + b3 (ONNX Gemm transB=1 / Elu)."""
    Ws = [(np.asarray(weights[f"W{k}"], dtype), np.asarray(weights[f"b{k}"], dtype)) for k in range(4)]

    def f(x):
        h = np.asarray(x, dtype)
        for i, (W, b) in enumerate(Ws):
            h = h @ W.T + b
            if i < len(Ws) - 1:
                h = elu(h)
        return h
    return f


def quat_rotate_inverse(q, v):
    """v in the frame of the (x, y, z, w) quaternions q (rows)."""
    qv, w = q[:, :3], q[:, 3:4]
    a = v * (2.0 * w * w - 1.0)
    b = np.cross(qv, v) * w * 2.0
    c = qv * np.sum(qv * v, axis=1, keepdims=True) * 2.0
    return a - b + c


def quat_to_euler(q):
    """sim2sim.py:57-77 quaternion_to_euler_array for (x, y, z, w) rows, then :212's wrap."""
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    roll = np.arctan2(2.0 * (w * x + y * z), 1.0 - 2.0 * (x * x + y * y))
    pitch = np.arcsin(np.clip(2.0 * (w * y - z * x), -1.0, 1.0))
    yaw = np.arctan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z))
    e = np.stack([roll, pitch, yaw], axis=1)
    return np.where(e > math.pi, e - 2.0 * math.pi, e)


class Sim2SimRef:
    """n envs of the reference simulator driven by a policy in the sim2sim loop.

    hc: HgCfg of the sim2sim configuration (humanoid.scripts.sim2sim.make_cfg + build_hg_cfg, with
    the profile's torque limits); model: HgModel; root [n,13], q / qd [n,12]: the initial state;
    mass0 / fric [n]: base mass and friction after the profile's changes; cmds [n,3]: per-env
    (vx, vy, wz) commands."""

    def __init__(self, hc, model, policy, root, q, qd, mass0, fric, cmds, precision="f64", cycle_time=0.64,
                 obs_scales=(2.0, 1.0, 1.0, 0.05), clip_obs=18.0, clip_actions=18.0, frame_stack=15,
                 default_dof_pos=None, lam=None, cause_slots=None, joint_perm=None, joint_sign=None,
                 omega_frame="base", euler="sim2sim", phase="sincos"):
        """Convention switches (scripts/onnx_sweep.py; defaults = the reference script's loop):
        joint_perm / joint_sign: the policy's joint i is the simulator's joint joint_perm[i] times
        joint_sign[i], for the observed q - q_default, qd, the last action and the action applied
        (obs and action together); omega_frame "base" (sim2sim.py's IMU gyro) | "world" | "neg";
        euler "sim2sim" (sim2sim.py:57-77 + its wrap) | "0_2pi" (isaacgym get_euler_xyz's range) |
        "neg"; phase "sincos" | "neg" (half a cycle shifted) | "swap" (cos, sin)."""
        n = root.shape[0]
        self.n, self.hc, self.policy = n, hc, policy
        self.sim = P.RefSim(hc, model, n, precision)
        self.sim.root[:], self.sim.q[:], self.sim.qd[:] = root, q, qd
        if lam is not None:
            self.sim.lam[:] = lam
        self.sim.mass0[:], self.sim.fric[:] = mass0, fric
        self.cmds = np.asarray(cmds, np.float64)
        self.cycle_time, self.dt = cycle_time, float(hc.dt)
        self.lin_s, self.ang_s, self.pos_s, self.vel_s = obs_scales
        self.clip_obs, self.clip_act, self.stack = clip_obs, clip_actions, frame_stack
        self.default = np.zeros(12) if default_dof_pos is None else np.asarray(default_dof_pos, np.float64)
        self.hist = np.zeros((n, 47 * frame_stack))
        self.action = np.zeros((n, 12))
        self.alive = np.ones(n, bool)
        self.fall_step = np.full(n, -1, np.int64)
        self.err_v = np.zeros(n)
        self.err_w = np.zeros(n)
        self.alive_steps = np.zeros(n)
        self.k = 0
        # fall cause (which contacts put force on the base at the terminating step):
        # {name: warm-start impulse slots}, e.g. base-box corners vs ground, hand / box pairs
        self.cause_slots = cause_slots or {}
        self.fall_cause = np.full(n, "", dtype=object)
        self.perm = np.arange(12) if joint_perm is None else np.asarray(joint_perm, np.int64)
        self.sign = np.ones(12) if joint_sign is None else np.asarray(joint_sign, np.float64)
        self.omega_frame, self.euler, self.phase = omega_frame, euler, phase
        self.travel = np.zeros(n)                      # base displacement along the command (m)
        self.x0 = self.sim.root[:, 0:2].astype(np.float64).copy()

    def frame(self):
        s = self.sim
        quat = s.root[:, 3:7].astype(np.float64)
        w_world = s.root[:, 10:13].astype(np.float64)
        omega = {"base": lambda: quat_rotate_inverse(quat, w_world), "world": lambda: w_world,
                 "neg": lambda: -quat_rotate_inverse(quat, w_world)}[self.omega_frame]()
        ph = 2.0 * math.pi * self.k * self.dt / self.cycle_time
        sn, cs = {"sincos": (math.sin(ph), math.cos(ph)), "neg": (-math.sin(ph), -math.cos(ph)),
                  "swap": (math.cos(ph), math.sin(ph))}[self.phase]
        f = np.empty((self.n, 47))
        f[:, 0], f[:, 1] = sn, cs
        f[:, 2] = self.cmds[:, 0] * self.lin_s
        f[:, 3] = self.cmds[:, 1] * self.lin_s
        f[:, 4] = self.cmds[:, 2] * self.ang_s
        f[:, 5:17] = (s.q - self.default)[:, self.perm] * self.sign * self.pos_s
        f[:, 17:29] = s.qd[:, self.perm] * self.sign * self.vel_s
        f[:, 29:41] = self.action
        f[:, 41:44] = omega
        e = quat_to_euler(quat)
        f[:, 44:47] = {"sim2sim": e, "0_2pi": np.mod(e, 2.0 * math.pi), "neg": -e}[self.euler]
        return np.clip(f, -self.clip_obs, self.clip_obs)

    def step(self):
        self.hist = np.concatenate([self.hist[:, 47:], self.frame()], axis=1)
        self.action = np.clip(self.policy(self.hist), -self.clip_act, self.clip_act)
        applied = np.empty_like(self.action)
        applied[:, self.perm] = self.action * self.sign
        self.sim.step(applied)
        self.k += 1
        s = self.sim
        fell = (np.linalg.norm(s.contact[:, 0, :], axis=1) > 1.0) | (s.nonfinite != 0)
        new = fell & self.alive
        self.fall_step[new] = self.k
        for e in np.nonzero(new)[0]:
            self.fall_cause[e] = "+".join(name for name, slots in self.cause_slots.items()
                                          if (s.lam[e, slots] > 0).any()) or "other"
        self.alive &= ~fell
        quat = s.root[:, 3:7].astype(np.float64)
        vb = quat_rotate_inverse(quat, s.root[:, 7:10].astype(np.float64))
        wb = quat_rotate_inverse(quat, s.root[:, 10:13].astype(np.float64))
        live = self.alive.astype(np.float64)
        self.err_v += live * np.linalg.norm(vb[:, :2] - self.cmds[:, :2], axis=1)
        self.err_w += live * np.abs(wb[:, 2] - self.cmds[:, 2])
        self.alive_steps += live
        # displacement along the commanded direction, frozen at the fall
        d = s.root[:, 0:2].astype(np.float64) - self.x0
        c = self.cmds[:, :2]
        cn = np.linalg.norm(c, axis=1)
        along = np.where(cn > 0, (d * c).sum(1) / np.maximum(cn, 1e-12), 0.0)
        self.travel = np.where(self.alive, along, self.travel)

    def run(self, steps):
        for _ in range(steps):
            self.step()
        return self.summary()

    def summary(self):
        a = np.maximum(self.alive_steps, 1.0)
        return dict(fell=(self.fall_step >= 0), fall_step=self.fall_step.copy(), lin_vel_error=self.err_v / a,
                    yaw_rate_error=self.err_w / a, survival_s=self.alive_steps * self.dt,
                    fall_cause=list(self.fall_cause), travel_m=self.travel.copy())
