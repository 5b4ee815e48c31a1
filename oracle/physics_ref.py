"""ctypes wrapper of oracle/libphysref.so (CPU reference physics).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product package.  See physics_ref.c for what it restates.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libphysref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def set_threads(n):
    """OpenMP threads of the C reference's env loop."""
    lib().ref_set_threads(ctypes.c_int(int(n)))


class RefSim:
    """AoS CPU simulator state for n envs (root[n,13], q/qd[n,12], warm-start lambdas)."""

    def __init__(self, cfg, model, n, precision="f64", heightfield=None):
        self.cfg, self.model, self.n = cfg, model, n
        self.dt = np.float64 if precision == "f64" else np.float32
        self.fn = getattr(lib(), "ref_step_" + precision)
        self.lamw = lib().ref_lamw_f64()
        self.root = np.zeros((n, 13), self.dt)
        self.root[:, 6] = 1.0
        self.q = np.zeros((n, 12), self.dt)
        self.qd = np.zeros((n, 12), self.dt)
        self.lam = np.zeros((n, self.lamw), self.dt)
        self.mass0 = np.full(n, model.mass[0], self.dt)
        self.fric = np.full(n, 1.0, self.dt)
        self.torques = np.zeros((n, 12), self.dt)
        self.contact = np.zeros((n, 13, 3), self.dt)
        self.rigid = np.zeros((n, 13, 13), self.dt)
        self.nonfinite = np.zeros(n, np.int32)
        self.dropped = np.zeros(n, np.int32)   # rows / contact points over the budget (cumulative)
        self.hf = None if heightfield is None else np.ascontiguousarray(heightfield, np.int16)

    def step(self, actions):
        a = np.ascontiguousarray(actions, self.dt)
        assert a.shape == (self.n, 12)
        hf = None if self.hf is None else _p(self.hf)
        self.fn(ctypes.byref(self.cfg), ctypes.byref(self.model), hf, ctypes.c_int(self.n), _p(self.root),
                _p(self.q), _p(self.qd), _p(self.lam), _p(a), _p(self.mass0), _p(self.fric), _p(self.torques),
                _p(self.contact), _p(self.rigid), _p(self.nonfinite), _p(self.dropped))


def rigid_states(model, root, q, qd, mass0=None, precision="f64"):
    """[n, 13, 13] body states (position, quaternion xyzw, linear / angular velocity, world frame)
    of n states, by the oracle's own forward kinematics (physics_ref.c rigid_states), no step."""
    dt = np.float64 if precision == "f64" else np.float32
    root = np.ascontiguousarray(np.atleast_2d(root), dt)
    n = root.shape[0]
    q = np.ascontiguousarray(np.broadcast_to(q, (n, 12)), dt)
    qd = np.ascontiguousarray(np.broadcast_to(qd, (n, 12)), dt)
    m0 = np.ascontiguousarray(np.full(n, model.mass[0] if mass0 is None else mass0), dt)
    out = np.zeros((n, 13, 13), dt)
    getattr(lib(), "ref_rigid_states_" + precision)(ctypes.byref(model), ctypes.c_int(n), _p(root), _p(q), _p(qd),
                                                    _p(m0), _p(out))
    return out


def ground(cfg, hf, x, y):
    """(height, unit normal[..., 3]) of the terrain under world points (x, y), numpy float64: the
    plane z = 0, or the int16 heightfield triangulated along the (i, j)-(i+1, j+1) diagonal —
    physics_ref.c:179-196 (`ground`) element for element.  For tests that classify contacts by
    the triangle they sit on."""
    x, y = np.asarray(x, np.float64), np.asarray(y, np.float64)
    if cfg.terrain_type == 0 or hf is None:
        n = np.zeros(x.shape + (3,))
        n[..., 2] = 1.0
        return np.zeros(x.shape), n
    hs, vs = float(cfg.hf_horizontal_scale), float(cfg.hf_vertical_scale)
    rows, cols = int(cfg.hf_rows), int(cfg.hf_cols)
    fx, fy = (x + cfg.hf_border) / hs, (y + cfg.hf_border) / hs
    i = np.clip(np.floor(fx).astype(np.int64), 0, rows - 2)
    j = np.clip(np.floor(fy).astype(np.int64), 0, cols - 2)
    u, v = np.clip(fx - i, 0, 1), np.clip(fy - j, 0, 1)
    H = np.asarray(hf).reshape(rows, cols).astype(np.float64) * vs
    h00, h10, h01, h11 = H[i, j], H[i + 1, j], H[i, j + 1], H[i + 1, j + 1]
    lower = u >= v
    h = np.where(lower, h00 + u * (h10 - h00) + v * (h11 - h10), h00 + v * (h01 - h00) + u * (h11 - h01))
    dx = np.where(lower, (h10 - h00) / hs, (h11 - h01) / hs)
    dy = np.where(lower, (h11 - h10) / hs, (h01 - h00) / hs)
    inv = 1 / np.sqrt(dx * dx + dy * dy + 1)
    return h, np.stack([-dx * inv, -dy * inv, inv], axis=-1)


def quat_rotate(q, v):
    """Rotate v[..., 3] by unit quaternions q[..., 4] (x, y, z, w), numpy."""
    u, w = q[..., :3], q[..., 3:4]
    t = 2 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def ground_candidates(model, rigid):
    """World centres [n, nc, 3] of the model's ground-contact spheres from rigid states
    [n, bodies, 13] (position, quaternion xyzw, ...): x = o_b + R_b cpos_c, the point whose
    (x, y) physics_ref.c:472-477 looks the terrain up under."""
    nc = len(model.contact_body)
    cb = np.array([model.contact_body[c] for c in range(nc)])
    cp = np.array([list(model.contact_pos[c]) for c in range(nc)], np.float64)
    rb = np.asarray(rigid, np.float64)[:, cb]
    return rb[..., 0:3] + quat_rotate(rb[..., 3:7], cp[None])


def dynamics(model, root, q, qd, mass0=None, gz=-9.81):
    """(M[18,18], h[18]) at a state, float64."""
    M = np.zeros((18, 18))
    h = np.zeros(18)
    root = np.ascontiguousarray(root, np.float64)
    q = np.ascontiguousarray(q, np.float64)
    qd = np.ascontiguousarray(qd, np.float64)
    m0 = model.mass[0] if mass0 is None else mass0
    lib().ref_dynamics_f64(ctypes.byref(model), _p(root), _p(q), _p(qd), ctypes.c_double(m0),
                           ctypes.c_double(gz), _p(M), _p(h))
    return M, h
