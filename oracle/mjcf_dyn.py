"""Independent equations of motion of the reference's MuJoCo description of XBot-L (Kane's method).

TEST INFRASTRUCTURE ONLY: imported by tests/test_fk_mjcf.py; never by the product package.

physics_ref.c (and K_step, which the GPU parity tests hold to it) builds the joint-space inertia M
by the composite-rigid-body algorithm and the bias force h by recursive Newton-Euler.  This module
gets the same two quantities another way, from the MJCF body tree (oracle/mjcf_fk.py: the
reference's XBot-L.xml, collapsed to the 13 jointed bodies) and nothing of the compiled model but
the trunk's mass properties (the MJCF leaves the neck / arm-base / hand masses out of its trunk,
tests/test_model_mjcf.py; Isaac Gym loads the URDF's):

  generalized velocity nu = [v (base-origin velocity, world), w (base angular velocity, world),
  qd (12)] — physics_ref.c's coordinates; body b's COM velocity v_c = J_c nu and angular velocity
  w_b = J_w nu, the Jacobian columns read off mjcf_fk.fk with one unit velocity each (fk is linear
  in the velocities);
  M = sum_b m_b J_c^T J_c + J_w^T I_w J_w   (I_w = R I R^T about the COM);
  h = sum_b J_c^T m_b (a_c + g_up) + J_w^T (I_w alpha + w_b x I_w w_b),
with (a_c, alpha) the COM and angular accelerations at nu-dot = 0 (base origin moving at constant
world velocity, base turning at constant world rate, joints at constant rate), by a central
difference of J(t) nu along that motion, and g_up = (0, 0, -gz).  M nu-dot + h = the generalized
applied forces: the equations of motion physics_ref's step integrates.
"""
import numpy as np

import mjcf_fk as MF


def mass_props(bodies, trunk=None):
    """[(mass, com (body frame), I (3x3 about the COM, body frame))] in MF.BODIES order from the
    collapsed MJCF; `trunk` (mass, com, I) replaces base_link's."""
    col = MF.collapse(bodies)
    out = [(col[n]["mass"], np.asarray(col[n]["com"], float), np.asarray(col[n]["I"], float)) for n in MF.BODIES]
    if trunk is not None:
        out[0] = trunk
    return out


def _quat_mul(a, b):  # xyzw
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def _jacobians(bodies, props, root, q):
    """(J_c [13, 3, 18], J_w [13, 3, 18], COM positions [13, 3], I_w [13, 3, 3]) at a pose."""
    base = np.array(root, float)
    base[7:13] = 0.0
    o, R, _, _ = MF.fk_array(bodies, base, q)
    cw = np.array([o[b] + R[b] @ props[b][1] for b in range(13)])
    Iw = np.array([R[b] @ props[b][2] @ R[b].T for b in range(13)])
    Jc = np.zeros((13, 3, 18))
    Jw = np.zeros((13, 3, 18))
    for k in range(18):
        r = base.copy()
        qd = np.zeros(12)
        if k < 6:
            r[7 + k] = 1.0
        else:
            qd[k - 6] = 1.0
        _, _, v, w = MF.fk_array(bodies, r, q, qd)
        for b in range(13):
            Jw[b, :, k] = w[b]
            Jc[b, :, k] = v[b] + np.cross(w[b], cw[b] - o[b])
    return Jc, Jw, cw, Iw


def _advance(root, q, nu, t):
    """The pose after time t of the motion with nu-dot = 0 (constant world velocities)."""
    r = np.array(root, float)
    r[0:3] = r[0:3] + nu[0:3] * t
    w = nu[3:6]
    th = np.linalg.norm(w) * t
    if th != 0.0:
        ax = w / np.linalg.norm(w)
        dq = np.concatenate([ax * np.sin(th / 2), [np.cos(th / 2)]])
        r[3:7] = _quat_mul(dq, r[3:7])
    return r, np.asarray(q, float) + nu[6:] * t


def dynamics(bodies, props, root, q, qd, gz=-9.81, eps=1e-5):
    """(M [18, 18], h [18]) at the state (root [13]: pos, quat xyzw, base-origin velocity, angular
    velocity, all world; q, qd [12]) by Kane's method over the MJCF tree."""
    root = np.asarray(root, float)
    nu = np.concatenate([root[7:10], root[10:13], np.asarray(qd, float)])
    Jc, Jw, _, Iw = _jacobians(bodies, props, root, q)
    M = np.zeros((18, 18))
    for b in range(13):
        m = props[b][0]
        M += m * Jc[b].T @ Jc[b] + Jw[b].T @ Iw[b] @ Jw[b]
    vel = []
    for t in (eps, -eps):
        r, qq = _advance(root, q, nu, t)
        Jc_t, Jw_t, _, _ = _jacobians(bodies, props, r, qq)
        vel.append((Jc_t @ nu, Jw_t @ nu))
    a_c = (vel[0][0] - vel[1][0]) / (2 * eps)
    alpha = (vel[0][1] - vel[1][1]) / (2 * eps)
    wb = Jw @ nu
    g_up = np.array([0.0, 0.0, -gz])
    h = np.zeros(18)
    for b in range(13):
        m = props[b][0]
        h += Jc[b].T @ (m * (a_c[b] + g_up)) + Jw[b].T @ (Iw[b] @ alpha[b] + np.cross(wb[b], Iw[b] @ wb[b]))
    return M, h
