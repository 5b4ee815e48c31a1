"""Independent forward kinematics of the reference's MuJoCo description of XBot-L.

TEST INFRASTRUCTURE ONLY: imported by tests/ (tests/test_fk_mjcf.py, the GPU FK pin in
tests/test_gpu_parity.py); never by the product package.

The reference ships two descriptions of the same robot: the URDF Isaac Gym loads (compiled by
tools/urdf_compile.py into model/xbotl_model.json, which the HIP kernels and physics_ref.c read) and
a MuJoCo model written separately, resources/robots/XBot/mjcf/XBot-L.xml (legs at :394-481; its
body tree is kept as plain data in tests/golden/mjcf_xbotl.json).  This module walks the MJCF tree
by MuJoCo's conventions, with none of the compiled model's code or data:
  * a body's frame is its parent's frame times (pos, quat) (quat as w, x, y, z);
  * a hinge joint (every leg joint sits at its body's origin, pos="0 0 0") then rotates the body by
    +q about its axis, given in the body frame (right-hand rule);
  * the free joint puts base_link's frame at the root pose (position, quaternion x, y, z, w as in
    Isaac Gym's root state, humanoid_env.py:235-254).
Velocities by the same tree: w_b = w_parent + (R_b axis) qd, v_b = v_parent + w_parent x (o_b -
o_parent) (the joint sits at the child's origin, so it does not move that origin).

So a simulator whose rigid_state agrees with this module at arbitrary q rotates each joint by +q
about the axis the reference's robot description gives — the only simulator-level kinematic pin
the reference holds.  The MJCF prints its quaternions to 6 digits, so the agreement is to ~1e-5.
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MJCF_JSON = os.path.join(os.path.dirname(HERE), "tests", "golden", "mjcf_xbotl.json")

# the build's 13 bodies (DOF order): body j + 1 carries joint j
BODIES = ["base_link",
          "left_leg_roll_link", "left_leg_yaw_link", "left_leg_pitch_link", "left_knee_link",
          "left_ankle_pitch_link", "left_ankle_roll_link",
          "right_leg_roll_link", "right_leg_yaw_link", "right_leg_pitch_link", "right_knee_link",
          "right_ankle_pitch_link", "right_ankle_roll_link"]


def _qmat_wxyz(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _axis_angle(axis, th):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def collapse(bodies):
    """MJCF tree -> {jointed body: dict(mass, com (body frame), I (3x3 about the COM, body frame),
    T (4x4 in the parent jointed body's frame), parent, joint)}, merging every joint-less MJCF body
    into its nearest jointed ancestor (Isaac Gym's collapse_fixed_joints, humanoid_config.py:93)."""
    by = {b["name"]: b for b in bodies}
    T_world = {}
    for b in bodies:  # bodies are listed parents first
        T = np.eye(4)
        T[:3, :3] = _qmat_wxyz(b["quat"])
        T[:3, 3] = b["pos"]
        T_world[b["name"]] = T if b["parent"] is None else T_world[b["parent"]] @ T

    def owner(name):
        while not by[name]["joints"]:
            name = by[name]["parent"]
        return name
    out = {}
    for b in bodies:
        if b["joints"]:
            par = owner(b["parent"]) if b["parent"] else None
            Tp = np.linalg.inv(T_world[par]) @ T_world[b["name"]] if par else np.eye(4)
            out[b["name"]] = dict(parent=par, T=Tp, joint=b["joints"][0], items=[])
    for b in bodies:
        inn = b.get("inertial")
        if inn is None:
            continue
        o = owner(b["name"])
        T = np.linalg.inv(T_world[o]) @ T_world[b["name"]]
        R = T[:3, :3] @ _qmat_wxyz(inn["quat"])
        c = T[:3, :3] @ np.asarray(inn["pos"]) + T[:3, 3]
        out[o]["items"].append((inn["mass"], c, R @ np.diag(inn["diaginertia"]) @ R.T))
    for rec in out.values():
        m = sum(i[0] for i in rec["items"])
        com = sum(i[0] * i[1] for i in rec["items"]) / m
        I = np.zeros((3, 3))
        for mi, ci, Ii in rec["items"]:
            d = ci - com
            I += Ii + mi * (d @ d * np.eye(3) - np.outer(d, d))
        rec.update(mass=m, com=com, I=I)
    return out


def load(path=MJCF_JSON):
    with open(path) as f:
        return json.load(f)["bodies"]


def fk(bodies, root, q, qd=None):
    """World states of BODIES for one root state (13: pos, quat xyzw, lin vel, ang vel) and joint
    positions q[12] (velocities qd[12]): dict name -> (o[3], R[3,3], v[3], w[3])."""
    root = np.asarray(root, float)
    q = np.asarray(q, float)
    qd = np.zeros(12) if qd is None else np.asarray(qd, float)
    jidx = {BODIES[j + 1].replace("_link", "_joint"): j for j in range(12)}
    x, y, z, w = root[3:7]
    st = {}
    for b in bodies:  # parents first
        if b["parent"] is None:
            st[b["name"]] = (root[0:3].copy(), _qmat_wxyz([w, x, y, z]), root[7:10].copy(), root[10:13].copy())
            continue
        op, Rp, vp, wp = st[b["parent"]]
        o = op + Rp @ np.asarray(b["pos"], float)
        R = Rp @ _qmat_wxyz(b["quat"])
        v = vp + np.cross(wp, o - op)
        wv = wp.copy()
        for jt in b["joints"]:
            if jt["type"] != "hinge":
                continue
            j = jidx[jt["name"]]
            R = R @ _axis_angle(jt["axis"], q[j])
            wv = wv + (R @ np.asarray(jt["axis"], float)) * qd[j]
        st[b["name"]] = (o, R, v, wv)
    return {n: st[n] for n in BODIES}


def fk_array(bodies, root, q, qd=None):
    """fk() as arrays: positions [13, 3], rotation matrices [13, 3, 3], linear and angular
    velocities [13, 3] in BODIES order."""
    s = fk(bodies, root, q, qd)
    return (np.array([s[n][0] for n in BODIES]), np.array([s[n][1] for n in BODIES]),
            np.array([s[n][2] for n in BODIES]), np.array([s[n][3] for n in BODIES]))


def quat_xyzw_to_mat(qq):
    """[..., 4] (x, y, z, w) -> [..., 3, 3]."""
    qq = np.asarray(qq, float)
    qq = qq / np.linalg.norm(qq, axis=-1, keepdims=True)
    x, y, z, w = qq[..., 0], qq[..., 1], qq[..., 2], qq[..., 3]
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
                     np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
                     np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)
