"""CPU analysis of the GPU contact-step dumps (scripts/contact_dump.py) against the oracle.

For each dump: the f64 step, the test's yardstick (3-member f32 ensemble + conditioning spread),
the GPU's envs outside K x yardstick, the null rate of independent f32 members, and for every
GPU outlier env whether its last-substep active set differs from the f64 step's (ground / pair
contacts with a positive normal impulse, joint limits, joint-friction rows at their bound).

  python scripts/contact_analysis.py gpurun_out/contact_dump_plane.npz [...]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import step_tolerance as ST  # noqa: E402


def active_sets(lam, nc, npair, nd, fric_bound):
    """Per env: (ground normals > 0, pair normals > 0, limits != 0, friction rows at the bound)."""
    g = lam[:, 0:3 * nc:3] > 0
    p = lam[:, 3 * nc:3 * (nc + npair):3] > 0
    lo = 3 * (nc + npair)
    lim = lam[:, lo:lo + nd] != 0
    fr = lam[:, lo + nd:lo + 2 * nd]
    at = np.abs(np.abs(fr) - fric_bound[None]) <= 1e-6 * np.maximum(fric_bound[None], 1e-12)
    at &= fric_bound[None] > 0
    return g, p, lim, at


def analyse(path, K=12.0, candidates=6):
    from humanoid import _native as N
    D = dict(np.load(path))
    hc = N.HgCfg.from_buffer_copy(D["hgcfg"].tobytes())
    model = N.HgModel.from_buffer_copy(D["model"].tobytes())
    hf = D.get("hf")
    S = {"root_states": D["root_states"], "dof_pos": D["dof_pos"], "dof_vel": D["dof_vel"], "lambda": D["lam"],
         "body_mass": D["body_mass"].reshape(len(D["dof_pos"]), -1),
         "env_frictions": D["env_frictions"].reshape(len(D["dof_pos"]), -1)}
    a_ref = D["a_ref"]
    assert np.allclose(D["gpu_actions"], a_ref, rtol=1e-5, atol=1e-6)
    fields = ST.FIELDS
    r64 = ST.ref_sim(hc, model, S, "f64", hf)
    r64.step(a_ref)
    ens = ST.f32_members(hc, model, S, a_ref, fields, hf, members=3)
    g32 = ST.gap(ens, r64, fields)
    spread = ST.f64_spread(hc, model, S, a_ref, r64, fields, hf)
    kp = np.array([hc.kp[j] for j in range(12)])
    kd = np.array([hc.kd[j] for j in range(12)])
    gpu = {"q": D["gpu_q"], "qd": D["gpu_qd"], "root": D["gpu_root"], "torques": D["gpu_torques"],
           "rigid": D["gpu_rigid"]}
    bad, head, tol = ST.compare(gpu, r64, g32, spread, fields, kp, kd, K)
    be = ST.bad_envs(bad)
    null = ST.flip_null_rate(hc, model, S, a_ref, r64, spread, fields, kp, kd, K, hf=hf, candidates=candidates)
    nc, npair, nd = N.HG_MAX_CONTACTS, N.HG_MAX_PAIRS, N.HG_MAX_DOF
    fb = np.array([model.joint_friction[b + 1] * hc.sim_dt for b in range(nd)])
    A_g = active_sets(D["gpu_lam"], nc, npair, nd, fb)
    A_r = active_sets(r64.lam, nc, npair, nd, fb)
    differ = np.zeros(len(be), bool)
    kinds = {}
    for name, a, b in zip(("ground", "pair", "limit", "friction_at_bound"), A_g, A_r):
        d = (a != b).any(axis=1)
        kinds[name] = int((d & be).sum())
        differ |= d
    base = ST.outputs(r64)
    err = {f: float(np.abs(gpu[f] - base[f]).max()) for f in fields}
    err_ok = {f: float(np.abs(gpu[f][~be] - base[f][~be]).max()) if (~be).any() else 0.0 for f in fields}
    err_bad = {f: float(np.abs(gpu[f][be] - base[f][be]).max()) if be.any() else 0.0 for f in fields}
    res = {"dump": os.path.basename(path), "envs": int(len(be)), "K": K,
           "ground_contact_gpu": float(A_g[0].any(axis=1).mean()), "ground_contact_f64": float(A_r[0].any(axis=1).mean()),
           "gpu_bad_envs": int(be.sum()), "gpu_bad_envs_with_active_set_change": int((be & differ).sum()),
           "active_set_change_kinds_in_bad_envs": kinds,
           "envs_with_active_set_change_total": int(differ.sum()),
           "null_bad_envs": null["bad_envs"], "null_max_err": null["max_err"],
           "null_dropped_mismatch_envs": null["dropped_mismatch_envs"],
           "gpu_max_err": err, "gpu_max_err_outside_bad_envs": err_ok,
           "gpu_max_err_in_bad_envs": err_bad, "headroom": head,
           "dropped_mismatch_envs": int((D["gpu_dropped"] != r64.dropped).sum()),
           "bad_env_ids": [int(i) for i in np.flatnonzero(be)[:40]]}
    return res


def main():
    out = []
    for p in sys.argv[1:]:
        r = analyse(p)
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
