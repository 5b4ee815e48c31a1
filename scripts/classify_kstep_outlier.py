"""Classify the K_step outlier envs of one dumped GPU step.

Input: the dump smoke() writes with HG_SMOKE_DUMP (__graft_entry__.py): the pre-step state, the
preprocessed actions, the GPU outputs and the GPU's final warm-start impulses.  On the CPU:

  1. the smoke env's hg_cfg / model are rebuilt (build_hg_cfg) and the shared verdict
     (step_tolerance.check_step) is recomputed from the dump — the same outlier ids and achieved
     multiples as the GPU run printed confirm the rebuild;
  2. for each outlier env, the step is replayed substep by substep (decimation 1, ten times: the
     same arithmetic as one 10-substep call) in f64, in MEMBERS plain-f32 builds and in MEMBERS
     "f32q" builds (physics_ref.c REF_APPROX_QUOT: the kernel's reciprocal / rsqrt quotient forms),
     each f32 build on the state perturbed by ~1 ulp (2^-22 relative, as the tolerance ensemble);
  3. each substep's DISCRETE signature is read off its impulses: the active contact rows (normal
     impulse > 0), the friction cones at their bound (|lambda_t| = mu lambda_n), the joint-friction
     rows at their bound f dt (slip) and the active joint-limit rows;
  4. a build whose signature leaves the f64 one at some substep and whose outputs fall outside the
     check's element tolerance (as the GPU's did) reproduces the outlier by a discrete event; the
     kind of the first differing row names the event; builds outside WITHOUT an event would point
     at continuous error growth (e.g. the quotients) instead.  The GPU's own final impulses are compared with the f64 ones
     the same way.

  python scripts/classify_kstep_outlier.py gpurun_out/r6_smoke/dump.npz [--members 64] [--out dir]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import physics_ref as P  # noqa: E402
import step_tolerance as ST  # noqa: E402

NC, NPAIR, ND = 24, 16, 12
LAM_PAIR, LAM_LIM = NC * 3, NC * 3 + NPAIR * 3
LAM_FRIC = LAM_LIM + ND


def smoke_cfg(n):
    from humanoid import _native as N
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import build_hg_cfg
    cfg = XBotLCfg()
    cfg.env.num_envs = n
    model, js = N.load_model(armature=cfg.sim.hg.armature)
    hc, _ = build_hg_cfg(cfg, n, cfg.sim.dt, 5, js)  # the seed enters only the env logic, not the physics
    return hc, model, js


def signature(lam, mu, jf, dt):
    """Discrete state of one substep's impulses lam[LAMW]: frozensets of row labels."""
    act, cone, slip, lim = set(), set(), set(), set()
    for c in range(NC + NPAIR):
        b = 3 * c
        ln = lam[b]
        if ln > 0:
            lab = f"ground{c}" if c < NC else f"pair{c - NC}"
            act.add(lab)
            lt = np.hypot(lam[b + 1], lam[b + 2])
            m = mu if c < NC else mu[1]
            m = m[0] if isinstance(m, tuple) else m
            if lt >= m * ln * (1 - 1e-4):
                cone.add(lab)
    for j in range(ND):
        if lam[LAM_LIM + j] != 0:
            lim.add(f"limit{j}")
        f = jf[j] * dt
        if f > 0 and abs(lam[LAM_FRIC + j]) >= f * (1 - 1e-5):
            slip.add(f"jfric{j}")
    return {"active": act, "cone": cone, "slip": slip, "limit": lim}


def diff(a, b):
    return {k: sorted(a[k] ^ b[k]) for k in a if a[k] ^ b[k]}


def replay(hc, model, S1, a1, precision, pert_rng=None):
    """Substep-by-substep replay of one env: (outputs after 10 substeps, [lam after each])."""
    hc1 = type(hc).from_buffer_copy(hc)
    dec = hc.decimation
    hc1.decimation = 1
    hc1.num_envs = 1
    S = dict(S1)
    if pert_rng is not None:
        for k in ("root_states", "dof_pos", "dof_vel"):
            x = np.asarray(S[k])
            S[k] = (x * (1 + 2.0 ** -22 * pert_rng.standard_normal(x.shape))).astype(np.float32)
    sim = ST.ref_sim(hc1, model, S, precision)
    lams = []
    for _ in range(dec):
        sim.step(a1)
        lams.append(sim.lam[0].astype(np.float64).copy())
    return ST.outputs(sim), lams, sim


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--members", type=int, default=64)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    D = np.load(args.dump, allow_pickle=False)
    S = {k[2:]: D[k] for k in D.files if k.startswith("S_")}
    gpu = {k[4:]: D[k] for k in D.files if k.startswith("gpu_")}
    a_ref, lam_gpu = D["a_ref"], D["lambda_out"]
    n = a_ref.shape[0]
    hc, model, js = smoke_cfg(n)
    r64, report, fails, bad = ST.check_step(hc, model, S, a_ref, gpu)
    print("recomputed verdict:", json.dumps(report), "fails:", fails)
    dt = float(hc.sim_dt)
    jf = [js["bodies"][j + 1]["joint"]["friction"] for j in range(12)]
    ground_fric = float(hc.ground_friction)
    out = {"dump": os.path.relpath(args.dump, REPO), "verdict": report, "fails": fails, "envs": {}}
    base = ST.outputs(r64)
    # the element tolerance of the check (same seeded ensemble and spread as check_step)
    fields = ST.FIELDS
    gap32 = ST.gap(ST.f32_members(hc, model, S, a_ref, fields, members=3), r64, fields)
    sp = ST.f64_spread(hc, model, S, a_ref, r64, fields)
    kp = np.array([hc.kp[j] for j in range(12)])
    kd = np.array([hc.kd[j] for j in range(12)])
    _, _, tols = ST.compare(gpu, r64, gap32, sp, fields, kp, kd, ST.STEP_TOL_K)
    for e in report["outlier_ids"]:
        S1 = {k: np.asarray(v)[e:e + 1] for k, v in S.items()}
        a1 = a_ref[e:e + 1]
        fr = float(np.asarray(S["env_frictions"]).reshape(-1)[e])
        mu = (0.5 * (fr + ground_fric), fr)
        o64, l64, _ = replay(hc, model, S1, a1, "f64")
        sig64 = [signature(lv, mu, jf, dt) for lv in l64]
        # the critical contact: the ground contact that comes closest to its friction cone in the
        # f64 run (ratio |lambda_t| / (mu lambda_n) of the substep's final impulses)
        def cone_ratios(lams):
            r = np.zeros((len(lams), NC))
            for s_, lv in enumerate(lams):
                ln = lv[0:3 * NC:3]
                lt = np.hypot(lv[1:3 * NC:3], lv[2:3 * NC:3])
                r[s_] = np.where(ln > 0, lt / np.maximum(mu[0] * ln, 1e-300), 0.0)
            return r
        r64c = cone_ratios(l64)
        crit = int(np.unravel_index(np.argmax(r64c), r64c.shape)[1])
        # the GPU's deviation in this env, in units of the element tolerance's yardstick
        gdev = {f: float(np.abs(np.asarray(gpu[f][e], np.float64) - base[f][e]).max()) for f in ST.FIELDS}
        rec = {"gpu_max_dev": gdev, "f64_signature_per_substep": [{k: sorted(v) for k, v in s.items()} for s in sig64],
               "gpu_final_vs_f64_final": diff(signature(lam_gpu[e].astype(np.float64), mu, jf, dt), sig64[-1]),
               "critical_contact": f"ground{crit}", "critical_f64_cone_ratio_per_substep": r64c[:, crit].round(6).tolist(),
               "builds": {}}
        for prec in ("f32", "f32q"):
            rng = np.random.default_rng(99 if prec == "f32" else 199)
            stats = {"members": args.members, "signature_left_f64": 0, "first_event_kinds": {}, "first_event_substeps": {},
                     "outside_tol": 0, "outside_tol_with_event": 0, "outside_tol_without_event": 0,
                     "max_dev": {f: 0.0 for f in ST.FIELDS}, "crit_max_ratio_outside": [], "crit_max_ratio_inside": []}
            for m in range(args.members):
                o, lams, _ = replay(hc, model, S1, a1, prec, rng if m else None)
                ev = None
                for s, lv in enumerate(lams):
                    d = diff(signature(lv, mu, jf, dt), sig64[s])
                    if d:
                        ev = (s, d)
                        break
                dev = {f: float(np.abs(np.asarray(o[f][0], np.float64) - o64[f][0]).max()) for f in ST.FIELDS}
                for f in ST.FIELDS:
                    stats["max_dev"][f] = max(stats["max_dev"][f], dev[f])
                # outside the check's element tolerance (against the full-step f64 outputs, as the GPU)
                reach = any(bool((np.abs(np.asarray(o[f][0], np.float64) - base[f][e]) > tols[f][e]).any())
                            for f in fields)
                stats["outside_tol"] += int(reach)
                stats["crit_max_ratio_outside" if reach else "crit_max_ratio_inside"].append(
                    round(float(cone_ratios(lams)[:, crit].max()), 6))
                if ev is not None:
                    stats["signature_left_f64"] += 1
                    kinds = ",".join(sorted(ev[1]))
                    stats["first_event_kinds"][kinds] = stats["first_event_kinds"].get(kinds, 0) + 1
                    stats["first_event_substeps"][str(ev[0])] = stats["first_event_substeps"].get(str(ev[0]), 0) + 1
                    stats["outside_tol_with_event"] += int(reach)
                    if "example" not in stats:
                        stats["example"] = {"member": m, "substep": ev[0], "rows": ev[1], "dev": dev}
                else:
                    stats["outside_tol_without_event"] += int(reach)
            rec["builds"][prec] = stats
        out["envs"][str(e)] = rec
        print(f"env {e}: GPU dev {gdev}")
        print(f"  critical contact ground{crit}: f64 cone ratio per substep {r64c[:, crit].round(4).tolist()}")
        print("  GPU final impulses vs f64 final:", rec["gpu_final_vs_f64_final"])
        for prec, st in rec["builds"].items():
            print(f"  {prec}: {st['signature_left_f64']}/{st['members']} builds leave the f64 signature "
                  f"(kinds {st['first_event_kinds']}, substeps {st['first_event_substeps']}); outside the element "
                  f"tolerance: {st['outside_tol_with_event']} with an event, {st['outside_tol_without_event']} without")
            print(f"    critical contact's max cone ratio: builds outside {sorted(st['crit_max_ratio_outside'])}; "
                  f"inside: min {min(st['crit_max_ratio_inside'], default=0):.6f} max {max(st['crit_max_ratio_inside'], default=0):.6f}")
    if args.out:
        os.makedirs(args.out, exist_ok=True)
        with open(os.path.join(args.out, "classification.json"), "w") as f:
            json.dump(out, f, indent=1, default=lambda x: sorted(x) if isinstance(x, set) else str(x))
    return out


if __name__ == "__main__":
    main()
