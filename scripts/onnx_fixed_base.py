"""Contact-free probe of the reference's trained actor (humanoid/OnnxTest.onnx): conventions vs physics.

The closed-loop sweep (scripts/onnx_sweep.py) cannot tell a wrong observation / action convention
from a contact model that differs from PhysX: every variant falls, with contact.  Here the robot is
first SUSPENDED — base link fixed in place (no ground contact is generated for a fixed base), every
self-collision pair dropped — so only the actor and the articulated legs remain.  A policy trained
with humanoid-gym's reference-gait reward (humanoid_env.py:714-744, compute_ref_state: hip pitch /
knee / ankle pitch at 0.17 / 0.34 / 0.17 rad x sin(2 pi phase), left leg on sin < 0, right leg on
sin > 0, zero within |sin| < 0.1, cycle 0.64 s) keeps stepping in the air at its gait phase; its
joints then move in phase with that reference gait in the ROBOT's joint frame (q - q_default, the
URDF's axes, where the reference defines it) if and only if the actor's joint conventions are the
robot's.  In the air the actor is close to an open-loop pattern generator driven by its phase input,
so the joint pattern it produces does not depend on how the observation is built — which is what
lets the probe isolate the joint conventions.

Per convention VARIANT of onnx_sweep.py (the physics variants are left out here) and command vx in
{0, 0.3, 0.5}: 5 s of the sim2sim loop (oracle/sim2sim_ref.py, f64 oracle physics, reference
sim2sim.py:185-236); over the last 4 s, for each leg's hip pitch, knee and ankle pitch, the
zero-lag correlation with compute_ref_state (at the phase the policy perceives), the best-lag
correlation within half a cycle and its lag, the amplitude ratio and the periodic fraction (variance
in the first four harmonics of 1 / cycle).  A variant MATCHES when both legs' hip pitch and knee are in phase
(zero-lag correlation > 0) at every command.  Controls: the zero-action policy (no gait), and an
actor trained from scratch on THIS physics (tests/golden/hg_trained_actor.npz, scripts/train_eval.sh,
3000 iterations), which walks here and matches: the probe's positive control.

Then: the joints the baseline moves AGAINST the reference gait are driven with the opposite sign
(the convention the air gait points to), the joints the air gait cannot judge (hip roll / yaw,
ankle roll) are flipped greedily by closed-loop survival, and the closed-loop sweep (ground
contact, 20 s) is re-run under the derived signs with one physics term changed per row: the rows
say which half of the round-4 deviation is conventions and which is physics.

  python scripts/onnx_fixed_base.py [--duration 5] [--closed-duration 20] [--out profiles/r5_onnx_fixed_base]

CPU only.  Writes <out>/onnx_fixed_base.json and <out>/onnx_fixed_base.md; tests/test_onnx_fixed_base.py
pins the outcome.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle"),
           os.path.join(REPO, "scripts")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import onnx_sweep as SW  # noqa: E402

FIXTURE = os.path.join(REPO, "tests", "golden", "onnx_actor.npz")
OWN = os.path.join(REPO, "tests", "golden", "hg_trained_actor.npz")
COMMANDS = ((0.0, 0.0, 0.0), (0.3, 0.0, 0.0), (0.5, 0.0, 0.0))
JOINTS = (2, 3, 4, 8, 9, 10)   # LAYOUT12.ref_idx: left / right hip pitch, knee, ankle pitch
JOINT_NAMES = ("l_pitch", "l_knee", "l_ankle", "r_pitch", "r_knee", "r_ankle")
DOF_NAMES = ("l_roll", "l_yaw", "l_pitch", "l_knee", "l_ankle", "l_ankle_roll",
             "r_roll", "r_yaw", "r_pitch", "r_knee", "r_ankle", "r_ankle_roll")
SKIP_S = 1.0
# the physical gait matches the reference gait when both legs' hip pitch and knee — the joints
# that carry the stepping motion — move IN phase with it: zero-lag correlation > 0 at every command
# (the actor trained here, the probe's positive control: 0.36-0.87 on those four, while its ankles,
# which also balance the foot, range -0.03..0.91; an inverted joint sits near -0.8).  Ankles are
# reported, and an ankle inverted at every command is flipped with the rest below.
CRIT = dict(zero_lag_corr=0.0, joints=("l_pitch", "l_knee", "r_pitch", "r_knee"))
PHYSICS = ("d11_gains", "action_scale_0.5", "no_joint_friction", "armature_0.01", "pgs_50_sweeps",
           "no_self_collision", "ground_friction_2.0", "substep_0.5ms")


def convention_variants():
    V = SW.variants()
    return {k: v for k, v in V.items() if k not in PHYSICS and not k.startswith("no_self_collision+")}


def perceived_phase(ph, mode):
    """Phase the policy perceives from the sin / cos it is fed (sim2sim_ref.Sim2SimRef.frame)."""
    return {"sincos": ph, "neg": ph + 0.5, "swap": 0.25 - ph}[mode]


def ref_gait(ph, scale=0.17):
    """compute_ref_state (humanoid_env.py:714-744) on the 12-DOF layout, at phases ph [T]."""
    s = np.sin(2 * math.pi * ph)
    ref = np.zeros((len(ph), 12))
    sl, sr = np.minimum(s, 0), np.maximum(s, 0)
    for k, (j, m) in enumerate(zip(JOINTS, (1, 2, 1, 1, 2, 1))):
        ref[:, j] = (sl if k < 3 else sr) * scale * m
    ref[np.abs(s) < 0.1] = 0
    return ref


def _pearson(a, b):
    a, b = a - a.mean(), b - b.mean()
    d = math.sqrt(float((a * a).sum() * (b * b).sum()))
    return float((a * b).sum() / d) if d > 0 else 0.0


def joint_metrics(x, r, dt, cycle):
    """x, r [T]: one joint's trajectory and reference; best-lag correlation within half a cycle."""
    half = int(round(cycle / dt / 2))
    best = (-2.0, 0)
    for lag in range(-half, half + 1):   # x[t] against r[t - lag]
        if lag >= 0:
            c = _pearson(x[lag:], r[:len(r) - lag])
        else:
            c = _pearson(x[:lag], r[-lag:])
        if c > best[0]:
            best = (c, lag)
    t = np.arange(len(x)) * dt
    cols = [np.ones_like(t)]
    for h in range(1, 5):
        w = 2 * math.pi * h / cycle
        cols += [np.sin(w * t), np.cos(w * t)]
    A = np.stack(cols, 1)
    coef, *_ = np.linalg.lstsq(A, x, rcond=None)
    var = float(((x - x.mean()) ** 2).sum())
    # a joint that does not move (std below 1e-6 rad: the zero-action control) has no periodic part
    periodic = 1.0 - float(((x - A @ coef) ** 2).sum()) / var if x.std() > 1e-6 else 0.0
    amp = float(x.std() / r.std()) if r.std() > 0 else 0.0
    return dict(corr=round(best[0], 4), lag_s=round(best[1] * dt, 3), amp=round(amp, 4),
                periodic=round(periodic, 4), zero_lag_corr=round(_pearson(x, r), 4))


def passes(jm):
    return all(jm[k]["zero_lag_corr"] > CRIT["zero_lag_corr"] for k in CRIT["joints"])


def run_fixed(name, v, W, duration):
    import sim2sim_ref as SR
    cmds = np.asarray(COMMANDS, np.float64)
    n = len(cmds)
    hc, model, default, cfg = SW.build(v, n, fixed_base=True)
    assert hc.fix_base_link == 1
    root = np.zeros((n, 13))
    root[:, 0:3] = cfg.init_state.pos
    root[:, 3:7] = cfg.init_state.rot
    policy = (lambda x: np.zeros((x.shape[0], 12))) if v.get("policy") == "zero" else SR.mlp(W)
    cycle = v.get("cycle", cfg.rewards.cycle_time)
    sim = SR.Sim2SimRef(hc, model, policy, root, default[None].repeat(n, 0), np.zeros((n, 12)), np.full(n, model.mass[0]),
                        np.ones(n), cmds, precision="f64", cycle_time=cycle, default_dof_pos=default,
                        joint_perm=v.get("perm"), joint_sign=v.get("sign"), omega_frame=v.get("omega", "base"),
                        euler=v.get("euler", "sim2sim"), phase=v.get("phase", "sincos"))
    dt = float(hc.dt)
    steps = int(round(duration / dt))
    traj, phases = np.zeros((steps, n, 12)), np.zeros(steps)
    t0 = time.time()
    for k in range(steps):
        phases[k] = k * dt / cycle           # the phase of the frame the action of step k came from
        sim.step()
        traj[k] = sim.sim.q - default   # the ROBOT's joint frame (the URDF's, where the reference gait lives)
    assert not sim.sim.nonfinite.any()
    skip = int(round(SKIP_S / dt))
    ref = ref_gait(perceived_phase(phases, v.get("phase", "sincos")))[skip:]
    per = []
    for c in range(n):
        jm = {JOINT_NAMES[i]: joint_metrics(traj[skip:, c, j], ref[:, j], dt, cycle) for i, j in enumerate(JOINTS)}
        per.append(dict(command=list(COMMANDS[c]), joints=jm, reproduces=passes(jm),
                        base_fixed=bool(np.allclose(sim.sim.root[c, 0:7], root[c, 0:7]))))
    return dict(name=name, commands=per, reproduces=all(p["reproduces"] for p in per), wall_s=round(time.time() - t0, 1))


def summary_row(r):
    cells = []
    for p in r["commands"]:
        jm = p["joints"]
        signs = " ".join(f"{k}{m['zero_lag_corr']:+.2f}" for k, m in jm.items())
        cells.append(f"{p['command'][0]:.1f}: {signs}; periodic {min(m['periodic'] for m in jm.values()):.2f}, "
                     f"amp {min(m['amp'] for m in jm.values()):.2f}..{max(m['amp'] for m in jm.values()):.2f}")
    return f"| {r['actor']} | {r['name']} | {'yes' if r['reproduces'] else 'no'} | " + " ; ".join(cells) + " |"


def inverted_joints(row):
    """Robot joints (indices) moving against the reference gait at every command of a row."""
    return [j for i, j in enumerate(JOINTS)
            if all(p["joints"][JOINT_NAMES[i]]["zero_lag_corr"] < 0 for p in row["commands"])]


def closed_loop(actor_w, conv, label, duration, envs_per_command):
    """The closed-loop (ground contact) sweep under convention set `conv` with one physics term
    changed per row (onnx_sweep.py's physics variants), 4 commands x envs_per_command envs."""
    V = SW.variants()
    rows = []
    for name in ("baseline",) + PHYSICS + ("hip_roll_yaw_sign_both", "legs_mirrored"):
        v = dict(conv)
        extra = {} if name == "baseline" else dict(V[name])
        if "sign" in extra:  # compose sign changes
            extra["sign"] = np.asarray(extra["sign"]) * np.asarray(conv.get("sign", np.ones(12)))
        v.update(extra)
        r = SW.run_variant(f"{label} + {name}" if name != "baseline" else label, v, actor_w, envs_per_command, duration)
        rows.append(r)
        print(f"  closed loop {r['name']:48s} falls {r['falls']:2d}/{r['envs']}  survival {r['mean_survival_s']:.2f} s",
              flush=True)
    return rows


UNSEEN = (0, 1, 5, 6, 7, 11)   # hip roll, hip yaw, ankle roll: no reference-gait motion to judge in the air


def refine_unseen(actor_w, sign, duration, envs_per_command=2, rounds=2):
    """Greedy closed-loop refinement of the joints the air probe cannot see (roll, yaw, ankle roll):
    flip the one whose flip raises the mean survival most, until none does."""
    sign = np.asarray(sign, np.float64).copy()
    best = SW.run_variant("refine", {"sign": sign}, actor_w, envs_per_command, duration)["mean_survival_s"]
    trail = [dict(flip=None, survival_s=round(best, 3))]
    for _ in range(rounds):
        pick = None
        for j in UNSEEN:
            t = sign.copy()
            t[j] = -t[j]
            s_ = SW.run_variant("refine", {"sign": t}, actor_w, envs_per_command, duration)["mean_survival_s"]
            trail.append(dict(flip=j, survival_s=round(s_, 3)))
            if s_ > best + 1e-6:
                best, pick = s_, j
        if pick is None:
            break
        sign[pick] = -sign[pick]
        trail.append(dict(taken=pick, survival_s=round(best, 3)))
        print(f"  refine: flip joint {pick} -> mean survival {best:.2f} s", flush=True)
    return sign, trail


def load(path):
    W = np.load(path, allow_pickle=False)
    return {k: W[k] for k in W.files}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--duration", type=float, default=5.0, help="air probe seconds per command")
    ap.add_argument("--closed-duration", type=float, default=20.0, help="closed-loop seconds")
    ap.add_argument("--closed-envs", type=int, default=8, help="closed-loop envs per command")
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "8")))
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r5_onnx_fixed_base"))
    a = ap.parse_args()
    import physics_ref as P
    P.set_threads(a.threads)
    actors = {"OnnxTest.onnx": FIXTURE}
    if os.path.exists(OWN):
        actors["hg-trained (control)"] = OWN
    rows = []
    for actor, path in actors.items():
        W = load(path)
        for name, v in convention_variants().items():
            if a.only and name not in a.only:
                continue
            if actor != "OnnxTest.onnx" and name not in ("baseline", "zero_action_policy (reference point)"):
                continue
            r = run_fixed(name, v, W, a.duration)
            r["actor"] = actor
            rows.append(r)
            print(summary_row(r), f"({r['wall_s']} s)", flush=True)
    W = load(FIXTURE)
    base = next(r for r in rows if r["actor"] == "OnnxTest.onnx" and r["name"] == "baseline")
    flips = inverted_joints(base)
    closed, derived = [], None
    if flips:
        # the convention the air gait points to: the actor's inverted joints driven with the opposite sign
        sign = np.ones(12)
        sign[flips] = -1.0
        conv = {"sign": sign}
        label = "air_gait_signs(" + ",".join(JOINT_NAMES[JOINTS.index(j)] for j in flips) + ")"
        derived = run_fixed(label, conv, W, a.duration)
        derived["actor"] = "OnnxTest.onnx"
        rows.append(derived)
        print(summary_row(derived), flush=True)
        # the joints the air gait cannot judge, by closed-loop survival (20 s horizon)
        sign, trail = refine_unseen(W, sign, a.closed_duration)
        extra = [j for j in UNSEEN if sign[j] < 0]
        if extra:
            label += " + " + ",".join(DOF_NAMES[j] for j in extra)
        conv = {"sign": sign}
        closed = closed_loop(W, conv, label, a.closed_duration, a.closed_envs)
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "onnx_fixed_base.json"), "w") as f:
        json.dump(dict(loop="oracle/sim2sim_ref.py, base fixed, no self-collision, f64 oracle physics",
                       reference_gait="compute_ref_state, humanoid_env.py:714-744 (12-DOF layout)",
                       frame="robot joint frame (q - q_default, URDF axes)", criteria=CRIT, skip_s=SKIP_S,
                       commands=[list(c) for c in COMMANDS], variants=rows,
                       inverted_joints_baseline=[JOINT_NAMES[JOINTS.index(j)] for j in flips],
                       derived_signs=(sign.tolist() if flips else None),
                       refinement=(trail if flips else None), closed_duration_s=a.closed_duration,
                       closed_loop_under_derived_signs=closed), f, indent=1)
    with open(os.path.join(a.out, "onnx_fixed_base.md"), "w") as f:
        f.write(f"# Suspended-robot probe of OnnxTest.onnx ({a.duration:g} s per command, last "
                f"{a.duration - SKIP_S:g} s analysed)\n\n")
        f.write("Regenerate: `python scripts/onnx_fixed_base.py` (CPU, oracle physics, base fixed, no self-collision; "
                "test: `tests/test_onnx_fixed_base.py`).  Per command vx: the zero-lag correlation of each hip-pitch / "
                "knee / ankle-pitch joint's motion (robot frame, q - q_default) with compute_ref_state "
                "(humanoid_env.py:714-744), the smallest periodic fraction (variance in the first four harmonics of the "
                "gait cycle) and the amplitude range relative to the reference.  Matches = both legs' hip pitch and "
                "knee in phase (zero-lag correlation > 0) at every command.\n\n")
        f.write("| actor | variant | matches | per command |\n|---|---|---|---|\n")
        for r in rows:
            f.write(summary_row(r) + "\n")
        if closed:
            f.write(f"\n## Closed loop (ground contact, {a.closed_envs} envs per command, {a.closed_duration:g} s) under "
                    f"the derived signs, one more term per row\n\n")
            f.write("Signs: the air probe's inverted joints, then the roll / yaw / ankle-roll joints it cannot judge "
                    "flipped greedily by closed-loop survival (refinement trail in the JSON).  "
                    "The first row is the derived convention set alone.\n\n")
            f.write(SW.table(closed, a.closed_duration))
    print("->", a.out)


if __name__ == "__main__":
    main()
