"""Convention sweep of the reference's trained actor (humanoid/OnnxTest.onnx) in the CPU reference
physics — the reproducible form of the PhysX-side probe.

The actor (weights fixture tests/golden/onnx_actor.npz) is driven closed-loop the way the
reference's deployment script drives it (/root/reference/humanoid/scripts/sim2sim.py:185-236),
on oracle/sim2sim_ref.py (numpy loop around oracle/physics_ref.c, f64), once per VARIANT: one
convention or physics term changed against the trained configuration.  Conventions change the
policy's view of the robot and its action together (joint permutation / signs, IMU frame, Euler
range, gait phase, default pose, cycle time); physics variants change the simulated robot.

  python scripts/onnx_sweep.py [--duration 5] [--envs_per_command 4] [--only name ...]
         [--out profiles/r4_onnx_sweep]

Writes <out>/onnx_sweep.json (per variant and command: falls, mean survival, tracking error,
distance walked along the command) and <out>/onnx_sweep.md (the table DESIGN.md §4 cites).
CPU only; nothing here touches the GPU.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FIXTURE = os.path.join(REPO, "tests", "golden", "onnx_actor.npz")
COMMANDS = ((0.0, 0.0, 0.0), (0.3, 0.0, 0.0), (0.5, 0.0, 0.0), (-0.25, 0.0, 0.0))
# DOF order of the model (Isaac Gym's depth-first order of XBot-L.urdf; tools/urdf_compile.py):
# 0..5 left roll, yaw, pitch, knee, ankle pitch, ankle roll; 6..11 the right leg
L_ROLL, L_YAW, L_PITCH, L_KNEE, L_APITCH, L_AROLL = range(6)
R_ = 6
SWAP = [6, 7, 8, 9, 10, 11, 0, 1, 2, 3, 4, 5]
# the fork's D11 sim2sim defaults (sim2sim.py:107-120): hip pitch -14.884 deg, knee 2x, ankle pitch
BENT = {2: -14.884 / 180 * math.pi, 3: 2 * 14.884 / 180 * math.pi, 4: -14.886 / 180 * math.pi}
D11_KP = [100, 100, 200, 200, 50, 25] * 2   # sim2sim.py:323-324
D11_KD = [10, 10, 10, 10, 2, 1] * 2


def _sign(*flips):
    s = np.ones(12)
    for j in flips:
        s[j] = -1.0
    return s


def variants():
    """name -> dict of switches (conventions: perm / sign / omega / euler / phase / cycle / default
    pose / action scale; physics: gains, armature, joint friction, sweeps, self-collision, ground
    friction, substep)."""
    V = {"baseline": {}, "zero_action_policy (reference point)": dict(policy="zero")}
    V["cycle_0.85"] = dict(cycle=0.85)
    V["bent_knee_default"] = dict(default=BENT)
    V["d11_gains"] = dict(kp=D11_KP, kd=D11_KD)
    V["bent_knee+d11_gains+cycle_0.85"] = dict(default=BENT, kp=D11_KP, kd=D11_KD, cycle=0.85)
    V["legs_swapped"] = dict(perm=SWAP)
    V["legs_mirrored"] = dict(perm=SWAP, sign=_sign(L_ROLL, L_YAW, L_AROLL, R_ + L_ROLL, R_ + L_YAW, R_ + L_AROLL))
    for side, o in (("left", 0), ("right", R_), ("both", None)):
        legs = (0, R_) if o is None else (o,)
        V[f"pitch_chain_sign_{side}"] = dict(sign=_sign(*[b + j for b in legs for j in (L_PITCH, L_KNEE, L_APITCH)]))
        V[f"hip_roll_sign_{side}"] = dict(sign=_sign(*[b + L_ROLL for b in legs]))
        V[f"hip_yaw_sign_{side}"] = dict(sign=_sign(*[b + L_YAW for b in legs]))
        V[f"hip_roll_yaw_sign_{side}"] = dict(sign=_sign(*[b + j for b in legs for j in (L_ROLL, L_YAW)]))
    V["ankle_roll_sign_both"] = dict(sign=_sign(L_AROLL, R_ + L_AROLL))
    V["omega_world_frame"] = dict(omega="world")
    V["omega_negated"] = dict(omega="neg")
    V["euler_0_2pi"] = dict(euler="0_2pi")
    V["euler_negated"] = dict(euler="neg")
    V["phase_half_cycle"] = dict(phase="neg")
    V["phase_sin_cos_swapped"] = dict(phase="swap")
    V["action_scale_0.5"] = dict(action_scale=0.5)
    V["no_joint_friction"] = dict(joint_friction=False)
    V["armature_0.01"] = dict(armature=0.01)
    V["pgs_50_sweeps"] = dict(pgs=50)
    V["no_self_collision"] = dict(self_collisions=False)
    V["ground_friction_2.0"] = dict(ground_friction=2.0)
    V["substep_0.5ms"] = dict(sim_dt=0.0005)
    V["no_self_collision+hip_roll_yaw_sign_both"] = dict(self_collisions=False, sign=_sign(L_ROLL, L_YAW, R_ + L_ROLL,
                                                                                            R_ + L_YAW))
    return V


def build(v, n, fixed_base=False):
    """(hc, model, default pose [12]) of a variant: the sim2sim URDF profile (humanoid.scripts.
    sim2sim.make_cfg) with the variant's physics changes, compiled as XBotLFreeEnv.create_sim does.
    fixed_base: the base link held in place (asset.fix_base_link; no ground contact is generated
    for a fixed base) and every self-collision pair dropped — the robot suspended in free space
    (scripts/onnx_fixed_base.py)."""
    from humanoid import _native as N
    from humanoid.envs.custom.humanoid_env import build_hg_cfg
    from humanoid.scripts.sim2sim import make_cfg
    cfg = make_cfg("urdf", n, 30.0, self_collisions=v.get("self_collisions", True) and not fixed_base)
    cfg.asset.fix_base_link = bool(fixed_base)
    if "default" in v:
        names = N.model_names(N.load_model()[1])[1]
        angles = dict(cfg.init_state.default_joint_angles)  # a class-level dict: never mutate it
        for j, a in v["default"].items():
            angles[names[j]] = a
        cfg.init_state.default_joint_angles = angles
    if "armature" in v:
        cfg.sim.hg.armature = v["armature"]
    if "joint_friction" in v:
        cfg.sim.hg.joint_friction = v["joint_friction"]
    if "pgs" in v:
        cfg.sim.hg.pgs_iterations = v["pgs"]
    if "ground_friction" in v:
        cfg.terrain.static_friction = v["ground_friction"]
    if "action_scale" in v:
        cfg.control.action_scale = v["action_scale"]
    sim_dt = v.get("sim_dt", cfg.sim.dt)
    if "sim_dt" in v:
        cfg.control.decimation = int(round(cfg.control.decimation * cfg.sim.dt / sim_dt))
    hgc = cfg.sim.hg
    model, js = N.load_model(armature=hgc.armature, joint_friction=getattr(hgc, "joint_friction", True),
                             self_collisions=cfg.asset.self_collisions == 0)
    hc, aux = build_hg_cfg(cfg, n, sim_dt, 5, js)
    if "kp" in v:
        for j in range(12):
            hc.kp[j], hc.kd[j] = v["kp"][j], v["kd"][j]
    return hc, model, np.array(aux["default_dof_pos"], np.float64), cfg


def run_variant(name, v, W, envs_per_command, duration, seed=3):
    import sim2sim_ref as SR
    cmds = np.repeat(np.asarray(COMMANDS, np.float64), envs_per_command, axis=0)
    n = len(cmds)
    hc, model, default, cfg = build(v, n)
    rng = np.random.default_rng(seed)
    root = np.zeros((n, 13))
    root[:, 0:3] = cfg.init_state.pos
    root[:, 3:7] = cfg.init_state.rot
    q = default + 0.02 * rng.uniform(-1, 1, (n, 12))   # a small per-env spread around the pose
    qd = np.zeros((n, 12))
    mass = np.full(n, model.mass[0])
    fric = np.full(n, 1.0)                              # the env's friction without randomisation
    policy = (lambda x: np.zeros((x.shape[0], 12))) if v.get("policy") == "zero" else SR.mlp(W)
    sim = SR.Sim2SimRef(hc, model, policy, root, q, qd, mass, fric, cmds, precision="f64",
                        cycle_time=v.get("cycle", cfg.rewards.cycle_time), default_dof_pos=default,
                        joint_perm=v.get("perm"), joint_sign=v.get("sign"), omega_frame=v.get("omega", "base"),
                        euler=v.get("euler", "sim2sim"), phase=v.get("phase", "sincos"))
    steps = int(round(duration / float(hc.dt)))
    t0 = time.time()
    r = sim.run(steps)
    per = []
    for c in range(len(COMMANDS)):
        s = slice(c * envs_per_command, (c + 1) * envs_per_command)
        per.append(dict(command=list(COMMANDS[c]), falls=int(r["fell"][s].sum()),
                        mean_survival_s=float(r["survival_s"][s].mean()),
                        lin_vel_error=float(r["lin_vel_error"][s].mean()), travel_m=float(r["travel_m"][s].mean())))
    return dict(name=name, switches={k: (list(map(float, x)) if isinstance(x, (list, np.ndarray)) else
                                         ({int(a): float(b) for a, b in x.items()} if isinstance(x, dict) else x))
                                     for k, x in v.items()},
                envs=n, duration_s=duration, falls=int(r["fell"].sum()), mean_survival_s=float(r["survival_s"].mean()),
                commands=per, wall_s=round(time.time() - t0, 1))


def table(rows, duration):
    out = ["| variant | falls | mean survival (s) | per command (vx: survival s / walked m) |", "|---|---|---|---|"]
    for r in rows:
        cells = ", ".join(f"{c['command'][0]:+.2f}: {c['mean_survival_s']:.2f} / {c['travel_m']:+.2f}"
                          for c in r["commands"])
        out.append(f"| {r['name']} | {r['falls']}/{r['envs']} | {r['mean_survival_s']:.2f} of {duration:g} | {cells} |")
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--duration", type=float, default=5.0)
    ap.add_argument("--envs_per_command", type=int, default=4)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "8")))
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r4_onnx_sweep"))
    a = ap.parse_args()
    import physics_ref as P
    P.set_threads(a.threads)
    W = np.load(FIXTURE, allow_pickle=False)
    W = {k: W[k] for k in W.files}
    rows = []
    for name, v in variants().items():
        if a.only and name not in a.only:
            continue
        r = run_variant(name, v, W, a.envs_per_command, a.duration)
        rows.append(r)
        print(f"{name:42s} falls {r['falls']:2d}/{r['envs']}  survival {r['mean_survival_s']:.2f} s  "
              + "  ".join(f"{c['command'][0]:+.2f}:{c['mean_survival_s']:.2f}s/{c['travel_m']:+.2f}m" for c in r["commands"])
              + f"  ({r['wall_s']} s)", flush=True)
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "onnx_sweep.json"), "w") as f:
        json.dump(dict(fixture="tests/golden/onnx_actor.npz (humanoid/OnnxTest.onnx initializers)",
                       loop="oracle/sim2sim_ref.py (reference sim2sim.py:185-236), f64 oracle physics",
                       commands=[list(c) for c in COMMANDS], variants=rows), f, indent=1)
    with open(os.path.join(a.out, "onnx_sweep.md"), "w") as f:
        f.write(f"# OnnxTest.onnx convention sweep ({a.envs_per_command} envs per command, {a.duration:g} s)\n\n")
        f.write("Regenerate: `python scripts/onnx_sweep.py` (CPU, oracle physics).  A fall = net contact force on "
                "the base link > 1 N (humanoid_env.py:811-816).\n\n")
        f.write(table(rows, a.duration))
    print("->", a.out)


if __name__ == "__main__":
    main()
