"""The reference's trained XBot-L actor (humanoid/OnnxTest.onnx, weights fixture
tests/golden/onnx_actor.npz) driven closed-loop on hg_sim (GPU) and on the CPU reference physics
(oracle/sim2sim_ref.py), from the same initial state, in the reference's sim2sim loop
(humanoid/scripts/sim2sim.py:185-280): the only artefact in the reference that carries PhysX
behaviour, so the only PhysX-side evidence the build's physics can get.

  python scripts/onnx_closed_loop.py [--profile urdf|mjcf] [--duration 20] [--envs_per_command 16]
         [--out profiles/r3_onnx]

Writes <out>/onnx_closed_loop_<profile>.json: per command the GPU and the CPU-oracle fall counts,
mean fall times, tracking errors, and the closed-loop divergence curves (max |q_gpu - q_f64| and
the CPU fp32 ensemble's max |q_f32 - q_f64| per policy step while the envs stand).
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

FIXTURE = os.path.join(REPO, "tests", "golden", "onnx_actor.npz")
COMMANDS = ((-0.25, 0.0, 0.0), (0.0, 0.0, 0.0), (0.3, 0.0, 0.0), (0.5, 0.0, 0.0))


def cause_slots(js, model):
    """Warm-start impulse slots of the contacts that put force on the base link: base-box corners
    vs the ground, hand capsules vs the thighs / shins, the box bottom face vs the thighs."""
    from humanoid import _native as N
    lp = N.HG_MAX_CONTACTS * 3
    corners = [3 * c for c, cd in enumerate(js["contacts"]) if cd["body"] == 0]
    caps = js["capsules"]
    pairs = js["pairs"][:model.num_pairs]
    hand = [lp + 3 * p for p, (a, b) in enumerate(pairs) if caps[a]["part"] == "hand"]
    box = [lp + 3 * p for p, (a, b) in enumerate(pairs) if caps[a]["part"] == "box_bottom"]
    return {"base_ground": corners, "hand_leg": hand, "box_thigh": box}


DOF_NAMES = ("l_roll", "l_yaw", "l_pitch", "l_knee", "l_ankle", "l_ankle_roll",
             "r_roll", "r_yaw", "r_pitch", "r_knee", "r_ankle", "r_ankle_roll")


def signed_policy(net, sign):
    """The actor with joint sign conventions (oracle/sim2sim_ref.Sim2SimRef joint_sign, identity
    permutation): the policy's joint j is the robot's joint j times sign[j] — its q, qd and last
    action observation columns of every stacked 47-wide frame and its action."""
    import torch
    s = torch.as_tensor(np.asarray(sign, np.float32))
    col = torch.ones(47)
    for off in (5, 17, 29):
        col[off:off + 12] = s
    col = col.repeat(15)

    class Signed(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.net = net
            self.register_buffer("col", col)
            self.register_buffer("sign", s)

        def forward(self, x):
            return self.net(x * self.col) * self.sign
    return Signed()


def compare(profile="urdf", commands=COMMANDS, envs_per_command=8, duration=3.0, ensemble=3, device="cuda:0",
            self_collisions=True, joint_sign=None):
    """GPU sim2sim and the CPU oracle (f64, plus an fp32 ensemble as the divergence yardstick)
    from the GPU env's initial state; ``joint_sign`` (12 x +-1): the actor's joint sign convention
    (scripts/onnx_fixed_base.py derives one).  Returns a dict of numpy arrays / numbers."""
    import torch
    import sim2sim_ref as SR
    from humanoid import _native as N
    from humanoid.scripts import sim2sim as S2
    W = np.load(FIXTURE, allow_pickle=False)
    cmds = np.asarray(commands, np.float32).reshape(-1, 3)
    n = len(cmds) * envs_per_command
    steps = int(round(duration / 0.01))
    env = S2.make_env(profile, n, duration, device, self_collisions=self_collisions)
    torch.cuda.synchronize()
    g = lambda t: t.detach().cpu().numpy().copy()  # noqa: E731
    init = dict(root=g(env.root_states), q=g(env.dof_pos), qd=g(env.dof_vel), lam=g(env._view(N.T["CONTACT_LAMBDA"])),
                mass=g(env.body_mass)[:, 0], fric=g(env.env_frictions)[:, 0])
    hc, model = env._hgcfg, env._model
    cyc = env.cfg.rewards.cycle_time
    slots = cause_slots(env._model_js, model)
    policy = S2.mlp_from_weights(W)
    if joint_sign is not None:
        policy = signed_policy(policy, joint_sign)
    summary, traces = S2.run(policy.to(device).eval(), profile, cmds, duration, envs_per_command,
                             device, env=env, record_q=True)
    q_gpu = traces["q_all"]
    per_cmd = np.repeat(cmds, envs_per_command, axis=0)

    def oracle(prec, pert=0.0, seed=0):
        rng = np.random.default_rng(seed)
        root, q, qd = (x.astype(np.float64) for x in (init["root"], init["q"], init["qd"]))
        if pert:
            q = q * (1 + pert * rng.standard_normal(q.shape))
            qd = qd * (1 + pert * rng.standard_normal(qd.shape))
        dt = np.float64 if prec == "f64" else np.float32
        sim = SR.Sim2SimRef(hc, model, SR.mlp(W, dt), root, q, qd, init["mass"], init["fric"], per_cmd,
                            precision=prec, cycle_time=cyc, lam=init["lam"], cause_slots=slots, joint_sign=joint_sign)
        qs = []
        for _ in range(steps):
            sim.step()
            qs.append(sim.sim.q.astype(np.float64).copy())
        return sim.summary(), np.stack(qs)

    ref64, q64 = oracle("f64")
    ens = [oracle("f32", 2.0 ** -23 if k else 0.0, seed=k) for k in range(ensemble)]
    alive_gpu = np.array(summary["fall_step"])
    # per step: envs still standing in every run (GPU, f64, each ensemble member)
    firsts = [alive_gpu, ref64["fall_step"]] + [e[0]["fall_step"] for e in ens]
    first_fall = np.min([np.where(f < 0, steps + 1, f) for f in firsts], axis=0)
    div_gpu, div_f32 = np.zeros(steps), np.zeros(steps)
    for t in range(steps):
        m = first_fall > t + 1
        if not m.any():
            div_gpu[t:] = np.nan
            div_f32[t:] = np.nan
            break
        div_gpu[t] = np.abs(q_gpu[t][m] - q64[t][m]).max()
        div_f32[t] = max(np.abs(e[1][t][m] - q64[t][m]).max() for e in ens)

    def stats(fall_step, lin_err, yaw_err):
        out = []
        for c in range(len(cmds)):
            s = slice(c * envs_per_command, (c + 1) * envs_per_command)
            fs = np.asarray(fall_step)[s]
            t_fall = np.where(fs < 0, steps, fs) * 0.01
            out.append(dict(command=[float(x) for x in cmds[c]], falls=int((fs >= 0).sum()),
                            mean_fall_time_s=float(t_fall.mean()), lin_vel_error=float(np.mean(lin_err[s])),
                            yaw_rate_error=float(np.mean(yaw_err[s]))))
        return out
    gpu_lin = np.array([c["lin_vel_error"] for c in summary["commands"] for _ in range(envs_per_command)])
    gpu_yaw = np.array([c["yaw_rate_error"] for c in summary["commands"] for _ in range(envs_per_command)])
    return dict(profile=profile, self_collisions=bool(self_collisions), envs=n, steps=steps, duration_s=duration,
                joint_sign=None if joint_sign is None else [float(x) for x in joint_sign],
                gpu=stats(alive_gpu, gpu_lin, gpu_yaw),
                oracle_f64=stats(ref64["fall_step"], ref64["lin_vel_error"], ref64["yaw_rate_error"]),
                oracle_f32=[stats(e[0]["fall_step"], e[0]["lin_vel_error"], e[0]["yaw_rate_error"]) for e in ens],
                fall_cause_f64={k: int(sum(1 for c in ref64["fall_cause"] if c == k))
                                for k in sorted(set(ref64["fall_cause"]))},
                fall_step_gpu=alive_gpu.tolist(), fall_step_f64=ref64["fall_step"].tolist(),
                fall_step_f32=[e[0]["fall_step"].tolist() for e in ens],
                div_gpu=div_gpu.tolist(), div_f32=div_f32.tolist())


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--profile", default="urdf", choices=["urdf", "mjcf"])
    ap.add_argument("--duration", type=float, default=20.0)
    ap.add_argument("--envs_per_command", type=int, default=16)
    ap.add_argument("--ensemble", type=int, default=2)
    ap.add_argument("--no-self-collisions", action="store_true", help="ablation: no self-collision pairs")
    ap.add_argument("--flip", default="", help="comma-separated joints the actor drives with the opposite sign "
                                                  "(scripts/onnx_fixed_base.py), e.g. l_yaw,l_knee,r_yaw,r_pitch,r_ankle")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r3_onnx"))
    a = ap.parse_args()
    sign = None
    if a.flip:
        sign = np.ones(12)
        for nm in a.flip.split(","):
            sign[DOF_NAMES.index(nm)] = -1.0
    import physics_ref as P
    P.set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    r = compare(a.profile, COMMANDS, a.envs_per_command, a.duration, a.ensemble,
                self_collisions=not a.no_self_collisions, joint_sign=sign)
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, f"onnx_closed_loop_{a.profile}{'_noself' if a.no_self_collisions else ''}"
                               f"{'_signs' if sign is not None else ''}.json")
    with open(path, "w") as f:
        json.dump(r, f, indent=1)
    for name in ("gpu", "oracle_f64"):
        for c in r[name]:
            print(f"{name:10s} cmd {c['command']}: falls {c['falls']}/{a.envs_per_command} mean fall time "
                  f"{c['mean_fall_time_s']:.2f} s |v - cmd| {c['lin_vel_error']:.3f} |wz| {c['yaw_rate_error']:.3f}")
    print("oracle f64 termination causes (contacts on the base at the first terminating step):", r["fall_cause_f64"])
    print("->", path)


if __name__ == "__main__":
    main()
