"""Fixed-base trajectory divergence probe (development tool): per-step max |dq| of K_step vs the
f64 oracle, with / without self-collision, and which warm-start slots are active."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(REPO, "humanoid-gym-with-comments_amd"), os.path.join(REPO, "oracle"), REPO,
          os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def run(fixed, sc, steps=1000, n=16):
    import pipeline_ref as PR
    env = T._make_env(n, asset__fix_base_link=fixed, asset__self_collisions=0 if sc else 1,
                      domain_rand__dynamic_randomization=0.0, domain_rand__push_robots=False, noise__add_noise=False)
    S, _, _ = T.snapshot(env)
    oc = T._oracle_cfg(env)
    r64 = T._ref_sim(env, S, "f64")
    prev = np.zeros((n, 12), np.float32)
    j = np.arange(12)
    from humanoid import _native as N
    lamv = env._view(N.T["CONTACT_LAMBDA"])
    for t in range(steps):
        a = np.tile(0.5 * np.sin(2 * np.pi * t * 0.01 / 0.64 + j * np.pi / 6), (n, 1)).astype(np.float32)
        a_ref = PR.preprocess_actions(oc, a, prev, t)
        T._step_only(env, torch.from_numpy(a).cuda(), t)
        prev = env.actions.cpu().numpy()
        r64.step(a_ref.astype(np.float64))
        dq = np.abs(env.dof_pos.cpu().numpy() - r64.q).max()
        lg = lamv.cpu().numpy()
        if t % 100 == 0 or dq > 2e-5:
            act_g = np.nonzero(np.abs(lg).max(0) > 0)[0]
            act_r = np.nonzero(np.abs(r64.lam).max(0) > 0)[0]
            print(f"fixed={fixed} sc={sc} t={t} dq={dq:.3g} gpu_slots={act_g.tolist()} ref_slots={act_r.tolist()}", flush=True)
            if dq > 2e-5:
                e = int(np.argmax(np.abs(env.dof_pos.cpu().numpy() - r64.q).max(1)))
                print(" env", e, "gpu lam", np.round(lg[e][np.abs(lg[e]) > 0], 5), "ref lam", np.round(r64.lam[e][np.abs(r64.lam[e]) > 0], 5))
                print(" gpu q", np.round(env.dof_pos.cpu().numpy()[e], 5), "\n ref q", np.round(r64.q[e], 5))
                break


for sc in (True,):
    run(True, sc)
