"""Constraint rows per env and per K_step wave (envs 2p, 2p + 1) at the bench's steady state: the
bench's runner (4096 envs, T = 24, random-init policy) after WARMUP iterations, rows counted from
the warm-start impulse table as bench.active_rows counts them.  Says how often both envs of a
wave fit 16 rows (the case a packed 32 x 32 Delassus tile, one env per 16-row half, would serve).

  python scripts/probes/rows_dist.py [--warmup 6] [--out gpurun_out/r6_kstep/rows_dist.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import bench
    from humanoid import _native as N
    from humanoid.algo.ppo import OnPolicyRunner
    torch.manual_seed(5)
    env = bench.make_env(4096, "cuda:0", seed=5)
    runner = OnPolicyRunner(env, bench.train_cfg(24), log_dir=None, device="cuda:0")
    res = {}
    for it in range(args.warmup):
        runner.learn(1, init_at_random_ep_len=(it == 0))
        lam = env._view(N.T["CONTACT_LAMBDA"]).cpu().numpy()
        nc3 = (N.HG_MAX_CONTACTS + N.HG_MAX_PAIRS) * 3
        contacts = (lam[:, 0:nc3:3] > 0).sum(1)
        limits = (lam[:, nc3:nc3 + N.HG_MAX_DOF] != 0).sum(1)
        fric = sum(1 for b in range(len(env._model.joint_friction)) if env._model.joint_friction[b] > 0)
        rows = 3 * np.minimum(contacts, 9) + limits + fric
        pair = np.maximum(rows[0::2], rows[1::2])
        res[it] = {"mean_rows": float(rows.mean()), "p50": float(np.median(rows)), "p90": float(np.quantile(rows, 0.9)),
                   "waves_max_rows_le_16": float((pair <= 16).mean()), "waves_max_rows_le_12": float((pair <= 12).mean()),
                   "hist": np.bincount(rows, minlength=33)[:33].tolist()}
        print(it, json.dumps(res[it]), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
