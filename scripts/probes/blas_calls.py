"""Which products of one PPO iteration still reach torch's BLAS (hipBLASLt): the bench's runner
(4096 envs, T = 24) runs one warm-up iteration, then one iteration under a TorchDispatchMode that
records every aten mm / addmm / bmm / baddbmm with its operand shapes and strides (the first
update() of a runner is the eager one, whose routes the captured graph replays).

  python scripts/probes/blas_calls.py [--out gpurun_out/r6_gemm/blas_calls.json]
"""
import argparse
import collections
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

OPS = {"mm", "addmm", "bmm", "baddbmm", "matmul", "linear", "_scaled_mm"}


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.calls = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name in OPS:
            desc = tuple((tuple(a.shape), tuple(a.stride()), str(a.dtype).replace("torch.", ""))
                         for a in args if isinstance(a, torch.Tensor))
            self.calls[(name, desc)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import bench
    from humanoid.algo.ppo import OnPolicyRunner
    from humanoid.utils.blas_tuning import use_tuned_gemms
    torch.manual_seed(5)
    use_tuned_gemms()
    env = bench.make_env(4096, "cuda:0", seed=5)
    runner = OnPolicyRunner(env, bench.train_cfg(24), log_dir=None, device="cuda:0")
    runner.alg.use_graphs = False  # every update eager: the routes are the graph's
    runner.learn(1, init_at_random_ep_len=True)
    log = Log()
    with log:
        runner.learn(1)
    torch.cuda.synchronize()
    rows = [{"op": k[0], "operands": [list(map(list, d[:2])) + [d[2]] for d in k[1]], "calls": v}
            for k, v in sorted(log.calls.items(), key=lambda kv: -kv[1])]
    for r in rows:
        print(r["calls"], r["op"], r["operands"])
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
