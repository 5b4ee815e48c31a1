"""Time the PPO iteration (collection / learn) under the BLAS back-end selected by the caller's
environment (hipBLASLt default, rocBLAS via TORCH_BLAS_PREFER_HIPBLASLT=0, TunableOp)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from humanoid.algo.ppo import OnPolicyRunner  # noqa: E402

dev = "cuda:0"
torch.manual_seed(5)
env = bench.make_env(4096, dev, 5)
runner = OnPolicyRunner(env, bench.train_cfg(24), log_dir=None, device=dev)
t0 = time.time()
runner.learn(int(os.environ.get("WARM", 3)), init_at_random_ep_len=True)
torch.cuda.synchronize()
print("warmup s", round(time.time() - t0, 1))
cs, ls = [], []
for _ in range(5):
    runner.learn(1)
    cs.append(runner.last_iteration_stats["collection_time"])
    ls.append(runner.last_iteration_stats["learn_time"])
print(os.environ.get("TAG", "?"), "collection ms", round(1e3 * min(cs), 2), "learn ms", round(1e3 * min(ls), 2))
