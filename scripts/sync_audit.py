"""List the host<->device synchronisations inside one PPO iteration (torch sync-debug mode)."""
import os
import sys
import warnings
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from humanoid.algo.ppo import OnPolicyRunner  # noqa: E402

dev = "cuda:0"
env = bench.make_env(1024, dev, 5)
runner = OnPolicyRunner(env, bench.train_cfg(24), log_dir=None, device=dev)
runner.learn(1, init_at_random_ep_len=True)
torch.cuda.synchronize()
seen = {}


def hook(message, category, filename, lineno, file=None, line=None):
    st = "".join(traceback.format_stack(limit=8)[:-1])
    seen[st] = seen.get(st, 0) + 1


warnings.showwarning = hook
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
runner.learn(1)
torch.cuda.set_sync_debug_mode(0)
for st, n in sorted(seen.items(), key=lambda x: -x[1]):
    print("=" * 20, n, "times")
    print(st)
