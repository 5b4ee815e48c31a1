"""Where does one PPO iteration spend its time?  torch.profiler over 2 iterations of the bench
workload; prints the top device kernels and the GPU-busy fraction of the wall clock."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
from humanoid.algo.ppo import OnPolicyRunner  # noqa: E402

dev = "cuda:0"
torch.manual_seed(5)
env = bench.make_env(int(os.environ.get("ENVS", 4096)), dev, 5)
runner = OnPolicyRunner(env, bench.train_cfg(24), log_dir=None, device=dev)
runner.learn(2, init_at_random_ep_len=True)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    t0 = time.time()
    runner.learn(2)
    torch.cuda.synchronize()
    wall = time.time() - t0
print("wall per iteration ms", wall / 2 * 1e3, runner.last_iteration_stats)
ka = prof.key_averages()
dev_total = sum(e.self_device_time_total for e in ka) / 1e3 / 2
print("device busy per iteration ms", dev_total)
print(ka.table(sort_by="self_device_time_total", row_limit=35, max_name_column_width=70))
print(ka.table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=70))
