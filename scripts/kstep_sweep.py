"""K_step launch time vs solver sweeps (timing only): isolates the PGS share of the kernel."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from humanoid.envs import XBotLCfg  # noqa: E402
from humanoid.envs.custom.humanoid_env import XBotLFreeEnv  # noqa: E402
from humanoid.utils.helpers import SimParams  # noqa: E402

for it in [int(x) for x in os.environ.get("ITERS", "1,2,5,10,20").split(",")]:
    cfg = XBotLCfg()
    cfg.env.num_envs = int(os.environ.get("ENVS", 4096))
    cfg.sim.hg.pgs_iterations = it
    env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
    for _ in range(10):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
    torch.cuda.synchronize()
    t = bench.KernelTimer()
    t.enabled = True
    env.kernel_timer = t
    for _ in range(30):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
    torch.cuda.synchronize()
    print(f"pgs_iterations={cfg.sim.hg.pgs_iterations} k_step {t.mean_ms('k_step'):.4f} ms rows {bench.active_rows(env):.2f}",
          flush=True)
    del env
