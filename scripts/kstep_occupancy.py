"""K_step launch time vs env count (timing only, 5 PGS sweeps, random actions x0.5): how the
kernel's time scales from one wave per SIMD group of envs to several dispatch rounds — the
evidence for DESIGN.md §6 "K_step mapping" (a wave's time is its own dependency chain)."""
import json
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

for n in [int(x) for x in os.environ.get("ENVS", "256,512,1024,2048,3072,4096,6144,8192,16384").split(",")]:
    torch.manual_seed(0)
    cfg = XBotLCfg()
    cfg.env.num_envs = n
    env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
    for _ in range(10):
        env.step(torch.randn(n, 12, device="cuda:0") * 0.5)
    torch.cuda.synchronize()
    t = bench.KernelTimer()
    t.enabled = True
    env.kernel_timer = t
    for _ in range(30):
        env.step(torch.randn(n, 12, device="cuda:0") * 0.5)
    torch.cuda.synchronize()
    ms = t.mean_ms("k_step")
    waves = (n + 1) // 2
    print(json.dumps({"envs": n, "waves": waves, "waves_per_simd": round(waves / 1024, 3), "k_step_ms": round(ms, 4),
                      "us_per_1k_envs": round(1e3 * ms / (n / 1024), 2), "rows": round(bench.active_rows(env), 2)}),
          flush=True)
    del env
    torch.cuda.empty_cache()
