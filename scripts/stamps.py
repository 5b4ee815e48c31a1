"""Per-phase cycle breakdown of K_step v2 from the diagnostic build (libhgsim_stamps.so)."""
import ctypes, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HG_LIB"] = os.path.join(REPO, "humanoid-gym-with-comments_amd", "csrc", "libhgsim_stamps.so")
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch
import bench
from humanoid import _native as N
env = bench.make_env(int(os.environ.get("ENVS", 4096)), "cuda:0", 5)
L = N.lib()
L.hg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 32)()
for _ in range(20):
    env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
torch.cuda.synchronize()
L.hg_debug_stamps(buf, 1)
t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
t0.record()
for _ in range(20):
    env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
t1.record(); torch.cuda.synchronize()
L.hg_debug_stamps(buf, 0)
names = ["prologue/loop-top", "A1 torques", "A2/A3 FK+RNEA fwd", "A4 per-body", "A5 backward chain",
         "A6/A7 mass matrix", "A8 Cholesky", "A9 M^-1", "A10 nu*", "A11 detect+alloc", "A12 J,Y", "A13 W",
         "A14 PGS", "A15 nu, forces", "A16 integrate", "epilogue FK"]
tot = sum(buf[k] for k in range(16))
out = {n: round(buf[k] / tot * 100, 2) for k, n in enumerate(names)}
print(json.dumps({"ms_per_20_steps": t0.elapsed_time(t1), "rows": bench.active_rows(env), "phase_pct": out}, indent=1))
