"""K_step A/B bit comparison (development tool): runs 20 env steps of 4096 envs with random actions
under the library named by HG_LIB and saves the physics state to OUT (npz); `compare A B` reports
the max abs difference per field.  Usage: HG_LIB=... OUT=a.npz python scripts/dev/kstep_bits.py run"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import numpy as np  # noqa: E402


def run():
    import torch
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    cfg = XBotLCfg()
    cfg.env.num_envs = int(os.environ.get("ENVS", 4096))
    env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
    g = torch.Generator(device="cuda:0").manual_seed(7)
    for _ in range(int(os.environ.get("STEPS", 20))):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0", generator=g) * 0.5)
    torch.cuda.synchronize()
    out = {k: getattr(env, k).detach().cpu().numpy() for k in
           ("root_states", "dof_pos", "dof_vel", "torques", "contact_forces", "rigid_state")}
    np.savez(os.environ["OUT"], **out)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for k in A.files:
        d = np.abs(A[k].astype(np.float64) - B[k])
        print(f"{k:16s} max|d| {d.max():.3e}  differing {int((d > 0).sum())} / {d.size}")


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else compare(sys.argv[2], sys.argv[3])
