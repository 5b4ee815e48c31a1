"""Diagnose K_step vs reference-simulator disagreements on the heightfield: several seeded
30-step histories, then one compared step; prints, for each env/DOF beyond the parity test's
tolerance, the GPU, CPU-f32 and CPU-f64 values."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "humanoid-gym-with-comments_amd")]
import test_gpu_parity as T  # noqa: E402
import pipeline_ref as PR  # noqa: E402

env = T._make_env(T.N_ENVS, "v2", terrain__mesh_type="heightfield", terrain__measure_heights=True)
g = lambda t: t.detach().cpu().numpy()  # noqa: E731
for seed in range(int(os.environ.get("SEEDS", 8))):
    torch.manual_seed(seed)
    for _ in range(30):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.3)
    S, _, _ = T.snapshot(env)
    cfg = T._oracle_cfg(env)
    actions = torch.randn(env.num_envs, 12, device="cuda:0") * 0.5
    a_ref = PR.preprocess_actions(cfg, actions.cpu().numpy(), S["actions"], 91)
    T._step_only(env, actions, 91)
    r64, r32 = T._ref_sim(env, S, "f64"), T._ref_sim(env, S, "f32")
    r64.step(a_ref)
    r32.step(a_ref)
    nbad = 0
    for name, gpu, a64, a32 in (("q", g(env.dof_pos), r64.q, r32.q), ("qd", g(env.dof_vel), r64.qd, r32.qd),
                                ("root", g(env.root_states), r64.root, r32.root)):
        tol = 20 * np.abs(a32 - a64) + 1e-3 * (1 + np.abs(a64))
        bad = np.argwhere(np.abs(gpu - a64) > tol)
        nbad += len(bad)
        for e, j in bad[:6]:
            print(f"seed {seed} {name}[{e},{j}] gpu {gpu[e, j]:+.5f} f32 {a32[e, j]:+.5f} f64 {a64[e, j]:+.5f} "
                  f"root_z {S['root_states'][e, 2]:.3f} origin_z {S['env_origins'][e, 2]:.3f} "
                  f"cf_feet {np.linalg.norm(S['contact_forces'][e, [6, 12]], axis=-1).round(1)}")
    print(f"seed {seed}: {nbad} beyond tolerance", flush=True)
