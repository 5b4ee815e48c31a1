"""Rollout policy forward: the fused one-launch actor (hg_policy_forward) against the per-layer path
(HG_POLICY_FUSED=0 routes: f32-MFMA / fused-register GEMM kernels + the skinny output layer) at
the rollout's row counts, on the env's strided observation view.  us per call (HIP events)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402

from humanoid.algo.ppo import ActorCritic, hg_mlp  # noqa: E402

ITERS = int(os.environ.get("ITERS", 50))
ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128]).cuda()


def timeit(fn):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / ITERS


for rows in (4096, 8192, 2048):
    buf = torch.randn(rows * 1880 + 705, device="cuda:0")
    obs = buf[141:141 + rows * 1880].view(rows, 1880)[:, :705]
    rec = {"rows": rows}
    with torch.inference_mode():
        for fused in (False, True):
            hg_mlp.POLICY_FUSED = fused
            rec["fused_us" if fused else "layers_us"] = round(timeit(lambda: ac._mlp(ac.actor, obs)), 2)
        params = [p.detach() for p in hg_mlp._params(ac.actor)]
        imgs = hg_mlp.x6_images([(params[0], 0, 512, 705), (params[2], 0, 256, 512), (params[4], 0, 128, 256)],
                                obs.device)
        rec["images_us"] = round(timeit(lambda: hg_mlp.x6_images(
            [(params[0], 0, 512, 705), (params[2], 0, 256, 512), (params[4], 0, 128, 256)], obs.device)), 2)
    print(json.dumps(rec), flush=True)
