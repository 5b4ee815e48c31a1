"""Host (Python) time to queue one rollout of the collection loop vs the GPU time it takes:
if the host needs about as long as the GPU, the GPU starves whenever the queue runs dry (the
first iteration of every learn() call).  Also times PPO.update queueing."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from humanoid.algo.ppo import OnPolicyRunner  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
env = bench.make_env(4096, "cuda:0", seed=5)
runner = OnPolicyRunner(env, bench.train_cfg(24, "fp32", "fp32"), log_dir=None, device="cuda:0")
runner.learn(3, init_at_random_ep_len=True)
alg = runner.alg
obs = env.get_observations()
critic = env.get_privileged_observations()
for rep in range(3):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.inference_mode():
        t0 = time.perf_counter()
        e0.record()
        for _ in range(24):
            a = alg.act(obs, critic)
            obs, critic, rew, dones, infos = env.step(a)
            alg.process_env_step(rew, dones, infos)
        e1.record()
        t1 = time.perf_counter()
        alg.compute_returns(critic)
        t2 = time.perf_counter()
    out = alg.update(sync=False)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"host: rollout {1e3 * (t1 - t0):.2f} ms, returns {1e3 * (t2 - t1):.2f} ms, update {1e3 * (t3 - t2):.2f} ms"
          f" | gpu rollout {e0.elapsed_time(e1):.2f} ms | wall to idle {1e3 * (t4 - t0):.2f} ms", flush=True)
# fixed cost per learn() call: wall time of learn(k) for several k
for k in (1, 2, 5, 10, 10, 20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.learn(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = runner.last_iteration_stats
    print(f"learn({k}): {1e3 * dt:.1f} ms = {1e3 * dt / k:.2f} ms/it; last it events {1e3 * (st['collection_time'] + st['learn_time']):.2f} ms",
          flush=True)
