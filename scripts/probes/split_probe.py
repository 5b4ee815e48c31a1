"""Collection-step overlap probe: one 4096-env instance stepping [actor inference -> env.step] on
one stream, against two 2048-env shards (global env ids 0.. and 2048.., bit-identical to the one
instance) each on its own stream, so one shard's K_step can run beside the other shard's post /
stacking / policy kernels.  Prints the per-step time of both forms (HIP events, 24-step rollouts)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from humanoid.algo.ppo import ActorCritic  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
dev = "cuda:0"
N = int(os.environ.get("ENVS", 4096))
T = 24
torch.manual_seed(0)
ac = ActorCritic(705, 219, 12, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
                 base_lin_vel_hidden_dims=[128, 128]).to(dev)


def chain(env, obs):
    with torch.inference_mode():
        mu = ac._mlp(ac.actor, obs)
        a = mu + 0.1 * torch.randn_like(mu)
        return env.step(a)[0]


def run_single(reps):
    env = bench.make_env(N, dev, seed=5)
    obs = env.get_observations()
    for _ in range(T):
        obs = chain(env, obs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps * T):
        obs = chain(env, obs)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * T)


def run_split(reps, k=2):
    n = N // k
    envs = [bench.make_env(n, dev, seed=5, env_offset=i * n, num_envs_total=N) for i in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    main = torch.cuda.current_stream()
    obs = [e.get_observations() for e in envs]
    for s in streams:
        s.wait_stream(main)

    def one_step():
        for i in range(k):
            with torch.cuda.stream(streams[i]):
                obs[i] = chain(envs[i], obs[i])

    for _ in range(T):
        one_step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in streams:
        s.wait_stream(main)
    for _ in range(reps * T):
        one_step()
    for s in streams:
        main.wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * T)


reps = int(os.environ.get("REPS", 5))
print(f"single {N}: {run_single(reps) * 1e3:.1f} us/step", flush=True)
for k in (2, 4):
    print(f"split {k}x{N // k} on {k} streams: {run_split(reps, k) * 1e3:.1f} us/step", flush=True)
