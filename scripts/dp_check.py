"""Data-parallel rehearsal on ONE GPU: N ranks (torchrun) share cuda:0 and talk over gloo.

Exercises the multi-GPU training path end to end on the device — per-rank env shards, parameter
broadcast, the captured update graphs with the gradient/KL all-reduces between them, global
advantage statistics — and checks that every rank ends with bit-identical parameters.  (RCCL
cannot put two ranks on one device, so the exchange runs over gloo here; bench.py --gpus N uses
backend "nccl" = RCCL with one GPU per rank.)

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 scripts/dp_check.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    dist.init_process_group(os.environ.get("DP_BACKEND", "gloo"))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = "cuda:0"
    torch.cuda.set_device(0)
    torch.manual_seed(5)
    from humanoid.algo.ppo import OnPolicyRunner
    env = bench.make_env(256, dev, seed=5, env_offset=rank * 256, num_envs_total=world * 256)  # global env shards
    tcfg = bench.train_cfg(8)
    runner = OnPolicyRunner(env, tcfg, log_dir=None, device=dev)
    runner.learn(3, init_at_random_ep_len=True)   # eager warm-up, capture, replay
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in runner.alg.actor_critic.parameters()]).cpu().double()
    outs = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(outs, flat)
    lr = torch.tensor([runner.alg.learning_rate], dtype=torch.float64)
    lrs = [torch.zeros_like(lr) for _ in range(world)]
    dist.all_gather(lrs, lr)
    ok = all(torch.equal(outs[0], o) for o in outs) and all(torch.equal(lrs[0], x) for x in lrs)
    st = runner.last_iteration_stats
    if rank == 0:
        print(f"dp_check world={world} params_identical={ok} lr={lr.item():.3e} "
              f"value_loss={st['value_loss']:.4f} finite={bool(torch.isfinite(flat).all())}", flush=True)
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
