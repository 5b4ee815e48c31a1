"""Training entry point (humanoid/scripts/train.py of the reference).

    python -m humanoid.scripts.train --task humanoid_ppo --run_name v1 --headless --num_envs 4096

Data parallel on one node (one process per GPU, RCCL over xGMI):

    python -m torch.distributed.run --standalone --nproc-per-node 8 -m humanoid.scripts.train --task humanoid_ppo

Each rank simulates ``num_envs`` environments on its own GPU: rank r holds the global envs
[r * num_envs, (r + 1) * num_envs) of world * num_envs, with one seed for every rank (the env
draws and the action noise are keyed by the global env id); PPO broadcasts the initial parameters, all-reduces gradients and the KL mean per minibatch and
the advantage statistics per iteration (humanoid/algo/ppo/ppo.py).  Only rank 0 writes logs and
checkpoints.
"""
import os

import torch
import torch.distributed as dist

from humanoid.envs import *  # noqa: F401,F403  (registers the tasks)
from humanoid.utils import get_args, task_registry


def _init_distributed(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    args.sim_device = args.rl_device = f"cuda:{local}"
    return dist.get_rank(), world


def train(args):
    rank, world = _init_distributed(args)
    env_cfg, train_cfg = task_registry.get_cfgs(name=args.task)
    if args.seed is None:
        args.seed = train_cfg.seed
    args.seed = int(args.seed)
    if args.num_envs is not None:
        env_cfg.env.num_envs = args.num_envs
    env_cfg.env.env_offset = rank * env_cfg.env.num_envs
    env_cfg.env.num_envs_total = world * env_cfg.env.num_envs
    env, env_cfg = task_registry.make_env(name=args.task, args=args, env_cfg=env_cfg)
    ppo_runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args,
                                                          log_root="default" if rank == 0 else None)
    ppo_runner.learn(num_learning_iterations=train_cfg.runner.max_iterations, init_at_random_ep_len=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    args = get_args()
    print(args)
    train(args)
