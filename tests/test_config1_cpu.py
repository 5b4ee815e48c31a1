"""BASELINE config 1 (XBot-L flat terrain, 4 envs, CPU sim + CPU PPO, 1 iteration): the plumbing
run on the host through the oracle port (C reference physics, numpy env logic, torch-CPU PPO) —
the same code bench.py times as its cpu_baseline.  The product (HIP) path has no CPU mode."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config1_one_iteration_on_cpu():
    import torch
    sys.path.insert(0, REPO)
    import bench
    n_threads = torch.get_num_threads()
    try:
        v, threads, dt = bench.cpu_baseline(4, 24, threads=1)
    finally:
        torch.set_num_threads(n_threads)
    assert v > 0 and threads == 1 and dt > 0
