"""bench.py's multi-GPU launcher on the CPU: `bench.py --gpus N` with no
external launcher starts N ranks itself and reports them, and a rank count that disagrees with
--gpus is refused instead of being reported as N GPUs."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=240)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--dist-backend", "gloo", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == n
    assert d["config"]["parallelism"] == f"dp{n}"
    # max over ranks: rank n-1 sleeps the longest (10 ms x n)
    assert d["ms_per_step"] >= 10.0 * n - 1.0


def test_bench_refuses_mismatched_world_size():
    r = _run(["--gpus", "4", "--launch-check"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_bench_single_rank_default():
    r = _run(["--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_line(r.stdout)["n_gpus"] == 1
