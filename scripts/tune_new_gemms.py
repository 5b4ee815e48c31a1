"""Add TunableOp results for GEMM shapes missing from the committed MI355X table (tunes only the
shapes run here; every existing entry is kept).  Writes gpurun_out/tunableop_mi355x_f32.csv.
Shapes: the split-K weight-gradient bmms of hg_mlp._DW_SPLIT at the 24576-row minibatch."""
import os
import sys
import shutil

import torch
import torch.cuda.tunable as tun

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
from humanoid.algo.ppo.hg_mlp import _DW_SPLIT  # noqa: E402

src = os.path.join(REPO, "humanoid-gym-with-comments_amd", "tuning", "tunableop_mi355x_f32.csv")
out = os.path.join(REPO, "gpurun_out", "tunableop_mi355x_f32.csv")
os.makedirs(os.path.dirname(out), exist_ok=True)
shutil.copy(src, out)
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(out, False)
assert tun.read_file(out)
R = 24576
for (n, k), S in _DW_SPLIT.items():
    gh = torch.randn(R, n, device="cuda:0")
    x = torch.randn(R, k, device="cuda:0")
    torch.bmm(gh.view(S, R // S, n).transpose(1, 2), x.view(S, R // S, k))
    torch.cuda.synchronize()
    print("tuned", n, k, S, flush=True)
# TunableOp writes the merged table to `out` at process exit
print(open(out).read().count("\n"), "lines")
