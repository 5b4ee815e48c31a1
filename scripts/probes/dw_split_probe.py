"""Split-K factor of the hipBLASLt weight gradients (hg_mlp._DW_SPLIT) timed WITH the chunk sum
(the batched column-sum launch), per weight shape at the 24576-row minibatch: the factors were
first chosen on the bmm alone.  One JSON line per shape."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "humanoid-gym-with-comments_amd"))
import torch  # noqa: E402

from humanoid.algo.ppo import hg_mlp  # noqa: E402
from humanoid.utils.blas_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
dev = "cuda:0"
ITERS = int(os.environ.get("ITERS", 30))
SHAPES = [(512, 705), (256, 512), (128, 256), (768, 219), (256, 768), (128, 705), (128, 128)]


def timeit(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / ITERS


rows = 24576
for n, k in SHAPES:
    gh = torch.randn(rows, n, device=dev)
    x = torch.randn(rows, k, device=dev)
    red = hg_mlp._Reductions()
    rec = {"n": n, "k": k, "current_S": hg_mlp._DW_SPLIT.get((n, k), 1)}
    keep = dict(hg_mlp._DW_SPLIT)
    for S in (1, 2, 4, 8, 16, 32, 64):
        hg_mlp._DW_SPLIT[(n, k)] = S

        def path():
            hg_mlp._weight_grad(gh, x, red)
            red.launch(dev)

        rec[f"S{S}_us"] = round(timeit(path), 2)
    hg_mlp._DW_SPLIT.clear()
    hg_mlp._DW_SPLIT.update(keep)
    print(json.dumps(rec), flush=True)
