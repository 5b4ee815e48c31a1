"""Pre-tuned GEMM selection for the PPO MLPs on MI355X (PyTorch TunableOp).

The policy/critic GEMMs (M = 4096 rollout rows or 24576 minibatch rows, K/N = 705, 219, 768,
512, 256, 128, 12, 3, 1) are fp32.  hipBLASLt's default heuristic picks tiles that reach
~50 TFLOP/s on the large ones; TunableOp benchmarks every hipBLASLt and rocBLAS solution once per
shape and keeps the fastest (~110-130 TFLOP/s for the 24576 x 705 x 512 family).  The table in
``tuning/tunableop_mi355x_f32.csv`` was produced on an MI355X with scripts/blas_probe.sh; loading
it costs nothing at run time and no tuning happens inside timed regions or graph capture.
Validators in the file (PyTorch / HIP / hipBLASLt versions, gfx950) make TunableOp ignore it on a
different stack.
"""
import os

DEFAULT_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                             "tuning", "tunableop_mi355x_f32.csv")


def use_tuned_gemms(path=DEFAULT_TABLE):
    """Enable TunableOp in lookup-only mode with the committed MI355X table.  Returns True when the
    table was loaded."""
    import torch
    import torch.cuda.tunable as tun
    if not torch.cuda.is_available() or not os.path.exists(path):
        return False
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    # anything TunableOp would persist goes to a scratch file, never next to the caller's cwd
    import tempfile
    tun.set_filename(os.path.join(tempfile.gettempdir(), "hg_tunableop_results.csv"), True)
    return bool(tun.read_file(path))
