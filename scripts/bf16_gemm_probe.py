"""bf16 policy GEMMs (config 5) on MI355X: forward addmm, dX and dW (fp32 output, split-K S row
chunks) for every layer of the actor / lin-vel / critic MLPs at the minibatch row count R.
Env: R (rows, default 49152), TUNE=1 turns TunableOp tuning on in this process (results file under
gpurun_out/).  Prints us per call and TFLOP/s."""
import os

if os.environ.get("TUNE") == "1":
    os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
    os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
    os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", "gpurun_out/bf16_tunable.csv")
import torch
import torch.nn.functional as F

R = int(os.environ.get("R", 49152))
dev = "cuda:0"
bf = torch.bfloat16


def t_us(f, n=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


LAYERS = [(705, 512), (512, 256), (256, 128), (705, 128), (128, 128), (219, 768), (768, 256)]
for k, n in LAYERS:
    x = torch.randn(R, k, device=dev).to(bf)
    W = torch.randn(n, k, device=dev).to(bf)
    b = torch.randn(n, device=dev).to(bf)
    gh = torch.randn(R, n, device=dev).to(bf)
    fl = 2 * R * n * k / 1e6
    tf = t_us(lambda: torch.addmm(b, x, W.t()))
    h = torch.addmm(b, x, W.t())
    te = t_us(lambda: F.elu(h))
    tdx = t_us(lambda: torch.mm(gh, W))
    line = f"{k:4d}->{n:4d}: fwd {tf:6.1f} us {fl / tf:6.0f} TF/s | elu {te:5.1f} | dx {tdx:6.1f} {fl / tdx:6.0f} TF/s | dW"
    tb = t_us(lambda: torch.mm(gh.t(), x))
    line += f" bf16out {tb:6.1f}"
    for S in (1, 2, 4, 8, 16, 32, 64):
        try:
            if S == 1:
                t = t_us(lambda: torch.mm(gh.t(), x, out_dtype=torch.float32))
            else:
                g3, x3 = gh.view(S, R // S, n).transpose(1, 2), x.view(S, R // S, k)
                t = t_us(lambda: torch.bmm(g3, x3, out_dtype=torch.float32))
                t += S * n * k * 4 / 4e6  # chunk-sum read at ~4 TB/s (batched colsum launch)
            line += f" S{S}:{t:6.1f}"
        except RuntimeError as e:
            line += f" S{S}:ERR({str(e)[:40]})"
    print(line, flush=True)
