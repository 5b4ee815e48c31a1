"""K_step per-phase time (development tool; never part of the product library).

Builds a variant library from a patched COPY of csrc/hg_physics.hip in which every wave accumulates
s_memtime deltas per phase of the substep (summed over the 10 substeps) and thread 0 of the first
NB blocks stores them at the end; run() prints the mean share of each phase.  The timer reads add
an s_waitcnt at each phase boundary, so shares are approximate.
    python scripts/dev/kstep_probe.py build     # here: writes build/kprobe/libhgsim.so
    python scripts/dev/kstep_probe.py run       # on the GPU
"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "humanoid-gym-with-comments_amd")
OUT = os.environ.get("PROBE_DIR") or os.path.join(REPO, "build", "kprobe")
NB, NM = 2048, 16

# (label of the phase that ENDS at the anchor, anchor): the mark goes right before the anchor line
MARKS = [
    ("prologue", "  for (int sub = 0; sub < decimation; sub++) {"),
    ("A1 torques", "    // ---- A2..A5:"),
    ("A2-5 kin+rnea", "    // base totals (lane 0)"),
    ("base totals", "    // ---- A6/A7:"),
    ("A6/7 M", "    // ---- A8:"),
    ("A8 cholesky", "    // ---- A9:"),
    ("A9 detect", "    const int nrows = E.nrows;"),
    ("A10 J, z", "    // ---- A11:"),
    ("A11 mfma W", "    // ---- A12:"),
    ("A12 group consts", "    // ---- A13:"),
    ("A13 pgs", "      // ---- A14:"),
    ("A14 backsub+cf", "    // ---- A16:"),
    ("A16 integrate", "    // a non-finite env keeps stepping"),
    ("epilogue", "  if (!valid) return;"),
]


def variant_source():
    s = open(os.path.join(PKG, "csrc", "hg_physics.hip")).read()
    head = ("__device__ unsigned long long hg_kprobe[%d * %d];\n"
            "#define HG_MARK(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
            "hg_acc[k] += t_ - hg_t; hg_t = t_; } while (0)\n" % (NB, NM))
    i = s.index("// FIXED = asset.fix_base_link")
    s = s[:i] + head + s[i:]
    j = s.index("  __shared__ EnvSh shm[2];")
    s = s[:j] + "  unsigned long long hg_acc[%d] = {0};\n  unsigned long long hg_t = __builtin_amdgcn_s_memtime();\n" % NM + s[j:]
    for k, (_, anchor) in enumerate(MARKS):
        j = s.index(anchor)
        mark = "  HG_MARK(%d);\n" % k
        if anchor == "  if (!valid) return;":
            mark += ("  if (threadIdx.x == 0 && blockIdx.x < %d) {\n#pragma unroll\n    for (int k = 0; k < %d; k++) "
                     "hg_kprobe[blockIdx.x * %d + k] = hg_acc[k];\n  }\n" % (NB, NM, NM))
        s = s[:j] + mark + s[j:]
    s += ('\nextern "C" int hg_kprobe_read(unsigned long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(hg_kprobe), sizeof(hg_kprobe));\n}\n')
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    objs = [f for f in os.listdir(os.path.join(PKG, "csrc")) if f.endswith(".o") and f != "hg_physics.o"]
    src = os.path.join(PKG, "csrc", "_kprobe_physics.hip")
    with open(src, "w") as f:
        f.write(variant_source())
    try:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fno-slp-vectorize",
                        "-c", src, "-o", os.path.join(OUT, "hg_physics.o")], check=True)
    finally:
        os.remove(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(OUT, "libhgsim.so"), os.path.join(OUT, "hg_physics.o")] +
                   [os.path.join(PKG, "csrc", o) for o in objs], check=True)
    print("built", flush=True)


def run():
    os.environ["HG_LIB"] = os.path.join(OUT, "libhgsim.so")
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    from humanoid import _native
    from humanoid.envs import XBotLCfg
    from humanoid.envs.custom.humanoid_env import XBotLFreeEnv
    from humanoid.utils.helpers import SimParams
    cfg = XBotLCfg()
    cfg.env.num_envs = int(os.environ.get("ENVS", 4096))
    env = XBotLFreeEnv(cfg, SimParams(), "hg_sim", "cuda:0", True)
    lib = _native.lib()
    lib.hg_kprobe_read.argtypes = [ctypes.c_void_p]
    buf = np.zeros(NB * NM, np.uint64)
    acc = np.zeros(len(MARKS))
    n = 0
    for it in range(40):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
        torch.cuda.synchronize()
        if it < 10:
            continue
        assert lib.hg_kprobe_read(buf.ctypes.data) == 0
        t = buf.reshape(NB, NM)[:, :len(MARKS)].astype(np.float64)
        nb = min(NB, (env.num_envs + 1) // 2)
        acc += t[:nb].mean(0)
        n += 1
    acc /= n
    tot = acc.sum()
    print(f"envs {env.num_envs}: mean wave clocks per launch {tot:.0f}")
    for (name, _), v in zip(MARKS, acc):
        print(f"  {name:18s} {v:10.0f}  {100 * v / tot:5.1f} %")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
