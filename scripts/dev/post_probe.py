"""K_post phase timestamps (development tool; never part of the product library).

Builds a variant library from a patched COPY of csrc/hg_envlogic.hip in which thread 0 of every
block of k_post_step stores s_memrealtime (100 MHz) at each phase boundary into a device array,
read back by an extra export.  Usage:
    python scripts/dev/post_probe.py build     # here: writes build/probe/libhgsim.so
    python scripts/dev/post_probe.py run       # on the GPU
"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "humanoid-gym-with-comments_amd")
OUT = os.environ.get("PROBE_DIR") or os.path.join(REPO, "build", "probe")
NB, NM = 1024, 8

# (label, anchor): the probe store goes right BEFORE the anchor line
MARKS = [
    ("start", "  // ---------------- L: staging loads"),
    ("loaded", "  const int64_t ep = (int64_t)__float_as_int(X(X_EP));"),
    ("derived", "  // ---------------- T: the reward terms"),
    ("terms", "  // ---------------- R: reset_idx"),
    ("reset", "  // ---------------- O: observation frames"),
    ("frames", "  // the frames, row-major"),
    ("end", "__global__ void __launch_bounds__(256) k_stack_stats"),
]


def variant_source():
    s = open(os.path.join(PKG, "csrc", "hg_envlogic.hip")).read()
    head = ("__device__ unsigned long long hg_probe[%d * %d];\n"
            "#define HG_PROBE(k) do { if (threadIdx.x == 0) hg_probe[blockIdx.x * %d + (k)] = "
            "__builtin_amdgcn_s_memrealtime(); } while (0)\n" % (NB, NM, NM))
    i = s.index("// K_post for a policy step")
    s = s[:i] + head + s[i:]
    for k, (_, anchor) in enumerate(MARKS):
        if anchor.startswith("__global__"):
            # the kernel's closing brace precedes the next kernel: probe before the final "}\n"
            j = s.index("// history stacking: dst[e]")
            end = s.rindex("\n}\n", 0, j)
            s = s[:end] + "\n  HG_PROBE(%d);" % k + s[end:]
        else:
            j = s.index(anchor)
            s = s[:j] + "  HG_PROBE(%d);\n" % k + s[j:]
    s += ('\nextern "C" int hg_probe_read(unsigned long long* host) {\n'
          '  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(hg_probe), sizeof(hg_probe));\n}\n'
          'extern "C" int hg_probe_clear() {\n'
          '  static unsigned long long z[%d * %d];\n'
          '  return (int)hipMemcpyToSymbol(HIP_SYMBOL(hg_probe), z, sizeof(z));\n}\n' % (NB, NM))
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    objs = [f for f in os.listdir(os.path.join(PKG, "csrc")) if f.endswith(".o") and f != "hg_envlogic.o"]
    src = os.path.join(PKG, "csrc", "_probe_envlogic.hip")
    with open(src, "w") as f:
        f.write(variant_source())
    try:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                        "-DHG_POST_PEB=" + os.environ.get("PEB", "16"), "-c", src, "-o", os.path.join(OUT, "hg_envlogic.o")], check=True)
    finally:
        os.remove(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(OUT, "libhgsim.so"), os.path.join(OUT, "hg_envlogic.o")] +
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
    lib.hg_probe_read.argtypes = [ctypes.c_void_p]
    buf = np.zeros(NB * NM, np.uint64)
    rows = []
    for it in range(60):
        env.step(torch.randn(env.num_envs, 12, device="cuda:0") * 0.5)
        torch.cuda.synchronize()
        if it < 10:
            continue
        assert lib.hg_probe_read(buf.ctypes.data) == 0
        assert lib.hg_probe_clear() == 0
        t = buf.reshape(NB, NM)[:, :len(MARKS)].astype(np.int64)
        t = t[t[:, 0] != 0]  # the launched blocks (buffer zeroed below after each read)
        t0 = t[:, 0].min()
        rel = (t - t0) * 10 / 1000.0  # us
        nres = int(env.reset_buf.sum().item())
        rows.append((nres, rel))
    for nres, rel in rows[:12]:
        seg = np.diff(rel, axis=1)
        print(f"resets {nres:4d}  start spread {rel[:, 0].max():6.2f}us  end max {rel[:, -1].max():6.2f}us  "
              "phase means " + " ".join(f"{m[0]}={v:.2f}" for m, v in zip(MARKS[1:], seg.mean(0))) +
              "  phase max " + " ".join(f"{v:.2f}" for v in seg.max(0)), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
