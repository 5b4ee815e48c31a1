"""K_step phase costs by repetition (development tool; never part of the product library).

Builds variant libraries from a patched COPY of csrc/hg_physics.hip in which one idempotent phase
of the substep runs twice, and times each with scripts/kstep_sweep.py (HG_LIB): the launch-time
delta against the unpatched build is that phase's cost.  Usage (GPU box, after building here):
    python scripts/dev/phase_cost.py build     # here: writes build/phase_*/libhgsim.so
    python scripts/dev/phase_cost.py run       # on the GPU
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "humanoid-gym-with-comments_amd")
OUT = os.path.join(REPO, "build", "phase")

# (name, start marker, end marker): the code between the markers is emitted twice
PHASES = {
    "kin": ("    // ---- A2..A5:", "    // base totals (lane 0)"),
    "mchol": ("    // ---- A6/A7:", "    // ---- A9:"),
    "detect": ("    // ---- A9:", "    const int nrows = E.nrows;"),
    "jz": ("    // ---- A10:", "    // the group constants below read"),
    "grpc": ("    // ---- A12:", "    // ---- A13:"),
}


def variant_source(name):
    s = open(os.path.join(PKG, "csrc", "hg_physics.hip")).read()
    if name == "base":
        return s
    a, b = PHASES[name]
    i, j = s.index(a), s.index(b)
    block = s[i:j]
    if name == "jz":  # the block declares z/v0 in the enclosing scope: repeat the inner body only
        block2 = block.replace("float z[18];\n    float v0 = 0.f;\n", "v0 = 0.f;\n")
        return s[:i] + block + "    __syncthreads();\n" + block2.replace("    // ---- A10:", "    // ---- A10 (repeat):", 1) + s[j:]
    if name == "kin":
        body = block.replace("const KinLane K", "KinLane K", 1)
        return s[:i] + "    {\n" + body + "    }\n    __syncthreads();\n" + block + s[j:]
    if name == "grpc":
        return s[:i] + block + "    __syncthreads();\n" + block + s[j:]
    return s[:i] + block + "    __syncthreads();\n" + block + s[j:]


def build():
    objs = [f for f in os.listdir(os.path.join(PKG, "csrc")) if f.endswith(".o") and f != "hg_physics.o"]
    for name in ["base"] + list(PHASES):
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        src = os.path.join(PKG, "csrc", f"_phase_{name}.hip")
        with open(src, "w") as f:
            f.write(variant_source(name))
        try:
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fno-slp-vectorize",
                            "-c", src, "-o", os.path.join(d, "hg_physics.o")], check=True)
        finally:
            os.remove(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libhgsim.so"), os.path.join(d, "hg_physics.o")] +
                       [os.path.join(PKG, "csrc", o) for o in objs], check=True)
        print("built", name, flush=True)


def run():
    env = dict(os.environ, ITERS="5")
    for name in ["base"] + list(PHASES):
        env["HG_LIB"] = os.path.join(OUT, name, "libhgsim.so")
        r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "kstep_sweep.py")], env=env,
                           capture_output=True, text=True, timeout=240)
        line = [x for x in r.stdout.splitlines() if "k_step" in x]
        print(name, line[-1] if line else r.stderr[-400:], flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
