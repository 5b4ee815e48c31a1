"""K_step A/B timing across variant builds (development tool; never part of the product library).

    python scripts/dev/kstep_variants.py build NAME [SRC]   # here: compile SRC (default: the current
                                                             # csrc/hg_physics.hip) into build/var/NAME/
    python scripts/dev/kstep_variants.py run NAME...         # GPU: time each variant, interleaved, twice
Timing is scripts/kstep_sweep.py (4096 envs, 5 PGS sweeps, random actions) under HG_LIB."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "humanoid-gym-with-comments_amd")
OUT = os.path.join(REPO, "build", "var")


def build(name, src=None):
    src = src or os.path.join(PKG, "csrc", "hg_physics.hip")
    d = os.path.join(OUT, name)
    os.makedirs(d, exist_ok=True)
    tmp = os.path.join(PKG, "csrc", f"_var_{name}.hip")
    with open(src) as f, open(tmp, "w") as g:
        g.write(f.read())
    objs = [os.path.join(PKG, "csrc", f) for f in sorted(os.listdir(os.path.join(PKG, "csrc")))
            if f.endswith(".o") and f != "hg_physics.o"]
    try:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fno-slp-vectorize",
                        "-c", tmp, "-o", os.path.join(d, "hg_physics.o")], check=True)
    finally:
        os.remove(tmp)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(d, "libhgsim.so"),
                    os.path.join(d, "hg_physics.o")] + objs, check=True)
    print("built", name)


def run(names):
    for rep in range(2):
        for name in names:
            env = dict(os.environ, ITERS="5", HG_LIB=os.path.join(OUT, name, "libhgsim.so"))
            r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "kstep_sweep.py")], env=env,
                               capture_output=True, text=True, timeout=240)
            line = [x for x in r.stdout.splitlines() if "k_step" in x]
            print(rep, name, line[-1] if line else r.stderr[-400:], flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        run(sys.argv[2:])
