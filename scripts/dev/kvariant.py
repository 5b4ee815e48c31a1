"""K_step A/B variants (development tool; never part of the product library).

Each variant is a list of (old, new) source replacements applied to a COPY of
csrc/hg_physics.hip; the variant's object is linked with the in-tree objects of the other sources
into build/kvar/<name>/libhgsim.so.  `run` times K_step of every built variant with
scripts/kstep_sweep.py (HG_LIB points the package at the variant library), in one process per
variant, and prints one line each.
    python scripts/dev/kvariant.py build [name ...]   # here
    python scripts/dev/kvariant.py run [name ...]     # on the GPU box
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "humanoid-gym-with-comments_amd")
OUT = os.path.join(REPO, "build", "kvar")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fno-slp-vectorize"]

VARIANTS = {
    "base": [],
    "no_round2": [("const int rounds = nitems > 32 ? 2 : 1;", "const int rounds = 1;")],
}


def build(names):
    src = open(os.path.join(PKG, "csrc", "hg_physics.hip")).read()
    others = [os.path.join(PKG, "csrc", f) for f in sorted(os.listdir(os.path.join(PKG, "csrc")))
              if f.endswith(".o") and f != "hg_physics.o"]
    for name in names:
        s = src
        for old, new in VARIANTS[name]:
            assert old in s, (name, old)
            s = s.replace(old, new)
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        hip = os.path.join(PKG, "csrc", f"_kvar_{name}.hip")   # next to hg_common.h
        open(hip, "w").write(s)
        try:
            r = subprocess.run([HIPCC] + FLAGS + ["-c", hip, "-o", os.path.join(d, "hg_physics.o"),
                                                  "-Rpass-analysis=kernel-resource-usage"],
                               capture_output=True, text=True)
        finally:
            os.remove(hip)
        if r.returncode:
            raise SystemExit(r.stderr[-3000:])
        use = re.findall(r"k_stepILb0.*?VGPRs: (\d+).*?ScratchSize \[bytes/lane\]: (\d+)", r.stderr, re.S)
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(d, "libhgsim.so"),
                        os.path.join(d, "hg_physics.o")] + others, check=True)
        print(f"built {name}: VGPRs / scratch {use[:1]}")


def run(names):
    for name in names:
        lib = os.path.join(OUT, name, "libhgsim.so")
        env = dict(os.environ, HG_LIB=lib, ITERS=os.environ.get("ITERS", "5"))
        r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "kstep_sweep.py")], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if "k_step" in ln]
        print(f"{name:16s} {line[-1] if line else r.stderr[-500:]}", flush=True)


if __name__ == "__main__":
    cmd, names = sys.argv[1], sys.argv[2:] or list(VARIANTS)
    (build if cmd == "build" else run)(names)
