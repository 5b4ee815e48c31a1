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

PGS_OLD = """            float db, dc;
            {
              const float l1 = lb - vb1 * G.invD[1], l2 = lc - vc1 * G.invD[2];
              const float lim = G.mu * na, nn2 = l1 * l1 + l2 * l2;
              const float sc = nn2 > lim * lim ? lim * __builtin_amdgcn_rsqf(nn2) : 1.f;
              const float nbs = clampf(lb + (G.tgt[1] - vb1) * G.invD[1], G.lo[1], G.hi[1]);
              const float dbs = nbs - lb;
              const float vc2 = vc1 + G.Wcb * dbs;
              const float ncs = clampf(lc + (G.tgt[2] - vc2) * G.invD[2], G.lo[2], G.hi[2]);
              const bool ct = G.mu >= 0.f;
              db = ct ? l1 * sc - lb : dbs;
              dc = ct ? l2 * sc - lc : ncs - lc;
            }"""
PGS_NEW = """            float db, dc;
            if (g < npts_lo) {  // a contact group in both envs of the wave
              const float l1 = lb - vb1 * G.invD[1], l2 = lc - vc1 * G.invD[2];
              const float lim = G.mu * na, nn2 = l1 * l1 + l2 * l2;
              const float sc = nn2 > lim * lim ? lim * __builtin_amdgcn_rsqf(nn2) : 1.f;
              db = l1 * sc - lb;
              dc = l2 * sc - lc;
            } else if (g >= npts_hi) {  // single rows in both envs
              const float nbs = clampf(lb + (G.tgt[1] - vb1) * G.invD[1], G.lo[1], G.hi[1]);
              const float dbs = nbs - lb;
              const float vc2 = vc1 + G.Wcb * dbs;
              const float ncs = clampf(lc + (G.tgt[2] - vc2) * G.invD[2], G.lo[2], G.hi[2]);
              db = dbs;
              dc = ncs - lc;
            } else {
              const float l1 = lb - vb1 * G.invD[1], l2 = lc - vc1 * G.invD[2];
              const float lim = G.mu * na, nn2 = l1 * l1 + l2 * l2;
              const float sc = nn2 > lim * lim ? lim * __builtin_amdgcn_rsqf(nn2) : 1.f;
              const float nbs = clampf(lb + (G.tgt[1] - vb1) * G.invD[1], G.lo[1], G.hi[1]);
              const float dbs = nbs - lb;
              const float vc2 = vc1 + G.Wcb * dbs;
              const float ncs = clampf(lc + (G.tgt[2] - vc2) * G.invD[2], G.lo[2], G.hi[2]);
              const bool ct = G.mu >= 0.f;
              db = ct ? l1 * sc - lb : dbs;
              dc = ct ? l2 * sc - lc : ncs - lc;
            }"""
PGS_NG_OLD = "      const int ng = (max(shm[0].nrows, shm[1].nrows) + 2) / 3;"
PGS_NG_NEW = ("      const int ng = (max(shm[0].nrows, shm[1].nrows) + 2) / 3;\n"
              "      const int npts_lo = min(shm[0].npts, shm[1].npts), npts_hi = max(shm[0].npts, shm[1].npts);")
DIV = [("  float s = denom > 1e-6f * a * e ? fminf(fmaxf((b * f - c * e) / denom, 0.f), 1.f) : 0.f;\n"
        "  float t = (b * s + f) / e;\n"
        "  if (t < 0.f) { t = 0.f; s = fminf(fmaxf(-c / a, 0.f), 1.f); }\n"
        "  else if (t > 1.f) { t = 1.f; s = fminf(fmaxf((b - c) / a, 0.f), 1.f); }",
        "  const float ia = __builtin_amdgcn_rcpf(a), ie = __builtin_amdgcn_rcpf(e);\n"
        "  float s = denom > 1e-6f * a * e ? fminf(fmaxf((b * f - c * e) * __builtin_amdgcn_rcpf(denom), 0.f), 1.f) : 0.f;\n"
        "  float t = (b * s + f) * ie;\n"
        "  if (t < 0.f) { t = 0.f; s = fminf(fmaxf(-c * ia, 0.f), 1.f); }\n"
        "  else if (t > 1.f) { t = 1.f; s = fminf(fmaxf((b - c) * ia, 0.f), 1.f); }"),
       ("    C.cn = dist > 1e-9f ? (1.0f / dist) * dv : mk(0.f, -1.f, 0.f);",
        "    C.cn = dist > 1e-9f ? __builtin_amdgcn_rcpf(dist) * dv : mk(0.f, -1.f, 0.f);")]

# compiler-flag variants (same source): AMDGPU machine-scheduler strategies for the latency-bound
# per-wave chain (scheduling only: bitwise identical results)
FLAG_VARIANTS = {
    "ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "iter_ilp": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "memclause": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    "trackers": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    "bias_lat": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
}

VARIANTS = {
    "base": [],
    "ilp": [], "iter_ilp": [], "memclause": [], "trackers": [], "bias_lat": [],
    "no_round2": [("const int rounds = nitems > 32 ? 2 : 1;", "const int rounds = 1;")],
    "pgs_spec": [(PGS_NG_OLD, PGS_NG_NEW), (PGS_OLD, PGS_NEW)],
    "fastdiv": DIV,
    "pgs_spec_fastdiv": [(PGS_NG_OLD, PGS_NG_NEW), (PGS_OLD, PGS_NEW)] + DIV,
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
            r = subprocess.run([HIPCC] + FLAGS + FLAG_VARIANTS.get(name, []) + ["-c", hip, "-o", os.path.join(d, "hg_physics.o"),
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
