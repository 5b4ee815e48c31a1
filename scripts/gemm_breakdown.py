"""Per-dispatch-class GEMM time per PPO iteration from a rocprofv3 kernel trace of bench.py: the
build's GEMM kernels (k_gemm, k_gemm_x6, k_wgrad_tr, k_splitk_finish) and hipBLASLt's (Cijk_*)
grouped by (kernel, grid in workgroups, workgroup size) — the grid names the shape — with launches
per iteration (iterations counted by K_gae's three launches each) and the mean duration.

    python scripts/gemm_breakdown.py gpurun_out/prof/trace/run_kernel_trace.csv > profiles/<set>/gemm_breakdown.txt
"""
import collections
import csv
import re
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    n_it = sum(1 for r in rows if "k_gae" in r["Kernel_Name"]) / 3
    agg = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if not ("gemm" in n.lower() or "Cijk" in n or "wgrad" in n or "splitk" in n):
            continue
        wg = int(r["Workgroup_Size_X"])
        agg[(n, int(r["Grid_Size_X"]) // wg, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out, tot = [], 0.0
    for (n, g, wg), v in agg.items():
        per_it, avg = len(v) / n_it, sum(v) / len(v)
        tot += per_it * avg
        m = re.search(r"(k_gemm_x6|k_gemm|k_wgrad_tr|k_splitk_finish|Cijk_\w{0,40})(<[^>]*>)?", n)
        out.append((per_it * avg, m.group(0)[:72] if m else n[:72], g, wg, per_it, avg))
    print(f"{n_it:.0f} iterations traced; GEMM kernels {tot / 1e3:.3f} ms per iteration")
    for t, nm, g, wg, pi, avg in sorted(out, reverse=True):
        print(f"{t / 1e3:7.3f} ms/it  {pi:5.1f} x {avg:8.2f} us  grid {g:6d}  wg {wg:4d}  {nm}")


if __name__ == "__main__":
    main(sys.argv[1])
