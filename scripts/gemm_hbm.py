"""HBM bytes per launch of every GEMM dispatch class (kernel template, grid in workgroups) from the
FETCH_SIZE / WRITE_SIZE passes of scripts/profile.sh, with the gfx950 correction of
scripts/pmc_summary.py (FETCH_SIZE doubled, WRITE_SIZE as is), and the class's mean duration from
the kernel trace of the same bench: HBM GB/s achieved.  (pmc_summary.py keys by short kernel name
and leaves the bf16-split GEMMs out.)

    python scripts/gemm_hbm.py gpurun_out/prof > profiles/<set>/gemm_hbm.txt
"""
import collections
import csv
import glob
import os
import re
import sys


def key(name, grid, wg):
    m = re.search(r"(k_gemm_x6|k_gemm|k_wgrad_tr|k_splitk_finish|Cijk_\w{0,40})(<[^>]*>)?", name)
    return (m.group(0)[:72] if m else name[:72], grid // max(wg, 1))


def counters(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if r["Counter_Name"] != counter or not ("gemm" in n.lower() or "Cijk" in n or "wgrad" in n or "splitk" in n):
                continue
            acc[key(n, int(r["Grid_Size"]), int(r["Workgroup_Size"]))].append(float(r["Counter_Value"]))
    return acc


def main(prof):
    fetch = counters(os.path.join(prof, "pmc_fetch"), "FETCH_SIZE")
    write = counters(os.path.join(prof, "pmc_write"), "WRITE_SIZE")
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_trace.csv"))):
        n = r["Kernel_Name"]
        if "gemm" in n.lower() or "Cijk" in n or "wgrad" in n or "splitk" in n:
            dur[key(n, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("HBM MB per launch (2 x FETCH_SIZE + WRITE_SIZE), mean us (trace), GB/s")
    rows = []
    for k in set(fetch) | set(write):
        f = sum(fetch[k]) / max(len(fetch[k]), 1)
        w = sum(write[k]) / max(len(write[k]), 1)
        mb = (2 * f + w) * 1024 / 1e6
        us = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
        rows.append((mb, k, us))
    for mb, (nm, g), us in sorted(rows, reverse=True):
        print(f"{mb:9.2f} MB  {us:8.2f} us  {mb / us * 1e3 if us == us else float('nan'):8.1f} GB/s  grid {g:6d}  {nm}")


if __name__ == "__main__":
    main(sys.argv[1])
