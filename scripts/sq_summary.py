"""Summarise the two SQ counter passes of scripts/pmc_sq.sh for k_step into per-wave figures.
Usage: python scripts/sq_summary.py <pmc_sq dir> <out.json>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1], sys.argv[2]
    tot, launches = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_step" not in r["Kernel_Name"][:24]:
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                launches[r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    # every launch has the same wave count; normalise per launch then per wave
    res = {k: int(v / max(len(launches[k]), 1)) for k, v in tot.items()}
    waves = res.get("SQ_WAVES", 0) or 2048
    res["per_wave"] = {k: round(v / waves, 1) for k, v in res.items() if k != "SQ_WAVES"}
    pw = res["per_wave"]
    wc = pw["SQ_WAVE_CYCLES"]
    res["fractions_of_wave_cycles"] = {
        "active_inst_any": round(pw["SQ_ACTIVE_INST_ANY"] / wc, 3), "wait_any": round(pw["SQ_WAIT_ANY"] / wc, 3),
        "wait_inst_any": round(pw["SQ_WAIT_INST_ANY"] / wc, 3),
        "active_valu": round(pw["SQ_ACTIVE_INST_VALU"] / wc, 3)}
    # two waves share each SIMD: the SIMD's VALU is busy ~2x one wave's VALU-active fraction
    res["simd_valu_busy_est"] = round(2 * pw["SQ_ACTIVE_INST_VALU"] / wc, 3)
    res["_note"] = ("k_step, 4096 envs, 5 PGS sweeps, random actions; 2 waves per SIMD; SQ cycle counters in "
                    "quad-cycles; two --pmc passes with --kernel-trace only (scripts/pmc_sq.sh)")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["fractions_of_wave_cycles"]), res["simd_valu_busy_est"])


if __name__ == "__main__":
    main()
