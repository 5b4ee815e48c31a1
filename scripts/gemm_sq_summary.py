"""Per-kernel figures from the two PMC passes of scripts/pmc_gemm.sh (gemm_micro.py's launches):
counter means per launch, grouped by kernel name (the template arguments tell the tiles apart),
MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) — the busy cycles
of all SIMDs over the launch's GPU-active cycles (GRBM counts once per XCD) — and the wait fraction
SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES.  Usage: python scripts/gemm_sq_summary.py <pmc_gemm dir> <out.json>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1], sys.argv[2]
    tot = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if not any(t in name for t in ("gemm", "wgrad", "Cijk")):
                    continue
                key = (name.replace("void ", "").replace("(anonymous namespace)::", "").split("((")[0]
                       if "Cijk" not in name else name[:60])
                tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[key][r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    res = {}
    for key, c in tot.items():
        per = {k: v / max(len(cnt[key][k]), 1) for k, v in c.items()}
        e = {k: int(v) for k, v in per.items()}
        if per.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in per:
            e["mfma_util"] = round(per["SQ_VALU_MFMA_BUSY_CYCLES"] / (128.0 * per["GRBM_GUI_ACTIVE"]), 3)
        if per.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in per:
            e["wait_inst_any_frac"] = round(per["SQ_WAIT_INST_ANY"] / per["SQ_WAVE_CYCLES"], 3)
        if per.get("SQ_WAVES"):
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA"):
                if k in per:
                    e[k.lower().replace("sq_insts_", "") + "_per_wave"] = round(per[k] / per["SQ_WAVES"])
        res[key] = e
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, e in res.items():
        print(k, "mfma_util", e.get("mfma_util"), "wait", e.get("wait_inst_any_frac"))


if __name__ == "__main__":
    main()
