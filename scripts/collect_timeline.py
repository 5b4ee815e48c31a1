"""Collection-phase timeline of one PPO iteration from a rocprofv3 kernel trace: for one policy
step (K_step end -> next K_step start) the kernels in between with their durations and the idle
gaps, and per-step averages of busy vs idle over the iteration.  Usage:
  python scripts/collect_timeline.py <kernel_trace.csv> [T]"""
import sys
import csv

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
T = int(sys.argv[2]) if len(sys.argv) > 2 else 24
ks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void k_step")]
it = ks[-2 * T:-T]  # K_step launches of the second-to-last iteration
busy = idle = 0
for a, b in zip(it[:-1], it[1:]):
    end = int(rows[a]["End_Timestamp"])
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        idle += max(0, s - end)
        busy += e - s if r is not rows[b] else 0
        end = max(end, e)
n = len(it) - 1
print(f"between K_steps, per step: busy {busy / n / 1e3:.1f} us, idle {idle / n / 1e3:.1f} us")
a, b = it[T // 2], it[T // 2 + 1]
end = int(rows[a]["End_Timestamp"])
print(f"step {T // 2}: K_step {(int(rows[a]['End_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3:.1f} us")
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  gap {(s - end) / 1e3:6.1f}  dur {(e - s) / 1e3:6.1f}  {r['Kernel_Name'][:90]}")
    end = e
