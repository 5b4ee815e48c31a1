"""Per-iteration GPU timeline from a rocprofv3 kernel trace: busy time by kernel class, idle gaps,
and the collection / learn split of the last PPO iteration (K_step launches delimit collection)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [i for i, r in enumerate(rows) if "k_step" in r["Kernel_Name"][:24]]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 24
# last full iteration: from the first K_step of the last group of T to the first K_step of... the end
first = ks[-T]
prev_first = ks[-2 * T]
seg = rows[prev_first:first]  # the second-to-last iteration (collection + learn)


def cls(n):
    if n.startswith("Cijk") or "gemm" in n.lower():
        return "gemm"
    for k in ("k_step", "elu_kernel", "k_act_bwd", "k_colsum", "index_elementwise", "reduce_kernel", "k_post",
              "k_stack", "k_window", "k_skinny", "k_adam", "k_sqnorm", "k_ppo_loss", "k_kl", "copyBuffer", "FillFunctor",
              "gather", "k_act", "k_env", "k_gae", "k_lr"):
        if k in n:
            return k
    return n[:60]


busy = collections.Counter()
cnt = collections.Counter()
t0 = int(seg[0]["Start_Timestamp"])
t1 = int(rows[first]["Start_Timestamp"])
last_end = t0
idle = 0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > last_end:
        idle += s - last_end
    last_end = max(last_end, e)
    c = cls(r["Kernel_Name"])
    busy[c] += e - s
    cnt[c] += 1
kend = int(rows[ks[-T - 1]]["End_Timestamp"])
print(f"iteration wall {1e-6 * (t1 - t0):.3f} ms  collection (to last K_step end) {1e-6 * (kend - t0):.3f} ms  "
      f"idle {1e-6 * idle:.3f} ms  kernels {len(seg)}")
for c, v in busy.most_common():
    print(f"  {1e-6 * v:7.3f} ms  {cnt[c]:5d}  {c}")
