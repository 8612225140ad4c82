"""Summarise a rocprofv3 kernel_stats.csv per train step: python tools/prof_summary.py CSV [steps] [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
S = float(sys.argv[2]) if len(sys.argv) > 2 else 14
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
cat = {}
for r in rows:
    n, t = r["Name"], float(r["TotalDurationNs"]) / 1e6 / S
    k = ("conv" if "conv_" in n or "wgrad_reduce" in n else "bn" if "bn_" in n or "act_bias" in n else
         "mx_other" if "mx::" in n else "torch/other")
    cat[k] = cat.get(k, 0) + t
print("per step ms:", {k: round(v, 3) for k, v in cat.items()}, "total", round(sum(cat.values()), 3))
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / S:8.3f} ms {int(r['Calls']) / S:6.1f} calls "
          f"{float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:120]}")
