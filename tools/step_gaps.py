"""Idle gaps inside bench.py's timed steps (between the trace markers) of a rocprofv3 kernel trace CSV:
python tools/step_gaps.py TRACE.csv [min_gap_us] -> per-step idle and the largest gaps with neighbours."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 40.0
names = [r["Kernel_Name"] for r in rows]
mk = [i for i, n in enumerate(names) if "trace_marker" in n]
a, b = mk[0], mk[1]
sub = rows[a:b + 1]
busy_end = int(sub[0]["End_Timestamp"])
gaps = []
for i in range(1, len(sub)):
    s = int(sub[i]["Start_Timestamp"])
    if s - busy_end > thr * 1000:
        gaps.append(((s - busy_end) / 1000, i))
    busy_end = max(busy_end, int(sub[i]["End_Timestamp"]))
span = (int(sub[-1]["End_Timestamp"]) - int(sub[0]["Start_Timestamp"])) / 1000
print(f"span {span:.1f} us, {len(gaps)} gaps > {thr} us totalling {sum(g for g, _ in gaps):.1f} us")


def sh(n):
    return n.replace("void ", "").replace("at::native::", "").replace("mx::", "").split("(")[0][:70]


agg = {}
for g, i in gaps:
    k = (sh(sub[i - 1]["Kernel_Name"]), sh(sub[i]["Kernel_Name"]))
    agg.setdefault(k, [0, 0.0])
    agg[k][0] += 1
    agg[k][1] += g
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{t:9.1f} us x{n:3d}  after {k[0]:60s} before {k[1]}")
