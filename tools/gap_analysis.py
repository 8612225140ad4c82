"""GPU idle-gap analysis of a rocprofv3 --kernel-trace CSV: python tools/gap_analysis.py TRACE.csv [top]
Prints total busy / idle time over the last steps and the largest gaps with the kernels around them."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# steady state: from the 4th-last per-step weight pack (one pack_batched_kernel per train step)
marks = [e[0] for e in ev if "pack_batched_kernel" in e[2]]
cut = marks[-4] if len(marks) >= 4 else ev[0][0]
ev = [e for e in ev if e[0] >= cut]
print(f"steps analysed: {min(4, len(marks))}")
busy, gaps, end = 0, [], ev[0][0]
for s, e, n in ev:
    if s > end:
        gaps.append((s - end, n, end))
    busy += max(0, e - max(s, end))
    end = max(end, e)
span = end - ev[0][0]
print(f"span {span/1e6:.2f} ms busy {busy/1e6:.2f} ms idle {(span-busy)/1e6:.2f} ms ({100*(span-busy)/span:.1f}%)")
gaps.sort(reverse=True)
tot = {}
for g, n, _ in gaps:
    k = n[:70]
    tot[k] = tot.get(k, 0) + g
print("largest idle gaps (us) and the kernel that ended them:")
for g, n, _ in gaps[:top]:
    print(f"{g/1e3:8.1f}  {n[:110]}")
print("idle by following kernel:")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:top]:
    print(f"{v/1e6:7.3f} ms  {k}")
