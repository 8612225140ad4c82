"""Kernel timeline around the boundary of bench.py's timed steps (rocprofv3 kernel trace CSV):
python tools/step_timeline.py TRACE.csv [n_first] [n_last] -> the last kernels of one step and the
first of the next with the idle gap before each (where the host is on the critical path)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 40
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 25
names = [r["Kernel_Name"] for r in rows]
mk = [i for i, n in enumerate(names) if "trace_marker" in n]
a, b = mk[0], mk[1]
sub = rows[a:b + 1]


def sh(n):
    return n.replace("void ", "").replace("at::native::", "").replace("mx::", "").split("(")[0][:60]


# steps: split the timed region at the largest gaps? print around the middle: find kernels named sgd_pack
idx = [i for i, r in enumerate(sub) if "sgd_pack" in r["Kernel_Name"]]
i0 = idx[len(idx) // 2] if idx else len(sub) // 2
end = int(sub[max(i0 - nl, 0)]["End_Timestamp"])
for r in sub[max(i0 - nl, 0) + 1: i0 + nf]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - end) / 1000
    print(f"{gap:8.1f} us gap | {(e - s) / 1000:8.1f} us | stream {r.get('Stream_Id', '?'):>3} | {sh(r['Kernel_Name'])}")
    end = max(end, e)
