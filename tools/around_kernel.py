"""Kernels around one kernel of a timed step in a rocprofv3 kernel trace: name, start / end relative to the
anchor's start (us), queue and stream ids -- what the GPU ran (and on which queue) before an idle gap.

    python tools/around_kernel.py TRACE.csv sgd_pack_kernel [--step 5] [--before 12] [--after 3]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("anchor")
ap.add_argument("--step", type=int, default=5)
ap.add_argument("--before", type=int, default=12)
ap.add_argument("--after", type=int, default=3)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
mk = [i for i, n in enumerate(names) if "trace_marker" in n]
sub = rows[mk[0] + 1:mk[1]]
idx = [i for i, r in enumerate(sub) if a.anchor in r["Kernel_Name"]]
i0 = idx[min(a.step, len(idx) - 1)]
t0 = int(sub[i0]["Start_Timestamp"])
qk = next((k for k in ("Queue_Id", "Queue_ID", "queue_id") if k in sub[0]), None)
sk = next((k for k in ("Stream_Id", "Stream_ID", "stream_id") if k in sub[0]), None)
# kernels whose end lies in the window before the anchor, by end time
win = sorted(sub[max(0, i0 - 400):i0 + a.after + 1], key=lambda r: int(r["End_Timestamp"]))
before = [r for r in win if int(r["End_Timestamp"]) <= t0][-a.before:]
after = [r for r in sub[i0:i0 + a.after + 1]]
for r in before + after:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    n = r["Kernel_Name"].replace("void ", "").replace("mx::", "")[:60]
    print(f"{s:10.1f} {e:10.1f}  q={r.get(qk, '?') if qk else '?'} s={r.get(sk, '?') if sk else '?'}  {n}")
