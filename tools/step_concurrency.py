"""Where the timed steps' wall time goes (rocprofv3 kernel trace CSV of bench.py, between its trace markers):
python tools/step_concurrency.py TRACE.csv [steps]

Prints per step: span, time with >= 1 kernel running (busy), idle split by gap length (< 5 us: launch /
dependency latency; 5-20 us; >= 20 us: host on the critical path), time with >= 2 kernels running, and
the kernel time by category (conv fwd/dgrad/wgrad, split reduces, BN, RoI, NMS/top-k, other). Also the
idle gaps of the backward graph region grouped by the kernels on either side."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
names = [r["Kernel_Name"] for r in rows]
mk = [i for i, n in enumerate(names) if "trace_marker" in n]
sub = rows[mk[0] + 1:mk[1]]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in sub]


def sh(n):
    return (n.replace("void ", "").replace("at::native::", "").replace("(anonymous namespace)::", "")
            .replace("mx::", "").split("(")[0][:48])


def cat(n):
    if "conv_wgrad" in n:
        return "conv wgrad"
    if "wgrad_reduce" in n:
        return "wgrad reduce"
    if "splitk_reduce" in n:
        return "split-K reduce"
    if "conv_x3_buf_kernel" in n or "conv_x3_kernel" in n or "conv_igemm" in n or "conv_stem" in n:
        return "conv dgrad" if ("<128, 1" in n or "<64, 1" in n or "<256, 1" in n) else "conv fwd"
    if "bn_" in n:
        return "batchnorm"
    if "roi_" in n:
        return "roi align"
    if "nms" in n or "topk" in n or "mbtopk" in n or "radix" in n.lower():
        return "nms/topk"
    if "sgd" in n or "pack" in n:
        return "sgd/pack"
    if "copyBuffer" in n or "fillBuffer" in n:
        return "copies"
    return "other"


t0, t1 = iv[0][0], max(e for _, e, _ in iv)
span = (t1 - t0) / 1e3
# sweep: busy, >=2 concurrent
ev = sorted([(s, 1) for s, _, _ in iv] + [(e, -1) for _, e, _ in iv])
busy = conc = 0
cur, last = 0, t0
for t, d in ev:
    if cur >= 1:
        busy += t - last
    if cur >= 2:
        conc += t - last
    cur += d
    last = t
gaps = defaultdict(float)
gcount = defaultdict(int)
pairs = defaultdict(lambda: [0, 0.0])
end = iv[0][1]
for i in range(1, len(iv)):
    s, e, n = iv[i]
    g = (s - end) / 1e3
    if g > 0:
        k = "<5us" if g < 5 else ("5-20us" if g < 20 else ">=20us")
        gaps[k] += g
        gcount[k] += 1
        if g >= 5:
            key = (sh(iv[i - 1][2]), sh(n))
            pairs[key][0] += 1
            pairs[key][1] += g
    end = max(end, e)
ktime = defaultdict(float)
for s, e, n in iv:
    ktime[cat(n)] += (e - s) / 1e3
print(f"{steps} steps: span {span / steps:.3f} us/step, busy {busy / 1e3 / steps:.3f}, idle {(span - busy / 1e3) / steps:.3f}, "
      f">=2 kernels {conc / 1e3 / steps:.3f} us/step")
for k in ("<5us", "5-20us", ">=20us"):
    print(f"  idle gaps {k:7s}: {gaps[k] / steps:8.3f} us/step in {gcount[k] / steps:6.1f} gaps/step")
print("kernel time by category (us/step, summed over streams):")
for k, v in sorted(ktime.items(), key=lambda kv: -kv[1]):
    print(f"  {k:15s} {v / steps:8.3f}")
print("largest idle pairs (gaps >= 5 us), us/step:")
for (a, b), (c, t) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"  {t / steps:7.3f} ({c / steps:5.1f}/step)  {a:48s} -> {b}")
