"""Per-step kernel table of bench.py's timed region from a rocprofv3 kernel trace.

bench.py launches trace_marker_kernel before its first and after its last timed step
(mx_trace_marker); this keeps only the dispatches between the first such pair, so warm-up, graph
capture, the per-shape conv tuner and its spin kernels, the roofline step and the CPU baseline are
all excluded. Input: a rocprofv3 output directory (rocpd SQLite *_results.db, or a
--output-format csv *kernel_trace.csv). Output: CSV rows kernel, calls_per_step, avg_us,
ms_per_step, share (sorted by time), plus a summary line on stderr.

    python tools/prof_steps.py gpurun_out/prof_a --steps 10 --out profiles/r02_f32_step_kernels.csv
"""
import argparse
import csv
import glob
import os
import sqlite3
import sys


def load(path):
    """[(name, start_ns, end_ns)] of every kernel dispatch, by start time."""
    dbs = glob.glob(os.path.join(path, "**", "*results.db"), recursive=True)
    if dbs:
        con = sqlite3.connect(dbs[0])
        rows = con.execute("select name, start, end from kernels order by start").fetchall()
        return [(r[0], int(r[1]), int(r[2])) for r in rows]
    csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not csvs:
        raise SystemExit(f"no rocpd db or kernel_trace.csv under {path}")
    out = []
    for r in csv.DictReader(open(csvs[0])):
        out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out, key=lambda t: t[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, required=True, help="timed steps between the markers")
    ap.add_argument("--out", default=None)
    ap.add_argument("--pair", type=int, default=0, help="which begin/end marker pair (0 = first timed region)")
    a = ap.parse_args()
    ks = load(a.path)
    marks = [i for i, k in enumerate(ks) if k[0].startswith("trace_marker_kernel")]
    if len(marks) < 2 * (a.pair + 1):
        raise SystemExit(f"found {len(marks)} trace markers, need a begin/end pair")
    b, e = marks[2 * a.pair], marks[2 * a.pair + 1]
    t0, t1 = ks[b][2], ks[e][1]
    sel = [k for k in ks[b + 1:e] if t0 <= k[1] <= t1]
    agg = {}
    for name, s, en in sel:
        d = agg.setdefault(name, [0, 0])
        d[0] += 1
        d[1] += en - s
    busy = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    out = open(a.out, "w", newline="") if a.out else sys.stdout
    w = csv.writer(out)
    w.writerow(["kernel", "calls_per_step", "avg_us", "ms_per_step", "share"])
    for name, (n, ns) in rows:
        w.writerow([name, round(n / a.steps, 3), round(ns / n / 1e3, 3), round(ns / a.steps / 1e6, 4),
                    round(ns / busy, 4)])
    if a.out:
        out.close()
    wall = (t1 - t0) / a.steps / 1e6
    print(f"{len(sel)} dispatches over {a.steps} steps: kernel busy {busy / a.steps / 1e6:.3f} ms/step, "
          f"wall between markers {wall:.3f} ms/step", file=sys.stderr)


if __name__ == "__main__":
    main()
