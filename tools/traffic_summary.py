"""Per-kernel HBM bytes per launch from the two rocprofv3 --pmc passes of tools/pmc_traffic.sh.
bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950: FETCH_SIZE reports half of a 16-B/lane
streaming read, MI355X_MICROARCH.md §HBM). Only the last 40% of dispatches (steady state) count."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{root}/{c}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == c]
    rows = rows[int(0.6 * len(rows)):]
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[name][c].append(float(r["Counter_Value"]))
out = {}
for name, d in per.items():
    fs, ws = d.get("FETCH_SIZE", []), d.get("WRITE_SIZE", [])
    if not fs or not ws:
        continue
    rd = 2 * 1024 * sum(fs) / len(fs)
    wr = 1024 * sum(ws) / len(ws)
    out[name] = {"launches": len(fs), "read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
print(json.dumps({"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bytes = 2*FETCH_SIZE*1024 "
                  "+ WRITE_SIZE*1024 per dispatch, mean over steady-state dispatches", "kernels": out}, indent=1))
