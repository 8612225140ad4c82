set -o pipefail
mkdir -p gpurun_out/tr
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/raw -o t -- python3 bench.py --steps 4 --warmup 3 --precision f32 --no-cpu-baseline --no-roofline --no-augment-variant > gpurun_out/tr/log 2>&1 || { tail gpurun_out/tr/log; exit 1; }
f=$(find gpurun_out/tr/raw -name '*kernel_trace.csv' | head -n 1)
python3 - $f <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names=[r["Kernel_Name"] for r in rows]
mk=[i for i,n in enumerate(names) if "trace_marker" in n]
sub=rows[mk[0]:mk[1]+1]
import csv as c2
w=c2.writer(open('gpurun_out/tr/steps.csv','w'))
w.writerow(["Kernel_Name","Start_Timestamp","End_Timestamp"])
for r in sub: w.writerow([r["Kernel_Name"][:120],r["Start_Timestamp"],r["End_Timestamp"]])
PY
python3 tools/all_gaps.py gpurun_out/tr/steps.csv > gpurun_out/tr/allgaps.txt
rm -rf gpurun_out/tr/raw
cat gpurun_out/tr/allgaps.txt
