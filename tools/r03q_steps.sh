set -o pipefail
T=${TAG:-r03q}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o prof -- python3 tools/hbm_ops_probe.py > gpurun_out/$T/probe.log 2>&1 || { tail -20 gpurun_out/$T/probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/probe.log | tail -40
f=$(find gpurun_out/$T/prof -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/$T/kstats.csv
grep -i "roi\|nms\|fill\|copy" gpurun_out/$T/kstats.csv | cut -c1-80,160-260
k=$(find gpurun_out/$T/prof -name '*kernel_trace.csv' | head -1)
python3 - "$k" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last 60 dispatches: the hbm_ops timing reps
for r in rows[-45:]:
    print(r["Kernel_Name"][:70], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
PY
rm -rf gpurun_out/$T/prof
