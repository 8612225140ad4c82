#!/bin/bash
# r06 final records, part 1: full GPU suite, PMC traffic pass (both precisions), rocprofv3 kernel trace +
# stats of a 10-step bench (per-step kernel table, step concurrency)
set -o pipefail
OUT=gpurun_out/r06f1
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/pmc_traffic.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
cp gpurun_out/pmc_traffic/traffic.json $OUT/traffic.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dp-variant > "$OUT/prof.log" 2>&1 \
  || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
for f in $(find "$OUT/prof" -name '*_stats.csv'); do cp "$f" "$OUT/"; done
python3 tools/prof_steps.py "$OUT/prof" --steps 10 --out "$OUT/step_kernels.csv" > "$OUT/step_kernels.log" 2>&1
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_concurrency.py "$tr" 10 > "$OUT/step_concurrency.txt" 2>&1
rm -rf "$OUT/prof"
head -4 "$OUT/step_concurrency.txt"
tail -1 "$OUT/prof.log"
echo "final1 done"
