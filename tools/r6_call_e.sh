#!/bin/bash
# r06e2: kernel trace of the eval leg (bench.py --mode eval: per-image eval forward), concurrency per image
set -o pipefail
OUT=gpurun_out/r06e2
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --mode eval --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof.log" 2>&1 || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_concurrency.py "$tr" 20 > "$OUT/conc.txt" 2>&1
python3 tools/prof_steps.py "$OUT/prof" --steps 20 --out "$OUT/steps.csv" > "$OUT/steps.log" 2>&1
rm -rf "$OUT/prof"
tail -1 "$OUT/prof.log" | cut -c1-200
head -40 "$OUT/conc.txt"
