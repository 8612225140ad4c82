#!/bin/bash
# r06u: what precedes the optimizer launch and the step's first launch (tools/around_kernel.py)
set -o pipefail
OUT=gpurun_out/r06u
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --precision f32 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
  --no-eval-variant --no-dp-variant > "$OUT/prof.log" 2>&1 || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
head -1 "$tr" > $OUT/columns.txt
python3 tools/around_kernel.py "$tr" sgd_pack_kernel --before 14 > $OUT/around_sgd.txt 2>&1
python3 tools/around_kernel.py "$tr" boxes_degenerate_kernel --before 6 --after 4 > $OUT/around_start.txt 2>&1
rm -rf "$OUT/prof"
cat $OUT/columns.txt $OUT/around_sgd.txt $OUT/around_start.txt
