#!/bin/bash
# Kernel + HIP API trace of the f32 headline step (rocprofv3 --kernel-trace --hip-trace, no counters):
# which host calls block (synchronize / memcpy) and how far the host runs ahead of the GPU.
# Usage: gpurun -- bash tools/api_trace.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/at -o at -- \
  python3 bench.py --precision f32 --steps 8 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
  --no-eval-variant --no-dp-variant > $OUT/api_trace.log 2>&1 || { echo "api trace failed"; tail -20 $OUT/api_trace.log; exit 1; }
for f in $(find $OUT/at -name '*kernel_trace.csv' -o -name '*hip_api_trace.csv'); do gzip -c "$f" > $OUT/$(basename $f).gz; done
rm -rf $OUT/at
ls -la $OUT
