#!/bin/bash
# wgrad kernel variants: parity tests, then per-shape timing (bf16x3, HIP-graph replays)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -k "wide_tiles or presplit" -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/bench_conv.py --dtype f32 --graph --reps 20 --wgrad "$@" > $OUT/bench_conv.log 2>&1 \
  || { echo "bench failed"; tail -20 $OUT/bench_conv.log; exit 1; }
grep -E "==|3x3|aggregate" $OUT/bench_conv.log
