#!/bin/bash
# r06g: GPU suite; A/B of the DP segment boundaries (one-rank nccl DataParallel step) and of the DMA
# wgrad tuner candidate (f32 headline)
set -o pipefail
OUT=gpurun_out/r06g
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06g_dp 2 30 "MX_BENCH_DP=1 MX_DP_BOUNDS=2345" "MX_BENCH_DP=1 MX_DP_BOUNDS=23" \
  "MX_BENCH_DP=1 MX_DP_BOUNDS=4" "MX_BENCH_DP=1 MX_DP_BOUNDS=5" "MX_DP_BOUNDS=23" || exit $?
bash tools/ab_multi.sh r06g_w 3 30 "MX_X3_DMAW=0" "MX_X3_DMAW=1"
