#!/bin/bash
# r06h: x3p parity + DP tests, then A/B of the pre-split planes (f32 headline) and of the DP segment
# boundaries (one-rank nccl DataParallel step)
set -o pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3p.py tests/test_gpu_dp.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06h_ab 3 30 "MX_X3_PLANES=0" "MX_X3_PLANES=1" "MX_BENCH_DP=1 MX_DP_BOUNDS=2345" "MX_BENCH_DP=1 MX_DP_BOUNDS=23"
