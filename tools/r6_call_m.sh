#!/bin/bash
# r06m: DataParallel tests after the host-work cuts, then the plain / DP step traces (r6_call_l.sh)
set -o pipefail
OUT=gpurun_out/r06m
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_dp.py tests/test_gpu_dp2.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
sed -i 's#OUT=gpurun_out/r06l#OUT=gpurun_out/r06m#' tools/r6_call_l.sh
bash tools/r6_call_l.sh
