#!/bin/bash
# r06i: x3p + DP tests, per-shape x3p timing
set -o pipefail
OUT=gpurun_out/r06i
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3p.py tests/test_gpu_dp.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_conv.py --dtype f32 --graph --reps 20 --planes > $OUT/bench_conv.log 2>&1 \
  || { echo "bench failed"; tail -20 $OUT/bench_conv.log; exit 1; }
cat $OUT/bench_conv.log | cut -c1-400
