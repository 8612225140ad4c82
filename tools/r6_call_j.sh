#!/bin/bash
# r06j: full GPU suite, then A/B of the pre-split planes (f32 headline)
set -o pipefail
OUT=gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06j_ab 3 30 "MX_X3_PLANES=0" "MX_X3_PLANES=1"
