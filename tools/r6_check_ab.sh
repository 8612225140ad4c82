#!/bin/bash
# GPU suite, then an A/B/C of environment settings -- the A/B runs even when tests FAIL (pytest rc 1),
# but not after a crash, a fault or a time limit (any other rc).
# Usage: gpurun -- bash tools/r6_check_ab.sh <tag> <rounds> <steps> "CFG" "CFG" ...
set -o pipefail
TAG=$1; R=$2; S=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh ${TAG}_ab $R $S "$@"
