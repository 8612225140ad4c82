#!/bin/bash
# r06b: GPU suite without the deferred-wgrad test, A/B of the conv tail and the RPN helper thread,
# then (last: it crashes the host process) the deferred-wgrad test alone with native backtraces.
set -o pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  --deselect "tests/test_gpu_dp.py::test_one_gpu_segmented_graphs_deferred_wgrads" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06b_ab 2 30 "MX_CONV_TAIL=0 MX_RPN_TARGETS_THREAD=0" "MX_CONV_TAIL=1 MX_RPN_TARGETS_THREAD=0" \
  "MX_CONV_TAIL=0 MX_RPN_TARGETS_THREAD=1" "MX_CONV_TAIL=1 MX_RPN_TARGETS_THREAD=1" || exit $?
MX_SEGV_BT=1 timeout -k 10 300 python -u -m pytest -p no:faulthandler -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_dp.py::test_one_gpu_segmented_graphs_deferred_wgrads" > $OUT/segv.log 2>&1
echo "segv repro rc=$?"
grep -A40 "segv_bt" $OUT/segv.log | head -60
