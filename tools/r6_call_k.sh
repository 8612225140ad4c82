#!/bin/bash
# r06k: fused sampler tests + the GPU tests touching the samplers, then A/B of MX_FUSED_SAMPLER (f32 headline)
set -o pipefail
OUT=gpurun_out/r06k
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_model.py tests/test_gpu_gt_race.py tests/test_gpu_graphs.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06k_ab 3 30 "MX_FUSED_SAMPLER=0" "MX_FUSED_SAMPLER=1"
