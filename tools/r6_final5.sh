#!/bin/bash
# r06 final sanity at HEAD (after the last rebuild): smoke, the conv / planes / model tests, a short bench
set -o pipefail
OUT=gpurun_out/r06f5
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_x3p.py tests/test_gpu_model.py tests/test_gpu_sample.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --precision f32 --no-augment-variant --no-eval-variant --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
