#!/bin/bash
# r06p: tests touching the RoI candidates / sampler validity, then A/B of MX_FUSED_SAMPLER and a step trace
set -o pipefail
OUT=gpurun_out/r06p
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_model.py tests/test_gpu_model_f32.py tests/test_gpu_graphs.py tests/test_gpu_guards.py tests/test_gpu_gt_race.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests.log | head; echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06p_ab 3 30 "MX_FUSED_SAMPLER=0" "MX_FUSED_SAMPLER=1" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --precision f32 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
  --no-eval-variant --no-dp-variant > "$OUT/prof.log" 2>&1 || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_concurrency.py "$tr" 10 > "$OUT/conc.txt" 2>&1
python3 tools/prof_steps.py "$OUT/prof" --steps 10 --out "$OUT/steps.csv" > "$OUT/steps.log" 2>&1
rm -rf "$OUT/prof"
head -4 "$OUT/conc.txt"
