#!/bin/bash
# r06fj: eval-side fold cache: eval / U-Net / model tests, then the eval legs and their trace
set -o pipefail
OUT=gpurun_out/r06fj
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_model_f32.py tests/test_gpu_scripts.py tests/test_gpu_rpn_canvas.py tests/test_gpu_conv.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests.log | head; echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_unet.py -x -q --timeout 300 > $OUT/tests_unet.log 2>&1 || { echo "unet tests failed"; tail -5 $OUT/tests_unet.log; exit 1; }
tail -1 $OUT/tests_unet.log
for mode in eval eval_restored; do
  timeout -k 10 400 python -u bench.py --mode $mode --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$mode.log 2>&1 || { echo "$mode failed"; tail -5 $OUT/$mode.log; exit 1; }
  tail -1 $OUT/$mode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:40], d["value"], d["ms_per_step"])'
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --mode eval --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof.log" 2>&1 || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_concurrency.py "$tr" 20 > "$OUT/conc.txt" 2>&1
python3 tools/prof_steps.py "$OUT/prof" --steps 20 --out "$OUT/steps.csv" > "$OUT/steps.log" 2>&1
rm -rf "$OUT/prof"
head -30 "$OUT/conc.txt"
