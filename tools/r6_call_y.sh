#!/bin/bash
# r06y: optimizer steady-state checks: x3p tests (incl. the planes-on/off train step), model tests, A/B
set -o pipefail
OUT=gpurun_out/r06y
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_x3p.py tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_rpn_canvas.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests.log | head; echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --precision f32 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
  --no-eval-variant --no-dp-variant > "$OUT/prof.log" 2>&1 || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_concurrency.py "$tr" 10 > "$OUT/conc.txt" 2>&1
python3 tools/prof_steps.py "$OUT/prof" --steps 10 --out "$OUT/steps.csv" > "$OUT/steps.log" 2>&1
rm -rf "$OUT/prof"
head -4 "$OUT/conc.txt"
grep -E "upsample|act_bias" "$OUT/steps.csv" | cut -c1-160
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --precision f32 --no-augment-variant --no-eval-variant --no-cpu-baseline \
    --no-roofline --no-dp-variant --steps 30 --warmup 5 > $OUT/b$i.log 2>&1 || { echo "bench $i failed"; tail -5 $OUT/b$i.log; exit 1; }
  tail -1 $OUT/b$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
done
