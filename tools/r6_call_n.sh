#!/bin/bash
# r06n: sampler tests, then kernel traces of the f32 headline step: plain, DataParallel (one-rank nccl),
# DataParallel without the NMS-flag host read (MX_DP_NMS_FLAG=0); step concurrency of each
set -o pipefail
OUT=gpurun_out/r06n
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sample.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests.log | head; echo "tests rc=$rc: stopping"; exit $rc; fi
for leg in plain dp dpnoflag; do
  case $leg in
    plain) ENVS="" ;;
    dp) ENVS="MX_BENCH_DP=1" ;;
    dpnoflag) ENVS="MX_BENCH_DP=1 MX_DP_NMS_FLAG=0" ;;
  esac
  env $ENVS timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_$leg" -o prof -- \
    python3 bench.py --precision f32 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
    --no-eval-variant --no-dp-variant > "$OUT/prof_$leg.log" 2>&1 || { echo "prof $leg failed rc=$?"; tail -30 "$OUT/prof_$leg.log"; exit 1; }
  tr=$(find "$OUT/prof_$leg" -name '*kernel_trace.csv' | head -n 1)
  python3 tools/step_concurrency.py "$tr" 10 > "$OUT/conc_$leg.txt" 2>&1
  python3 tools/prof_steps.py "$OUT/prof_$leg" --steps 10 --out "$OUT/steps_$leg.csv" > "$OUT/steps_$leg.log" 2>&1
  rm -rf "$OUT/prof_$leg"
  echo "$leg: $(tail -1 "$OUT/prof_$leg.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  head -4 "$OUT/conc_$leg.txt"
done
