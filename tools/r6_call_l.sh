#!/bin/bash
# r06l: kernel traces of the f32 headline step, plain and through DataParallel in a one-rank nccl group
# (MX_BENCH_DP=1): step concurrency of each (where the DP leg's extra ms/step goes)
set -o pipefail
OUT=gpurun_out/r06l
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for leg in plain dp; do
  if [ $leg = dp ]; then export MX_BENCH_DP=1; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_$leg" -o prof -- \
    python3 bench.py --precision f32 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
    --no-eval-variant --no-dp-variant > "$OUT/prof_$leg.log" 2>&1 || { echo "prof $leg failed rc=$?"; tail -30 "$OUT/prof_$leg.log"; exit 1; }
  tr=$(find "$OUT/prof_$leg" -name '*kernel_trace.csv' | head -n 1)
  python3 tools/step_concurrency.py "$tr" 10 > "$OUT/conc_$leg.txt" 2>&1
  python3 tools/prof_steps.py "$OUT/prof_$leg" --steps 10 --out "$OUT/steps_$leg.csv" > "$OUT/steps_$leg.log" 2>&1
  rm -rf "$OUT/prof_$leg"
  tail -1 "$OUT/prof_$leg.log"; head -4 "$OUT/conc_$leg.txt"
done
unset MX_BENCH_DP
