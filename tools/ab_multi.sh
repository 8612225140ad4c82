#!/bin/bash
# A/B/C... of environment settings in one box call: the f32 headline step, each setting ROUNDS times,
# alternating (S timed steps per run).
# Usage: gpurun -- bash tools/ab_multi.sh <tag> <rounds> <steps> "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
OUT=gpurun_out/$1; R=$2; S=$3; shift 3
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in $(seq 1 $R); do
  k=0
  for cfg in "$@"; do
    k=$((k+1))
    env $cfg timeout -k 10 300 python -u bench.py --precision f32 --no-augment-variant --no-eval-variant --no-dp-variant \
      --no-cpu-baseline --no-roofline --steps $S --warmup 5 > $OUT/ab_${k}_$i.log 2>&1 || { echo "[$cfg] $i failed"; tail -5 $OUT/ab_${k}_$i.log; exit 1; }
    echo "[$cfg] $i $(tail -1 $OUT/ab_${k}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
