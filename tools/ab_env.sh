#!/bin/bash
# A/B of an environment switch in one box call: the f32 headline step, alternating VAR=A / VAR=B,
# ROUNDS times each (30 timed steps per run).
# Usage: gpurun -- bash tools/ab_env.sh <tag> <VAR> <A> <B> [rounds] [steps]
set -o pipefail
OUT=gpurun_out/$1; VAR=$2; A=$3; B=$4; R=${5:-3}; S=${6:-30}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --precision f32 --no-augment-variant --no-eval-variant --no-dp-variant \
      --no-cpu-baseline --no-roofline --steps $S --warmup 5 > $OUT/ab_${v}_$i.log 2>&1 || { echo "$v $i failed"; tail -5 $OUT/ab_${v}_$i.log; exit 1; }
    echo "$VAR=$v $i $(tail -1 $OUT/ab_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
