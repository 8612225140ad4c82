#!/bin/bash
# A/B of two builds of libmx_det in one box call: the f32 headline step, alternating
# mx_det/libmx_det_prev.so (A) and mx_det/libmx_det.so (B), ROUNDS times each.
# Usage: gpurun -- bash tools/ab_lib.sh <tag> [rounds]
set -o pipefail
OUT=gpurun_out/$1
R=${2:-2}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in $(seq 1 $R); do
  for v in prev cur; do
    lib=robust-object-detection_amd/mx_det/libmx_det.so
    [ $v = prev ] && lib=robust-object-detection_amd/mx_det/libmx_det_prev.so
    MX_DET_LIB=$PWD/$lib timeout -k 10 240 python -u bench.py --precision f32 --no-augment-variant --no-eval-variant --no-dp-variant \
      --no-cpu-baseline --no-roofline --steps 30 --warmup 5 > $OUT/ab_${v}_$i.log 2>&1 || { echo "$v $i failed"; tail -5 $OUT/ab_${v}_$i.log; exit 1; }
    echo "$v $i $(tail -1 $OUT/ab_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
