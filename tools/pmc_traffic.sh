#!/bin/bash
# HBM traffic of the step's kernels from PMC counters (MI355X_MICROARCH.md §HBM: FETCH_SIZE and
# WRITE_SIZE in separate passes; gfx950 FETCH_SIZE counts half of a wide streaming read).
# MX_PMC_PRECISION=f32 | bf16 | both (default: both, merged: the f32 headline's kernels plus the
# bf16-only conv kernels). Writes gpurun_out/pmc_traffic/traffic.json (per kernel: launches, mean
# bytes per launch).
set -o pipefail
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
export TMPDIR=/tmp MX_GRAPHS=0
P=${MX_PMC_PRECISION:-both}
[ "$P" = both ] && PRECS="f32 bf16" || PRECS=$P
for prec in $PRECS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/$prec/$c -o p -- \
      python3 bench.py --steps 2 --warmup 1 --precision $prec --no-cpu-baseline --no-roofline --no-augment-variant \
      --no-eval-variant --no-dp-variant > $OUT/$prec-$c.log 2>&1 || { echo "pmc $prec $c failed"; tail -5 $OUT/$prec-$c.log; exit 1; }
  done
  python3 tools/traffic_summary.py $OUT/$prec > $OUT/traffic_$prec.json && rm -rf $OUT/$prec || exit 1
done
if [ "$P" = both ]; then
  python3 tools/merge_traffic.py $OUT/traffic_f32.json $OUT/traffic_bf16.json > $OUT/traffic.json || exit 1
else
  cp $OUT/traffic_$P.json $OUT/traffic.json
fi
head -c 600 $OUT/traffic.json
