#!/bin/bash
# HBM traffic of the step's kernels from PMC counters (MI355X_MICROARCH.md §HBM: FETCH_SIZE and
# WRITE_SIZE in separate passes; gfx950 FETCH_SIZE counts half of a wide streaming read).
# Writes gpurun_out/pmc_traffic/traffic.json (per kernel: launches, mean bytes per launch).
set -o pipefail
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
export TMPDIR=/tmp MX_GRAPHS=0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o p -- \
    python3 bench.py --steps 2 --warmup 1 --precision ${MX_PMC_PRECISION:-f32} --no-cpu-baseline --no-roofline > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 tools/traffic_summary.py $OUT > $OUT/traffic.json && rm -rf $OUT/FETCH_SIZE $OUT/WRITE_SIZE && head -c 600 $OUT/traffic.json
