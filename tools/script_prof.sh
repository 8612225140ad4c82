#!/bin/bash
# Kernel trace of bench.py --mode script (the drop-in script's loop) cut to its timed steps, next to
# the same for the bench's own step: per-step kernel tables + idle-gap summaries for the A/B.
# Usage: gpurun -- bash tools/script_prof.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/sp -o sp -- \
  python3 bench.py --mode script --steps 10 --warmup 5 > $OUT/script_prof.log 2>&1 || { echo "script prof failed"; tail -20 $OUT/script_prof.log; exit 1; }
python3 tools/prof_steps.py $OUT/sp --steps 10 --out $OUT/script_step_kernels.csv > $OUT/script_steps.log 2>&1
tr=$(find $OUT/sp -name '*kernel_trace.csv' | head -n 1)
[ -n "$tr" ] && python3 tools/step_gaps.py "$tr" 20 > $OUT/script_gaps.log 2>&1
[ -n "$tr" ] && gzip -c "$tr" > $OUT/script_trace.csv.gz
rm -rf $OUT/sp
tail -2 $OUT/script_steps.log; tail -5 $OUT/script_gaps.log
