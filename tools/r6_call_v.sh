#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06v
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/opt_host_profile.py > $OUT/opt.txt 2>&1 || { echo "failed rc=$?"; tail -20 $OUT/opt.txt; exit 1; }
grep -v "^$" $OUT/opt.txt | head -40
