#!/bin/bash
# r06q: torch-level op table + call sites of one steady-state train step
set -o pipefail
OUT=gpurun_out/r06q
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/torch_ops_profile.py --sites > $OUT/ops.txt 2>&1 || { echo "ops profile failed rc=$?"; tail -30 $OUT/ops.txt; exit 1; }
wc -l $OUT/ops.txt
