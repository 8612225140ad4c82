#!/bin/bash
# r06o: host timeline of the DataParallel step vs the plain step (tools/dp_host_timeline.py)
set -o pipefail
OUT=gpurun_out/r06o
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/dp_host_timeline.py --steps 10 > $OUT/timeline.txt 2>&1 && MX_DP_NMS_FLAG=0 timeout -k 10 400 python -u tools/dp_host_timeline.py --steps 10 > $OUT/timeline_noflag.txt 2>&1 || { echo "timeline failed rc=$?"; tail -30 $OUT/timeline*.txt; exit 1; }
tail -20 $OUT/timeline.txt
tail -14 $OUT/timeline_noflag.txt
