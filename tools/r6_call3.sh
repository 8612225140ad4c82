#!/bin/bash
# r06c: A/B (single-model runs) of the conv tail, the RPN helper thread and the deferred-wgrad one-graph
# backward; then the second-model crash probe (keep / graphs / del: the crashing one last).
set -o pipefail
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="MX_CONV_TAIL=0 MX_RPN_TARGETS_THREAD=0 MX_SEG_GRAPHS=0"
bash tools/ab_multi.sh r06c_ab 3 40 "$B" "MX_CONV_TAIL=1 MX_RPN_TARGETS_THREAD=0 MX_SEG_GRAPHS=0" \
  "MX_CONV_TAIL=0 MX_RPN_TARGETS_THREAD=1 MX_SEG_GRAPHS=0" "MX_CONV_TAIL=0 MX_RPN_TARGETS_THREAD=0 MX_SEG_GRAPHS=1" || exit $?
for m in keep graphs del; do
  timeout -k 10 240 python -u tools/seg_probe.py --mode $m > $OUT/probe_$m.log 2>&1
  rc=$?
  echo "probe $m rc=$rc: $(tail -1 $OUT/probe_$m.log)"
  [ $rc -ne 0 ] && exit $rc
done
