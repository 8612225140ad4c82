#!/bin/bash
# A/B on one box: concurrent small levels (MX_FPN_STREAMS / MX_RPN_STREAMS) on vs off, train + eval.
set -o pipefail
OUT=gpurun_out/r03z_ab; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --precision f32 --no-cpu-baseline --no-roofline --no-augment-variant \
    > $OUT/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -20 $OUT/$tag.log; exit 1; }
  python3 - "$OUT/$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[2], "train", d["value"], d["ms_per_step"], "eval", d.get("eval_variant", {}).get("value"),
      "eval_restored", d.get("eval_restored_variant", {}).get("value"), flush=True)
PY
}
run on1 MX_FPN_STREAMS=1 && run off1 MX_FPN_STREAMS=0 MX_RPN_STREAMS=0 && run on2 MX_FPN_STREAMS=1 && \
  run off2 MX_FPN_STREAMS=0 MX_RPN_STREAMS=0
