#!/bin/bash
# r06z: tile-order tests, A/B of MX_CONV_NMAJOR (0 = M-major, 1 = auto), x3 kernels' PMC traffic both ways
set -o pipefail
OUT=gpurun_out/r06z
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_x3p.py tests/test_gpu_model.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests.log | head; echo "tests rc=$rc: stopping"; exit $rc; fi
bash tools/ab_multi.sh r06z_ab 3 30 "MX_CONV_NMAJOR=0" "MX_CONV_NMAJOR=1" || exit 1
for mode in 0 1; do
  MX_CONV_NMAJOR=$mode MX_PMC_PRECISION=f32 bash tools/pmc_traffic.sh > $OUT/pmc_$mode.log 2>&1 || { echo "pmc $mode failed"; tail -5 $OUT/pmc_$mode.log; exit 1; }
  cp gpurun_out/pmc_traffic/traffic.json $OUT/traffic_$mode.json
done
python3 - <<'PY'
import json
a = json.load(open("gpurun_out/r06z/traffic_0.json"))["kernels"]
b = json.load(open("gpurun_out/r06z/traffic_1.json"))["kernels"]
for k in sorted(set(a) & set(b)):
    if "conv_x3_buf" in k:
        print(f"{a[k]['bytes_per_launch']/1e6:9.2f} -> {b[k]['bytes_per_launch']/1e6:9.2f} MB  {k[:70]}")
PY
