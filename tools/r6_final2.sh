#!/bin/bash
# r06 final records, part 2: the DataParallel / RCCL tests, then the default bench line (reads
# profiles/r06_traffic.json and profiles/r06_in_step_table.txt) and smoke()
set -o pipefail
OUT=gpurun_out/r06f2
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_dp2.py tests/test_gpu_rccl.py tests/test_gpu_bench_ranks.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $OUT/tests.log | head; echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
python3 -c 'import json; d=json.load(open("gpurun_out/r06f2/bench.json")); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("in_step",{}).get("dominant") if d["roofline"].get("in_step") else None, d["dp_variant"]["ratio_to_headline"], d["cpu_baseline"]["value"])'
