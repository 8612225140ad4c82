#!/bin/bash
# r06 final records, part 4: full GPU suite, smoke, a 10-step kernel trace
# (per-step table + concurrency), then the default bench line
set -o pipefail
OUT=gpurun_out/r06f7
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python3 bench.py --precision f32 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-augment-variant \
  --no-eval-variant --no-dp-variant > "$OUT/prof.log" 2>&1 || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
for f in $(find "$OUT/prof" -name '*_stats.csv'); do cp "$f" "$OUT/"; done
tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_concurrency.py "$tr" 10 > "$OUT/step_concurrency.txt" 2>&1
python3 tools/prof_steps.py "$OUT/prof" --steps 10 --out "$OUT/step_kernels.csv" > "$OUT/step_kernels.log" 2>&1
rm -rf "$OUT/prof"
head -4 "$OUT/step_concurrency.txt"
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
python3 -c 'import json; d=json.load(open("gpurun_out/r06f7/bench.json")); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["dp_variant"]["ratio_to_headline"], d["bf16_variant"]["value"])'
