#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench line, rocprofv3 kernel stats of a short bench.
# Usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_check.sh <tag> [tests|bench|prof ...]
set -o pipefail
TAG=${1:-run}; shift
STEPS=${*:-tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -40 "$OUT/tests.log"; exit 1; }
      tail -3 "$OUT/tests.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { echo "smoke failed rc=$?"; tail -30 "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 \
        || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.log"; exit 1; }
      tail -1 "$OUT/bench.log" ;;
    script)
      timeout -k 10 400 python -u bench.py --mode script --steps 20 --warmup 5 > "$OUT/script.log" 2>&1 \
        || { echo "script bench failed rc=$?"; tail -30 "$OUT/script.log"; exit 1; }
      tail -1 "$OUT/script.log" ;;
    breakdown)
      timeout -k 10 300 python -u tools/step_breakdown.py --top 60 > "$OUT/breakdown.log" 2>&1 \
        || { echo "breakdown failed rc=$?"; tail -30 "$OUT/breakdown.log"; exit 1; }
      tail -5 "$OUT/breakdown.log" ;;
    benchfast)
      timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 \
        || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.log"; exit 1; }
      tail -1 "$OUT/bench.log" ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
        python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dp-variant > "$OUT/prof.log" 2>&1 \
        || { echo "prof failed rc=$?"; tail -30 "$OUT/prof.log"; exit 1; }
      for f in $(find "$OUT/prof" -name '*_stats.csv'); do cp "$f" "$OUT/"; done
      python3 tools/prof_steps.py "$OUT/prof" --steps 10 --out "$OUT/step_kernels.csv" > "$OUT/step_kernels.log" 2>&1 \
        || { echo "prof_steps failed"; tail -5 "$OUT/step_kernels.log"; }
      tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
      [ -n "$tr" ] && python3 tools/step_gaps.py "$tr" 20 > "$OUT/step_gaps.log" 2>&1
      [ -n "$tr" ] && python3 tools/step_concurrency.py "$tr" 10 > "$OUT/step_concurrency.log" 2>&1
      [ -n "$tr" ] && gzip -c "$tr" > "$OUT/kernel_trace.csv.gz"
      rm -rf "$OUT/prof"
      tail -1 "$OUT/prof.log" ;;
    pmc)
      timeout -k 10 500 bash tools/pmc_traffic.sh > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; tail -20 "$OUT/pmc.log"; exit 1; }
      cp gpurun_out/pmc_traffic/traffic.json "$OUT/traffic.json"; tail -3 "$OUT/pmc.log" ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_check $TAG done"
