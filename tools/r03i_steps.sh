set -o pipefail
T=${TAG:-r03i}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/step_breakdown.py --top 70 > gpurun_out/$T/breakdown.log 2>&1 || { echo breakdown failed; tail -30 gpurun_out/$T/breakdown.log; exit 1; }
cat gpurun_out/$T/breakdown.log | cut -c1-140
