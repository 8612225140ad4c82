set -o pipefail
T=${TAG:-r03f}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o p -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --precision f32 --no-augment-variant > gpurun_out/$T/bench.log 2>&1 || { echo prof failed; tail -30 gpurun_out/$T/bench.log; exit 1; }
python3 tools/prof_steps.py gpurun_out/$T/prof --steps 10 --out gpurun_out/$T/step_kernels.csv 2> gpurun_out/$T/step_summary.txt || exit 1
cat gpurun_out/$T/step_summary.txt
head -45 gpurun_out/$T/step_kernels.csv | cut -c1-160
