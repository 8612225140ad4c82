set -o pipefail
T=${TAG:-r03n}
bash tools/gpu_steps.sh $T t:tests/test_gpu_ops.py || exit 1
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/bench_roialign.py > gpurun_out/$T/roi.log 2>&1 || { echo roi failed; tail gpurun_out/$T/roi.log; exit 1; }
grep "fwd" gpurun_out/$T/roi.log
MX_ROI_FWD_WIN=0 timeout -k 10 300 python -u tools/bench_roialign.py > gpurun_out/$T/roi0.log 2>&1 || exit 1
grep "fwd" gpurun_out/$T/roi0.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-augment-variant > gpurun_out/$T/bench_plain.log 2>&1 || { echo bench failed; tail -20 gpurun_out/$T/bench_plain.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/bench_plain.log
