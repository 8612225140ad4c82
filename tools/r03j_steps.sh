set -o pipefail
T=${TAG:-r03j}
bash tools/gpu_steps.sh $T t:tests/test_gpu_conv.py::test_sgd_fused_pack_equals_sgd_then_refresh t:tests/test_gpu_bn.py || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-augment-variant > gpurun_out/$T/bench_plain.log 2>&1 || { echo bench failed; tail -20 gpurun_out/$T/bench_plain.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/bench_plain.log
MX_SGD_PACK=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-augment-variant --no-roofline --precision f32 > gpurun_out/$T/bench_nopack.log 2>&1 || { echo bench failed; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/bench_nopack.log
TAG=$T bash tools/r03f_steps.sh > /dev/null || exit 1
python3 tools/step_gaps.py gpurun_out/$T/prof/p_kernel_trace.csv 30
