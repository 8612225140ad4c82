set -o pipefail
T=${TAG:-r03l}
bash tools/gpu_steps.sh $T t:tests/test_gpu_ops.py t:tests/test_gpu_rpn_canvas.py t:tests/test_gpu_graphs.py t:tests/test_gpu_model.py t:tests/test_gpu_dp.py t:tests/test_gpu_dp2.py t:tests/test_gpu_model_f32.py || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-augment-variant > gpurun_out/$T/bench_plain.log 2>&1 || { echo bench failed; tail -20 gpurun_out/$T/bench_plain.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/bench_plain.log
TAG=$T bash tools/r03f_steps.sh > /dev/null || exit 1
cat gpurun_out/$T/step_summary.txt
python3 tools/step_gaps.py gpurun_out/$T/prof/p_kernel_trace.csv 30 | head -8
mkdir -p gpurun_out/$T && timeout -k 10 300 python -u tools/bench_roialign.py > gpurun_out/$T/roi.log 2>&1; tail -12 gpurun_out/$T/roi.log
