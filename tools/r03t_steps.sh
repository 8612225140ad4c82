set -o pipefail
T=${TAG:-r03ds}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_rpn_canvas.py tests/test_gpu_graphs.py tests/test_gpu_dp.py tests/test_gpu_dp2.py tests/test_gpu_model_f32.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -1 gpurun_out/$T/t.log
for v in 0 1 0 1; do
MX_DS_STREAMS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-augment-variant --no-eval-variant --precision f32 --steps 30 > gpurun_out/$T/b$v.log 2>&1 || { tail -20 gpurun_out/$T/b$v.log; exit 1; }
echo "ds $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/b$v.log)"
done
