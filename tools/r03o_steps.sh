set -o pipefail
T=${TAG:-r03o}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/graph_vs_eager.py > gpurun_out/$T/gve1.log 2>&1 || { tail -20 gpurun_out/$T/gve1.log; exit 1; }
cat gpurun_out/$T/gve1.log
MX_GRAD_CHAIN=0 timeout -k 10 300 python -u tools/graph_vs_eager.py > gpurun_out/$T/gve0.log 2>&1 || { tail -20 gpurun_out/$T/gve0.log; exit 1; }
cat gpurun_out/$T/gve0.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread -k residual > gpurun_out/$T/x3.log 2>&1; tail -3 gpurun_out/$T/x3.log
