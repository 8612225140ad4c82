set -o pipefail
mkdir -p gpurun_out/topk
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "topk or sampler" > gpurun_out/topk/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/topk/tests.log; exit 1; }
tail -2 gpurun_out/topk/tests.log
timeout -k 10 200 python -u tools/bench_topk.py 2>&1 | tee gpurun_out/topk/bench.log
