set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_stream_guard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05c/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05c/tests.log; exit 1; }
tail -2 gpurun_out/r05c/tests.log
bash tools/ab_env.sh r05c MX_WGRAD_FORK_EARLY 0 1 3 30 || exit 1
bash tools/ab_env.sh r05c DEBUG_HIP_FORCE_GRAPH_QUEUES 2 1 1 30 || exit 1
bash tools/gpu_check.sh r05c prof
