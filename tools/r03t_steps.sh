set -o pipefail
T=${TAG:-r03m32}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -2 gpurun_out/$T/t.log
timeout -k 10 500 python -u tools/bench_conv.py --dtype f32 --graph --stages 0,7 --tiles 0x0,128x128 > gpurun_out/$T/bc.log 2>&1 || { tail -20 gpurun_out/$T/bc.log; exit 1; }
grep -v amdgpu gpurun_out/$T/bc.log
