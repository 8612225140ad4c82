set -o pipefail
T=${TAG:-r03r}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/bench_conv.py --dtype f32 --graph --only thin --tiles 0x0,64x64,64x128,128x128 --stages 0,3,5 --splits 0,1 > gpurun_out/$T/thin.log 2>&1 || { tail -20 gpurun_out/$T/thin.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/thin.log
