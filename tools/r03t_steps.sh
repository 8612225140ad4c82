set -o pipefail
T=${TAG:-r03sgd}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_bn.py tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "sgd or roi" > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -1 gpurun_out/$T/t.log
bash tools/gpu_check.sh $T prof > gpurun_out/$T/prof.out 2>&1 || { tail -20 gpurun_out/$T/prof.out; exit 1; }
grep -E "sgd_pack|roi_align_fwd|roi_bwd" gpurun_out/$T/step_kernels.csv | cut -c1-60,150-
tail -1 gpurun_out/$T/step_kernels.log
