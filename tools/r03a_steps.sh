set -o pipefail
T=${TAG:-r03c}
bash tools/gpu_steps.sh $T t:tests/test_gpu_x3.py t:tests/test_gpu_conv.py t:tests/test_gpu_ssim.py t:tests/test_transform.py t:tests/test_torch_ops.py t:tests/test_gpu_unet_train.py t:tests/test_jpeg.py || exit 1
bash tools/gpu_steps.sh $T bench || exit 1
timeout -k 10 300 python -u tools/roi_order_probe.py > gpurun_out/$T/roi_order.log 2>&1 || { echo roi probe failed; tail -20 gpurun_out/$T/roi_order.log; exit 1; }
tail -4 gpurun_out/$T/roi_order.log
bash tools/trace_gaps.sh || { echo trace failed; exit 1; }
head -30 gpurun_out/tr/gaps.txt
