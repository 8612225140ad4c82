set -o pipefail
T=r03e
bash tools/gpu_steps.sh $T t:tests/test_gpu_x3.py t:tests/test_gpu_ops.py t:tests/test_gpu_model.py t:tests/test_gpu_ssim.py || exit 1
timeout -k 10 300 python -u tools/bench_conv.py --dtype f32 --wgrad 3,5 --reps 10 > gpurun_out/$T/bc_w.log 2>&1 || { echo bench_conv failed; tail gpurun_out/$T/bc_w.log; exit 1; }
grep -v "^$" gpurun_out/$T/bc_w.log | grep "wgrad\|==" | cut -c1-200
bash tools/gpu_steps.sh $T bench || exit 1
