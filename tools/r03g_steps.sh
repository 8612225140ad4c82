set -o pipefail
T=${TAG:-r03g}
bash tools/gpu_steps.sh $T t:tests/test_gpu_ops.py t:tests/test_gpu_graphs.py || exit 1
bash tools/r03f_steps.sh
