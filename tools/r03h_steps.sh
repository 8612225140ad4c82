set -o pipefail
T=${TAG:-r03h}
bash tools/gpu_steps.sh $T t:tests/test_gpu_ops.py t:tests/test_gpu_conv.py::test_sgd_fused_pack_equals_sgd_then_refresh t:tests/test_gpu_conv.py::test_weight_packer_batched_matches_single_and_tracks_versions t:tests/test_gpu_bn.py t:tests/test_gpu_model.py t:tests/test_gpu_graphs.py t:tests/test_gpu_dp.py t:tests/test_gpu_dp2.py t:tests/test_gpu_model_f32.py t:tests/test_gpu_rpn_canvas.py || exit 1
TAG=$T bash tools/r03f_steps.sh
TAG=$T bash tools/r03i_steps.sh
