set -o pipefail
T=${TAG:-r03split2}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_torch_ops.py -x -q --timeout 120 --timeout-method thread -k "roi" > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -1 gpurun_out/$T/t.log
for sp in 4 8 4 8; do
MX_ROI_SPLIT=$sp timeout -k 10 300 python -u tools/hbm_ops_probe.py > gpurun_out/$T/p$sp.log 2>&1 || { tail -20 gpurun_out/$T/p$sp.log; exit 1; }
echo "split $sp $(grep -m1 avg_launch_us gpurun_out/$T/p$sp.log)"
done
for sp in 1 4 8; do
MX_ROI_SPLIT=$sp timeout -k 10 300 python -u tools/bench_roialign.py > gpurun_out/$T/roi$sp.log 2>&1 || exit 1
echo "hot split $sp $(grep '^fwd' gpurun_out/$T/roi$sp.log)"
done
