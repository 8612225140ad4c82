set -o pipefail
T=${TAG:-r03w}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_torch_ops.py -x -q --timeout 120 --timeout-method thread -k "roi" > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -2 gpurun_out/$T/t.log
for st in 2 30; do for sw in 4 2; do
MX_ROI_STRIP=$sw MX_PROBE_STEPS=$st timeout -k 10 300 python -u tools/bench_roialign.py > gpurun_out/$T/roi$st.$sw.log 2>&1 || { tail -20 gpurun_out/$T/roi$st.$sw.log; exit 1; }
echo "steps $st strip $sw"; grep "bwd deterministic=1\|max 5\|fwd" gpurun_out/$T/roi$st.$sw.log
done; done
timeout -k 10 300 python -u tools/hbm_ops_probe.py > gpurun_out/$T/probe.log 2>&1 || { tail -20 gpurun_out/$T/probe.log; exit 1; }
grep -E "avg_|frac" gpurun_out/$T/probe.log
