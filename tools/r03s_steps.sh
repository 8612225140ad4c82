set -o pipefail
T=${TAG:-r03s}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_torch_ops.py -x -q --timeout 120 --timeout-method thread -k "roi" > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -2 gpurun_out/$T/t.log
timeout -k 10 300 python -u tools/bench_roialign.py > gpurun_out/$T/roi.log 2>&1 || { tail -20 gpurun_out/$T/roi.log; exit 1; }
grep -v amdgpu gpurun_out/$T/roi.log | tail -15
timeout -k 10 300 python -u tools/hbm_ops_probe.py > gpurun_out/$T/probe.log 2>&1 || { tail -20 gpurun_out/$T/probe.log; exit 1; }
grep -E "avg_|frac" gpurun_out/$T/probe.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/$T/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], json.dumps(d['hbm_ops'])[:700])
"
