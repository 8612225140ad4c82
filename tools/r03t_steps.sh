set -o pipefail
T=${TAG:-r03deg}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_model_f32.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/t.log 2>&1 || { tail -30 gpurun_out/$T/t.log; exit 1; }
tail -2 gpurun_out/$T/t.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/$T/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['bf16_variant']['value'], d['augment_variant']['value'])
"
