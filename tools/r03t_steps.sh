set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/pmc3
timeout -k 10 300 python -u -m pytest tests/test_gpu_model_f32.py -x -q --timeout 200 --timeout-method thread -k "drift or unpinned" > gpurun_out/pmc3/t.log 2>&1; tail -15 gpurun_out/pmc3/t.log

MX_PMC_PRECISION=f32 timeout -k 10 500 bash tools/pmc_traffic.sh > gpurun_out/pmc3/f32.log 2>&1 || { tail -20 gpurun_out/pmc3/f32.log; exit 1; }
cp gpurun_out/pmc_traffic/traffic.json gpurun_out/pmc3/f32.json
MX_PMC_PRECISION=bf16 timeout -k 10 500 bash tools/pmc_traffic.sh > gpurun_out/pmc3/bf16.log 2>&1 || { tail -20 gpurun_out/pmc3/bf16.log; exit 1; }
cp gpurun_out/pmc_traffic/traffic.json gpurun_out/pmc3/bf16.json
ls -la gpurun_out/pmc3
