set -o pipefail
mkdir -p gpurun_out/tr
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/raw -o t -- python3 bench.py --steps 6 --warmup 3 --precision f32 --no-cpu-baseline --no-roofline --no-augment-variant > gpurun_out/tr/log 2>&1 || { tail gpurun_out/tr/log; exit 1; }
f=$(find gpurun_out/tr/raw -name '*kernel_trace.csv' | head -n 1)
python3 tools/step_gaps.py $f 20 > gpurun_out/tr/gaps.txt
python3 tools/gap_analysis.py $f 20 > gpurun_out/tr/gaps2.txt 2>&1 || true
rm -rf gpurun_out/tr/raw
head -50 gpurun_out/tr/gaps.txt
