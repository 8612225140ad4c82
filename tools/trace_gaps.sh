mkdir -p gpurun_out/tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr/raw -o t -- python3 bench.py --steps 6 --warmup 3 --precision ${PREC:-f32} --no-cpu-baseline --no-roofline > gpurun_out/tr/log 2>&1 || exit 1
f=$(find gpurun_out/tr/raw -name '*kernel_trace.csv' | head -n 1)
python3 tools/gap_analysis.py $f 40 > gpurun_out/tr/gaps.txt
cp $f gpurun_out/tr/trace.csv
rm -rf gpurun_out/tr/raw
