set -o pipefail
export TMPDIR=/tmp
SHAPE=2,200,336,256,256,3,1,1 PASSES="wgrad fwd" DTYPE=f32 TAG=p2w timeout -k 10 500 bash tools/pmc_conv.sh > gpurun_out/pmc_p2w.log 2>&1 || { echo pmc failed; tail -20 gpurun_out/pmc_p2w.log; exit 1; }
tail -60 gpurun_out/pmc_p2w.log
timeout -k 10 300 python -u tools/bench_conv.py --dtype f32 --only "P2 3x3" --wgrad 3,4 --wtarget 0,256,1024 --reps 10 > gpurun_out/bc_w.log 2>&1 || { echo bench_conv failed; tail gpurun_out/bc_w.log; exit 1; }
cat gpurun_out/bc_w.log
timeout -k 10 300 python -u bench.py --precision f32 --no-cpu-baseline --no-augment-variant --no-roofline > gpurun_out/ab_side1.log 2>&1 || { echo bench failed; tail gpurun_out/ab_side1.log; exit 1; }
MX_SIDE_WGRAD=0 timeout -k 10 300 python -u bench.py --precision f32 --no-cpu-baseline --no-augment-variant --no-roofline > gpurun_out/ab_side0.log 2>&1 || { echo bench failed; tail gpurun_out/ab_side0.log; exit 1; }
tail -1 gpurun_out/ab_side1.log | cut -c1-160
tail -1 gpurun_out/ab_side0.log | cut -c1-160
