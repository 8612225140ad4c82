#!/bin/bash
# Ad-hoc GPU-box steps (each under its own time limit, stop at the first failure).
# Usage: gpurun -- bash tools/gpu_steps.sh <tag> <step> [<step> ...]
#   t:<pytest node or file>   run tests
#   eval | eval_restored      bench.py --mode ... (short)
#   rehearse                  bench.py with 2 gloo ranks on cuda:0 (multi-rank code path)
#   bench                     default bench.py
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
n=0
for s in "$@"; do
  n=$((n+1))
  case $s in
    t:*)
      timeout -k 10 600 python -u -m pytest "${s#t:}" -x -v --timeout 300 --timeout-method thread > "$OUT/t$n.log" 2>&1 \
        || { echo "tests $s failed"; tail -40 "$OUT/t$n.log"; exit 1; }
      tail -2 "$OUT/t$n.log" ;;
    eval|eval_restored|unet_train|jpeg)
      timeout -k 10 400 python -u bench.py --mode $s --steps 20 --warmup 3 > "$OUT/$s.log" 2>&1 \
        || { echo "$s failed"; tail -30 "$OUT/$s.log"; exit 1; }
      tail -1 "$OUT/$s.log" ;;
    rehearse)
      MX_BENCH_REHEARSE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --precision f32 \
        --no-roofline > "$OUT/rehearse.log" 2>&1 || { echo "rehearse failed"; tail -30 "$OUT/rehearse.log"; exit 1; }
      tail -1 "$OUT/rehearse.log" ;;
    hbm)
      timeout -k 10 300 python -u bench.py --precision f32 --no-augment-variant --no-eval-variant --no-dp-variant --no-cpu-baseline \
        --steps 10 --warmup 3 > "$OUT/hbm.log" 2>&1 || { echo "hbm bench failed"; tail -30 "$OUT/hbm.log"; exit 1; }
      tail -1 "$OUT/hbm.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d.get('hbm_ops')))" ;;
    script)
      timeout -k 10 400 python -u bench.py --mode script --steps 20 --warmup 5 > "$OUT/script.log" 2>&1 \
        || { echo "script bench failed"; tail -30 "$OUT/script.log"; exit 1; }
      tail -1 "$OUT/script.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 \
        || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
      tail -1 "$OUT/bench.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_steps $TAG done"
