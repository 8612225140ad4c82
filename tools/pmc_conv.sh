#!/bin/bash
# PMC passes over one conv shape / pass (tools/conv_one.py), one rocprofv3 run per counter group.
# Usage: SHAPE=2,100,168,128,512,1,1,0 PASSES="fwd" DTYPE=f32 TAG=l2c3 bash tools/pmc_conv.sh
set -o pipefail
TAG=${TAG:-pmc}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE=${SHAPE:-2,200,336,256,256,3,1,1}
for pass in ${PASSES:-fwd}; do
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/${pass}_$i -o p -- \
      python3 tools/conv_one.py --shape $SHAPE --pass $pass --reps 5 --dtype ${DTYPE:-f32} > $OUT/${pass}_$i.log 2>&1 \
      || { echo "pmc $pass group $i failed"; tail -5 $OUT/${pass}_$i.log; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
