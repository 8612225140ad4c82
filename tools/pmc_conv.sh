set -o pipefail
mkdir -p gpurun_out/pmc
cd /root/repo
for pass in ${PASSES:-fwd wgrad}; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc/$pass -o p -- python3 tools/conv_one.py --pass $pass --reps 5 > gpurun_out/pmc/$pass.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc/${pass}2 -o p -- python3 tools/conv_one.py --pass $pass --reps 5 > gpurun_out/pmc/${pass}2.log 2>&1 || exit 1
done
find gpurun_out/pmc -name "*counter_collection.csv" | head
