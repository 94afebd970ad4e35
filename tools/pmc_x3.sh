#!/bin/bash
# PMC passes over the product GEMM of tools/ubench_x3 (one rocprofv3 run per pass).
out=gpurun_out/${1:-x3pmc}; mkdir -p $out; export TMPDIR=/tmp
p=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  p=$((p+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $out/p$p -o pmc --output-format csv -- tools/ubench_x3 262144 5 prod > $out/p$p.log 2>&1 || { echo "pass $p failed"; exit 1; }
done
echo done
