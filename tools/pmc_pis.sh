#!/bin/bash
# PMC passes over the PISGradNet side kernels (k_pis_final, k_pis_time, k_pis_base_final) of the HJB bench.
out=gpurun_out/${1:-pmcpis}; mkdir -p $out; export TMPDIR=/tmp
p=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_pis_final|k_pis_time|k_pis_base" -d $out/p$p -o pmc --output-format csv -- \
    python bench.py --workload hjb --steps 4 --warmup 1 --no-cpu-baseline --no-prepare > $out/p$p.log 2>&1 || echo "pass $p rc=$?"
done
echo done
