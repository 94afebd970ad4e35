# PMC passes over tools/pmc_probe.py (k_paths only); summaries -> gpurun_out/pmc*/
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex k_paths -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python tools/pmc_probe.py > gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS --kernel-include-regex k_paths -d gpurun_out/pmc2 -o pmc2 --output-format csv -- python tools/pmc_probe.py > gpurun_out/pmc2.log 2>&1
