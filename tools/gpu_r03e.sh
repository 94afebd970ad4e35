#!/bin/bash
# r03e: GBM phase timings + two PMC passes of the network-phase kernels.
set -e
out=gpurun_out/r03e
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_check.sh 300 $out/perf_gbm.log python tools/perf_gbm.py
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex k_paths -d $out/pg1 -o pg1 --output-format csv -- python tools/pmc_gbm.py > $out/pg1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM --kernel-include-regex k_paths -d $out/pg2 -o pg2 --output-format csv -- python tools/pmc_gbm.py > $out/pg2.log 2>&1
echo done
