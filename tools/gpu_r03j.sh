#!/bin/bash
# r03j part A: round-end check of the committed binary — counter list, the whole -m gpu suite, the
# bench line of every workload, the GBM product PMC passes.
set -e
out=gpurun_out/r03j
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory" "$2"; then echo "fault in $2"; exit 3; fi; }
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1 || true
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run 300 $out/bench_burgers.log python bench.py
run 300 $out/bench_burgers_cfg3.log python bench.py --workload burgers_cfg3
run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
run 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 10 --warmup 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex k_paths -d $out/pg1 -o pg1 --output-format csv -- python tools/pmc_gbm.py > $out/pg1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM --kernel-include-regex k_paths -d $out/pg2 -o pg2 --output-format csv -- python tools/pmc_gbm.py > $out/pg2.log 2>&1
echo done
