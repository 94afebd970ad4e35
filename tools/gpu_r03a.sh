#!/bin/bash
# r03a: GPU tests, Burgers bench lines (configs[1] and configs[3] at N = 1), configs[3] PMC passes.
set -e
out=gpurun_out/r03a
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run 300 $out/bench_burgers.log python bench.py
run 300 $out/bench_burgers_cfg3.log python bench.py --workload burgers_cfg3
wl=burgers_cfg3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex k_paths -d $out/pmc_valu_$wl -o pmc --output-format csv -- \
  python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_valu_$wl.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce" -d $out/pmc_${wl}_$c -o pmc \
    --output-format csv -- python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_${wl}_$c.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o trace --output-format csv -- \
  python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_$wl.log 2>&1
echo done
