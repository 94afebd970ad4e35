#!/bin/bash
# round 5, call i: the round's profile of the current binary — bench lines, kernel traces, HBM
# (FETCH_SIZE / WRITE_SIZE) and VALU PMC passes for every bench workload (tools/make_profiles.py)
set -e
out=gpurun_out/r05i; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 300 $out/bench_burgers.log python bench.py --steps 100 --warmup 10
run 300 $out/bench_burgers_cfg3.log python bench.py --workload burgers_cfg3 --steps 20 --warmup 3 --no-cpu-baseline
run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 30 --warmup 3 --no-cpu-baseline
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 50 --warmup 5 --no-cpu-baseline
run 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 30 --warmup 3 --no-cpu-baseline
P="--steps 10 --warmup 2 --no-cpu-baseline --no-fp32-pass"
for wl in burgers burgers_cfg3 hjb gbm gbm_hess; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o trace --output-format csv -- \
    python bench.py --workload $wl $P > $out/trace_$wl.log 2>&1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce|k_noise" -d $out/pmc_${wl}_$c -o pmc \
      --output-format csv -- python bench.py --workload $wl $P > $out/pmc_${wl}_$c.log 2>&1
  done
done
for wl in burgers burgers_cfg3 gbm gbm_hess; do
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_paths|k_noise" -d $out/pmc_valu_$wl -o pmc --output-format csv -- python bench.py --workload $wl $P > $out/pmc_valu_$wl.log 2>&1
done
echo done
