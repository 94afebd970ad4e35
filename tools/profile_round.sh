#!/bin/bash
# Round profile: bench lines for the three workloads, kernel-trace stats and separate PMC passes
# (FETCH_SIZE / WRITE_SIZE per MI355X_MICROARCH.md, one counter block per pass) of the bench.
# usage: tools/profile_round.sh <tag>     outputs under gpurun_out/<tag>/
set -e
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_check.sh 300 $out/bench_burgers.log python bench.py --steps 50 --warmup 5
tools/gpu_check.sh 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
tools/gpu_check.sh 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
tools/gpu_check.sh 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 10 --warmup 2
for wl in burgers gbm gbm_hess hjb; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o trace --output-format csv -- \
    python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_$wl.log 2>&1
done
for wl in burgers hjb gbm gbm_hess; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce" -d $out/pmc_${wl}_$c -o pmc \
      --output-format csv -- python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_${wl}_$c.log 2>&1
  done
done
