#!/bin/bash
# r03p: HJB prepare-stream rollout grid size A/B on one box (blocks per CU per grid), alternating.
set -e
out=gpurun_out/r03p
mkdir -p $out
for rep in 1 2; do
  for k in ${KS:-1 2 3}; do
    DPI_PIS_PREP_PER_CU=$k tools/gpu_check.sh 300 $out/bench_hjb_prep${k}_rep${rep}.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
  done
done
echo done
