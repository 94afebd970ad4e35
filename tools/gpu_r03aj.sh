#!/bin/bash
# r03aj: same-box A/B of GBM's k_paths noise loops with 4 Philox chains per wave
# (tools/variants/libdpi_var.so, -DDPI_NOISE_UNROLL_GBM=4) against the product's 2.
set -e
out=gpurun_out/${OUT:-r03aj}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
for rep in 1 2 3; do
  run 200 $out/bench_gbm_u2_rep$rep.log python bench.py --workload gbm --steps 20 --warmup 3 --no-cpu-baseline
  DPI_HIP_LIB=$PWD/tools/variants/libdpi_var.so run 200 $out/bench_gbm_u4_rep$rep.log python bench.py --workload gbm --steps 20 --warmup 3 --no-cpu-baseline
done
echo done
