#!/bin/bash
# r03al: same-box A/B of the Hessian-label k_paths noise loops with 2 Philox chains per wave
# (tools/variants/libdpi_var.so, -DDPI_NOISE_UNROLL_HESS=2) against the product's 1.
set -e
out=gpurun_out/${OUT:-r03al}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
for rep in 1 2 3; do
  run 200 $out/bench_hess_u1_rep$rep.log python bench.py --workload gbm_hess --steps 10 --warmup 2 --no-cpu-baseline
  DPI_HIP_LIB=$PWD/tools/variants/libdpi_var.so run 200 $out/bench_hess_u2_rep$rep.log python bench.py --workload gbm_hess --steps 10 --warmup 2 --no-cpu-baseline
done
echo done
