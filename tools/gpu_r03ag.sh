#!/bin/bash
# r03ag: same-box A/B of the first-order k_paths noise loops with 4 Philox chains per wave
# (tools/variants/libdpi_u4.so, -DDPI_NOISE_UNROLL_FO=4) against the product's 2.
set -e
out=gpurun_out/${OUT:-r03ag}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
for rep in 1 2 3; do
  run 200 $out/bench_burgers_u2_rep$rep.log python bench.py --no-cpu-baseline
  DPI_HIP_LIB=$PWD/tools/variants/libdpi_u4.so run 200 $out/bench_burgers_u4_rep$rep.log python bench.py --no-cpu-baseline
done
run 200 $out/bench_cfg3_u2.log python bench.py --workload burgers_cfg3 --no-cpu-baseline
DPI_HIP_LIB=$PWD/tools/variants/libdpi_u4.so run 200 $out/bench_cfg3_u4.log python bench.py --workload burgers_cfg3 --no-cpu-baseline

run 200 $out/perf_host_burgers.log python tools/perf_host.py burgers
echo done
