#!/bin/bash
# round 5, call l: k_baseline chain prefetch with compile-time register sets; sweep unroll A/B
set -e
out=gpurun_out/r05l; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
DPI_HIP_LIB=tools/variants/libdpi_bstamps.so run 200 $out/base_stamps.txt python tools/base_stamps.py
DPI_HIP_LIB=tools/variants/libdpi_bstamps_u2.so run 200 $out/base_stamps_u2.txt python tools/base_stamps.py
run 600 $out/gpu_tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_tanh.py tests/test_gpu_canary.py -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
  run 200 $out/bench_burgers_$i.log python bench.py --steps 100 --warmup 10 --no-cpu-baseline
  run 200 $out/bench_gbm_$i.log python bench.py --workload gbm --steps 50 --warmup 5 --no-cpu-baseline
  DPI_HIP_LIB=tools/variants/libdpi_sweep_u2.so run 200 $out/bench_gbm_u2_$i.log python bench.py --workload gbm --steps 50 --warmup 5 --no-cpu-baseline
done
echo done
