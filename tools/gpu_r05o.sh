#!/bin/bash
# round 5, call o: k_baseline owner sums with every slice read issued first
set -e
out=gpurun_out/r05o; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
DPI_HIP_LIB=tools/variants/libdpi_bstamps.so run 200 $out/base_stamps.txt python tools/base_stamps.py
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
  run 200 $out/bench_burgers_$i.log python bench.py --steps 100 --warmup 10 --no-cpu-baseline
  run 200 $out/bench_gbm_$i.log python bench.py --workload gbm --steps 50 --warmup 5 --no-cpu-baseline
  run 200 $out/bench_gbm_hess_$i.log python bench.py --workload gbm_hess --steps 30 --warmup 3 --no-cpu-baseline
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $out/trace_burgers -o trace --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-pass > $out/trace_burgers.log 2>&1
echo done
