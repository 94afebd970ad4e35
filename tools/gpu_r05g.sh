#!/bin/bash
# round 5, call g: packed Hessian reduce (thread per packed word, XCD-major points); group size
# 1 (default) against 4 (DPI_HESS_GROUP=4) — tests, bench pairs, FETCH / WRITE passes for both
set -e
out=gpurun_out/r05g; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 600 $out/hess_tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_canary.py tests/test_gpu_tanh.py tests/test_gpu_fused.py -k "hess or Hess" -m gpu -x -v --timeout 300 --timeout-method thread
DPI_HESS_GROUP=4 run 600 $out/hess_tests_g4.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_canary.py -k "hess or Hess" -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  run 200 $out/bench_gbm_hess_g1_$i.log python bench.py --workload gbm_hess --steps 30 --warmup 3 --no-cpu-baseline --no-fp32-pass
  DPI_HESS_GROUP=4 run 200 $out/bench_gbm_hess_g4_$i.log python bench.py --workload gbm_hess --steps 30 --warmup 3 --no-cpu-baseline --no-fp32-pass
done
for g in 1 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DPI_HESS_GROUP=$g timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_reduce" -d $out/pmc_g${g}_$c -o pmc \
      --output-format csv -- python bench.py --workload gbm_hess --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-pass > $out/pmc_g${g}_$c.log 2>&1
  done
done
DPI_HESS_GROUP=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace_g1 -o trace --output-format csv -- python bench.py --workload gbm_hess --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-pass > $out/trace_g1.log 2>&1
echo done
