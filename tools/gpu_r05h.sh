#!/bin/bash
# round 5, call h: Hessian labels with one workgroup per block again (grouping removed), packed
# block sums, the thread-per-packed-word XCD-major reduce — tests, bench, FETCH / WRITE, trace
set -e
out=gpurun_out/r05h; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 600 $out/hess_tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_canary.py tests/test_gpu_tanh.py tests/test_gpu_fused.py tests/test_gpu_dataset.py -k "hess or Hess" -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  run 200 $out/bench_gbm_hess_$i.log python bench.py --workload gbm_hess --steps 30 --warmup 3 --no-cpu-baseline --no-fp32-pass
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_reduce" -d $out/pmc_$c -o pmc \
    --output-format csv -- python bench.py --workload gbm_hess --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-pass > $out/pmc_$c.log 2>&1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python bench.py --workload gbm_hess --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-pass > $out/trace.log 2>&1
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done
