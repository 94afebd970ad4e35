#!/bin/bash
# r03d: GBM 8-wave sweep — GBM / Hessian parity tests, then the gbm bench and a kernel trace.
set -e
out=gpurun_out/r03d
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 600 $out/gbm_tests.log python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_range.py -k "gbm or GBM or hess"
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_gbm -o trace --output-format csv -- \
  python bench.py --workload gbm --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_gbm.log 2>&1
echo done
