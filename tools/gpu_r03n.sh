#!/bin/bash
# r03n: GBM sweep with z_0 software-pipelined — GBM/Hessian parity tests, gbm and gbm_hess benches.
set -e
out=gpurun_out/r03n
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory" "$2"; then echo "fault in $2"; exit 3; fi; }
run 600 $out/gbm_tests.log python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_range.py -k "gbm or GBM or hess"
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
run 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 10 --warmup 2
run 300 $out/perf_gbm.log python tools/perf_gbm.py
echo done
