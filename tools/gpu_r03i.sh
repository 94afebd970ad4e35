#!/bin/bash
# r03i: k_baseline with every weight slice prefetched — parity tests that read the baseline
# (Burgers / OU MLP / GBM goldens and oracle checks), the Burgers and GBM benches, a Burgers trace.
set -e
out=gpurun_out/r03i
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory" "$2"; then echo "fault in $2"; exit 3; fi; }
run 900 $out/parity_tests.log python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_dataset.py tests/test_capi.py
run 300 $out/bench_burgers.log python bench.py
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_burgers -o trace --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_burgers.log 2>&1
echo done
