#!/bin/bash
# The wide-dimension tests first (new kernels), then the whole GPU suite and the bench lines they touch.
# usage: tools/gpu_wide.sh <tag>     outputs under gpurun_out/<tag>/
out=gpurun_out/${1:-wide}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 300 $out/gpu_wide.log python -u -m pytest tests/test_gpu_wide.py -v --timeout 120 --timeout-method thread
tools/gpu_check.sh 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tools/gpu_check.sh 300 $out/bench_burgers.log python bench.py --no-cpu-baseline
tools/gpu_check.sh 300 $out/bench_burgers_nx256.log python bench.py --workload burgers_nx256 --no-cpu-baseline
tools/gpu_check.sh 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3 --no-cpu-baseline
