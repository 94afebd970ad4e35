#!/bin/bash
# round 5, first call: the new range-guard / canary tests, the whole GPU suite, the guard's cost on Burgers
set -e
out=gpurun_out/r05a; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 600 $out/new_tests.log python -u -m pytest tests/test_gpu_range.py tests/test_gpu_canary.py tests/test_gpu_fused.py -m gpu -x -v --timeout 300 --timeout-method thread
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
for i in 1 2; do
  for m in off step region; do
    run 200 $out/bench_burgers_${m}_$i.log python bench.py --no-cpu-baseline --range-check $m
  done
done
run 300 $out/bench_hjb_step.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
run 300 $out/bench_hjb_off.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --range-check off
