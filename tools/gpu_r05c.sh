#!/bin/bash
# round 5, call c: fixed padding tests + whole suite; HJB shared-rollout priority A/B (variants)
set -e
out=gpurun_out/r05c; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 300 $out/tanh_tests.log python -u -m pytest tests/test_gpu_tanh.py tests/test_gpu_parity.py -k "padded or unsupported" -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  run 200 $out/bench_hjb_base_$i.log python bench.py --workload hjb --steps 30 --warmup 3 --no-cpu-baseline --no-fp32-pass
  DPI_HIP_LIB=tools/variants/libdpi_prio3.so run 200 $out/bench_hjb_prio3_$i.log python bench.py --workload hjb --steps 30 --warmup 3 --no-cpu-baseline --no-fp32-pass
  DPI_HIP_LIB=tools/variants/libdpi_prio1.so run 200 $out/bench_hjb_prio1_$i.log python bench.py --workload hjb --steps 30 --warmup 3 --no-cpu-baseline --no-fp32-pass
done
echo done
