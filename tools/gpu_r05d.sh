#!/bin/bash
# round 5, call d: GBM noise pre-pass on the prepare stream (k_noise_shared) — parity, canaries, A/B
set -e
out=gpurun_out/r05d; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 400 $out/prep_tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_canary.py -k "side_stream or gbm or prepared" -m gpu -x -v --timeout 300 --timeout-method thread
for i in 1 2; do
  run 200 $out/bench_gbm_plain_$i.log python bench.py --workload gbm --steps 50 --warmup 3 --no-cpu-baseline --no-fp32-pass
  run 200 $out/bench_gbm_prep_$i.log python bench.py --workload gbm --steps 50 --warmup 3 --no-cpu-baseline --no-fp32-pass --prepare
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_gbm_prep -o trace --output-format csv -- \
  python bench.py --workload gbm --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-pass --prepare > $out/trace_gbm_prep.log 2>&1
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done
