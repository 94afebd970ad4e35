#!/bin/bash
# 128 x 128 two-blocks-per-CU split GEMM (default) vs the 256 x 128 product (DPI_X3_TILE=256).
out=gpurun_out/${1:-x3h}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
for t in 256 128 256 128; do
  DPI_X3_TILE=$t tools/gpu_check.sh 300 $out/bench_hjb_t$t.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
  grep '^{' $out/bench_hjb_t$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tile $t prepare', d['ms_per_step'])"
  DPI_X3_TILE=$t tools/gpu_check.sh 300 $out/bench_hjb_one_t$t.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline --no-prepare
  grep '^{' $out/bench_hjb_one_t$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tile $t one-stream', d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_hjb_onestream.log 2>&1
