#!/bin/bash
# DELU staged epilogue operands: ubench A/B (bitwise), HJB A/B (prepare and one-stream), GPU tests.
out=gpurun_out/${1:-stage}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
tools/gpu_check.sh 240 $out/ubench_stage.log tools/ubench_x3 262144 20 stage
grep -v gpu_check $out/ubench_stage.log
for s in 0 1 0 1; do
  DPI_X3_STAGE=$s tools/gpu_check.sh 300 $out/bench_hjb_s$s.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
  grep '^{' $out/bench_hjb_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stage $s prepare', d['ms_per_step'])"
  DPI_X3_STAGE=$s tools/gpu_check.sh 300 $out/bench_hjb_one_s$s.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline --no-prepare
  grep '^{' $out/bench_hjb_one_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stage $s one-stream', d['ms_per_step'])"
done
