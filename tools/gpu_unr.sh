#!/bin/bash
# PISGradNet rollout unroll 4 (default) vs 2 (DPI_PIS_UNROLL=2): PIS tests, HJB A/B under the prepare schedule.
out=gpurun_out/${1:-unr}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pis or hjb or ou or side_stream or graph"
grep -E "passed|failed" $out/gpu_tests.log | tail -1
for u in 2 4 2 4 2 4; do
  DPI_PIS_UNROLL=$u tools/gpu_check.sh 300 $out/bench_hjb_u$u.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
  grep '^{' $out/bench_hjb_u$u.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('unroll $u prepare', d['ms_per_step'])"
done
