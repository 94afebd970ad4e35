#!/bin/bash
# HJB prepare-schedule bench repeats plus a prepare trace (per-kernel averages under co-running).
out=gpurun_out/${1:-hjbab}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pis or hjb or ou or side_stream or graph"
grep -E "passed|failed" $out/gpu_tests.log | tail -1
for r in 1 2 3; do
  tools/gpu_check.sh 300 $out/bench_hjb_$r.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
  grep '^{' $out/bench_hjb_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hjb prepare', d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/trace_hjb_prep -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb_prep.log 2>&1
