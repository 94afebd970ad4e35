#!/bin/bash
out=gpurun_out/${1:-tail}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
tools/gpu_check.sh 300 $out/ubench_stage.log tools/ubench_x3 262144 10 stage
grep -c "differing words 0" $out/ubench_stage.log
tools/gpu_check.sh 300 $out/bench_hjb.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
grep '^{' $out/bench_hjb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hjb prepare', d['ms_per_step'])"
tools/gpu_check.sh 300 $out/bench_hjb_one.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline --no-prepare
grep '^{' $out/bench_hjb_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hjb one-stream', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_hjb_onestream.log 2>&1
