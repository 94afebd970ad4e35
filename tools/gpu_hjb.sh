#!/bin/bash
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pis or hjb or ou or side_stream or graph"
tail -2 $out/gpu_tests.log
for r in 1 2; do
  tools/gpu_check.sh 300 $out/bench_hjb_$r.log python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline
  grep '^{' $out/bench_hjb_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hjb', d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_prep -o trace --output-format csv -- python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb_prep.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_hjb_one.log 2>&1
