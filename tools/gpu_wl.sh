#!/bin/bash
# GPU tests, then bench lines and one-stream kernel traces for the named workloads.
# usage: tools/gpu_wl.sh <tag> <workload ...>        outputs under gpurun_out/<tag>/
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 $out/gpu_tests.log
for wl in "$@"; do
  tools/gpu_check.sh 300 $out/bench_$wl.log python bench.py --workload $wl --steps 20 --warmup 3
  grep '^{' $out/bench_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', d['ms_per_step'], d['value'], d['roofline']['frac'], d['config']['rel_l2_vs_ref'], d.get('cpu_baseline', {}).get('value'))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o trace --output-format csv -- \
    python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_$wl.log 2>&1
done
