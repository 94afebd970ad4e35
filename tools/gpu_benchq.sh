#!/bin/bash
out=gpurun_out/${1:-bq}; mkdir -p $out; export TMPDIR=/tmp
set -e
for wl in burgers gbm hjb; do
  tools/gpu_check.sh 300 $out/bench_$wl.log python bench.py --workload $wl --no-cpu-baseline
  grep '^{' $out/bench_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
