#!/bin/bash
# Same-box A/B of bench lines: a variant package (tools/variants/<VARIANT>: a git worktree of an
# earlier commit with its library built in place; untracked) against this tree, alternating, twice.
# usage: VARIANT=r06pre tools/ab_bench.sh <tag> [workloads...]     outputs under gpurun_out/<tag>/
out=gpurun_out/${1:-ab}; shift; mkdir -p $out; export TMPDIR=/tmp
var=${VARIANT:-r06pre}
wls=${*:-burgers hjb gbm gbm_hess}
set -e
for rep in 1 2; do
  for wl in $wls; do
    steps=100; [ $wl = hjb ] && steps=20; [ $wl = gbm_hess ] && steps=20
    a="--workload $wl --steps $steps --warmup 3 --no-cpu-baseline --no-fp32-pass"
    (cd tools/variants/$var && ../../gpu_check.sh 200 ../../../$out/${var}_${wl}_$rep.log python bench.py $a)
    tools/gpu_check.sh 200 $out/head_${wl}_$rep.log python bench.py $a
  done
done
for f in $out/*_*_[12].log; do grep -h '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4), round(d['roofline']['frac'], 3))"; done
