#!/bin/bash
# Same-box A/B of bench lines: the round-5 package (tools/variants/r05pkg: its bench.py, package and
# oracle, built from round 5's last commit; untracked) against this tree, alternating, twice.
# usage: tools/ab_bench.sh <tag> [workloads...]     outputs under gpurun_out/<tag>/
out=gpurun_out/${1:-ab}; shift; mkdir -p $out; export TMPDIR=/tmp
wls=${*:-burgers hjb gbm gbm_hess}
set -e
for rep in 1 2; do
  for wl in $wls; do
    steps=100; [ $wl = hjb ] && steps=20; [ $wl = gbm_hess ] && steps=20
    a="--workload $wl --steps $steps --warmup 3 --no-cpu-baseline --no-fp32-pass"
    (cd tools/variants/r05pkg && ../../gpu_check.sh 200 ../../../$out/r05_${wl}_$rep.log python bench.py $a)
    tools/gpu_check.sh 200 $out/r06_${wl}_$rep.log python bench.py $a
  done
done
for f in $out/r0*_*.log; do grep -h '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'], 4), round(d['roofline']['frac'], 3))"; done
