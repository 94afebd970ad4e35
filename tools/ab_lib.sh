#!/bin/bash
# Same-box A/B of this tree's library against a variant library (tools/build_variant.py output,
# loaded with DPI_HIP_LIB), alternating, twice.  usage: tools/ab_lib.sh <tag> <variant.so> [workloads...]
out=gpurun_out/${1:-ablib}; lib=$2; shift 2; mkdir -p $out; export TMPDIR=/tmp
wls=${*:-burgers}
set -e
for rep in 1 2; do
  for wl in $wls; do
    a="--workload $wl --steps 100 --warmup 3 --no-cpu-baseline --no-fp32-pass"
    DPI_HIP_LIB=$lib tools/gpu_check.sh 200 $out/var_${wl}_$rep.log python bench.py $a
    tools/gpu_check.sh 200 $out/head_${wl}_$rep.log python bench.py $a
  done
done
for f in $out/*_*_[12].log; do grep -h '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4))"; done
