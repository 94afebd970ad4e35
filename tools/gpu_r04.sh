#!/bin/bash
# r04u: GBM with AGPR-pinned weights as the product: GBM / Hessian / TD GPU tests, bench lines.
out=gpurun_out/${1:-r04u}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "gbm or GBM or sdgd or SDGD or hess or td or TD"
tail -1 $out/gpu_tests.log
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for w in gbm gbm_hess; do
  tools/gpu_check.sh 300 $out/$w.log $B --workload $w
  grep -h '^{' $out/$w.log | python -c "$S" $w || true
done
for r in a b; do
  tools/gpu_check.sh 300 $out/hjb_hi_$r.log $B --workload hjb
  grep -h '^{' $out/hjb_hi_$r.log | python -c "$S" hjb_hi_$r || true
  DPI_BENCH_MAIN_PRIORITY=default tools/gpu_check.sh 300 $out/hjb_def_$r.log $B --workload hjb
  grep -h '^{' $out/hjb_def_$r.log | python -c "$S" hjb_def_$r || true
done
