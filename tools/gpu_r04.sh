#!/bin/bash
# r04o: GBM noise-loop unroll A/B (same box): product (4), 8, 16; Hessian labels 1 vs 4.
out=gpurun_out/${1:-r04o}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "gbm or GBM or sdgd or SDGD or hess"
tail -1 $out/gpu_tests.log
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
lib() { if [ $1 = product ]; then echo deeppicarditeration_amd/libdpi_hip.so; else echo tools/variants/libdpi_$1.so; fi; }
for r in a b; do
  for v in product unr8; do
    DPI_HIP_LIB=$(lib $v) tools/gpu_check.sh 300 $out/gbm_${v}_$r.log $B --workload gbm
    grep -h '^{' $out/gbm_${v}_$r.log | python -c "$S" gbm_${v}_$r || true
  done
  for v in product hunr4; do
    DPI_HIP_LIB=$(lib $v) tools/gpu_check.sh 300 $out/gbmh_${v}_$r.log $B --workload gbm_hess
    grep -h '^{' $out/gbmh_${v}_$r.log | python -c "$S" gbmh_${v}_$r || true
  done
done
