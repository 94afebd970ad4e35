#!/bin/bash
# r04j: PIS tests (NT split); HJB NT A/B; HJB HBM passes; GBM phase timings with / without the
# fused reduce; gbm_hess bench.
out=gpurun_out/${1:-r04j}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pis or hjb or ou or PIS"
tail -1 $out/gpu_tests.log
grep -E "FAILED" $out/gpu_tests.log | head -20 || true
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for r in a b; do
  for nt in 2 1; do
    DPI_PIS_NT=$nt tools/gpu_check.sh 300 $out/hjb_nt${nt}_$r.log $B --workload hjb
    grep -h '^{' $out/hjb_nt${nt}_$r.log | python -c "$S" hjb_nt${nt}_$r || true
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce" -d $out/pmc_hjb_$c -o pmc \
    --output-format csv -- python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_hjb_$c.log 2>&1
done
timeout -k 10 300 python tools/perf_gbm.py > $out/perf_gbm.txt 2>&1
DPI_FUSED_REDUCE=0 timeout -k 10 300 python tools/perf_gbm.py > $out/perf_gbm_nofuse.txt 2>&1
tools/gpu_check.sh 300 $out/gbm_hess.log $B --workload gbm_hess
grep -h '^{' $out/gbm_hess.log | python -c "$S" gbm_hess || true
