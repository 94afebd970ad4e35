#!/bin/bash
# r04i: the whole -m gpu suite (g(x) moved into k_pis_base_final); HJB prepare-fraction sweep and
# kernel trace; k_pis_net's HBM writes with and without the non-temporal hint.
out=gpurun_out/${1:-r04i}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
grep -E "FAILED" $out/gpu_tests.log | head -20 || true
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for fr in 0.92 1.0 0.85 0.92; do
  DPI_PIS_PREP_FRAC=$fr tools/gpu_check.sh 300 $out/hjb_f$fr.log $B --workload hjb
  grep -h '^{' $out/hjb_f$fr.log | python -c "$S" hjb_f$fr || true
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb.log 2>&1
for nt in 1 0; do
  DPI_PIS_NT=$nt timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_pis_net" -d $out/pmc_nt${nt}_WRITE_SIZE -o pmc \
    --output-format csv -- python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_nt${nt}.log 2>&1
done
timeout -k 10 300 python tools/perf_gbm.py > $out/perf_gbm.txt 2>&1
for r in a b; do
  tools/gpu_check.sh 300 $out/burgers_prep_$r.log $B --workload burgers --prepare
  grep -h '^{' $out/burgers_prep_$r.log | python -c "$S" burgers_prep_$r || true
  tools/gpu_check.sh 300 $out/burgers_$r.log $B --workload burgers
  grep -h '^{' $out/burgers_$r.log | python -c "$S" burgers_$r || true
done
