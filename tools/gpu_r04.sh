#!/bin/bash
# r04r: PIS rollout in four dim parts per path: PIS tests; HJB prepare-fraction sweep; trace.
out=gpurun_out/${1:-r04r}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pis or hjb or ou or PIS or td"
tail -1 $out/gpu_tests.log
grep -E "FAILED" $out/gpu_tests.log | head -20 || true
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for fr in 0.92 0.85 0.78 1.0 0.92; do
  DPI_PIS_PREP_FRAC=$fr tools/gpu_check.sh 300 $out/hjb_f$fr.log $B --workload hjb
  grep -h '^{' $out/hjb_f$fr.log | python -c "$S" hjb_f$fr || true
done
tools/gpu_check.sh 300 $out/hjb_one.log $B --workload hjb --no-prepare
grep -h '^{' $out/hjb_one.log | python -c "$S" hjb_one || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb.log 2>&1
