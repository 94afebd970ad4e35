#!/bin/bash
# r04l: PIS tests (GX partial sums in LDS); HJB prepared and one-stream; trace; HBM passes.
out=gpurun_out/${1:-r04l}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pis or hjb or ou or PIS or td"
tail -1 $out/gpu_tests.log
grep -E "FAILED" $out/gpu_tests.log | head -20 || true
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for r in a b; do
  tools/gpu_check.sh 300 $out/hjb_$r.log $B --workload hjb
  grep -h '^{' $out/hjb_$r.log | python -c "$S" hjb_$r || true
done
tools/gpu_check.sh 300 $out/hjb_one.log $B --workload hjb --no-prepare
grep -h '^{' $out/hjb_one.log | python -c "$S" hjb_one || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_hjb_onestream.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce" -d $out/pmc_hjb_$c -o pmc \
    --output-format csv -- python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_hjb_$c.log 2>&1
done
