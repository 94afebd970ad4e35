#!/bin/bash
# r04za: PIS points sampled one prepare() ahead on their own stream: PIS tests; HJB A/B (same box).
out=gpurun_out/${1:-r04z}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pis or hjb or ou or PIS or side or prepare or shard"
tail -1 $out/gpu_tests.log
grep -E "FAILED" $out/gpu_tests.log | head -20 || true
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for r in a b; do
  tools/gpu_check.sh 300 $out/hjb_ahead_$r.log $B --workload hjb
  grep -h '^{' $out/hjb_ahead_$r.log | python -c "$S" hjb_ahead_$r || true
  DPI_BENCH_SAMPLE_AHEAD=0 tools/gpu_check.sh 300 $out/hjb_noahead_$r.log $B --workload hjb
  grep -h '^{' $out/hjb_noahead_$r.log | python -c "$S" hjb_noahead_$r || true
done
