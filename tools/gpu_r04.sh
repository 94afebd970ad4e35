#!/bin/bash
# r04h: the whole -m gpu suite (two-launch sample_with_gradients, fused label reduce, shared
# prepare-stream rollout); HJB prepare-fraction sweep; Burgers and GBM bench lines; kernel traces.
out=gpurun_out/${1:-r04h}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
grep -E "FAILED" $out/gpu_tests.log | head -20 || true
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"])'
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
for fr in 0.92 0.85 1.0 0.88; do
  DPI_PIS_PREP_FRAC=$fr tools/gpu_check.sh 300 $out/hjb_f$fr.log $B --workload hjb
  grep -h '^{' $out/hjb_f$fr.log | python -c "$S" hjb_f$fr || true
done
tools/gpu_check.sh 300 $out/burgers.log $B --workload burgers
grep -h '^{' $out/burgers.log | python -c "$S" burgers || true
DPI_FUSED_REDUCE=0 tools/gpu_check.sh 300 $out/burgers_nofuse.log $B --workload burgers
grep -h '^{' $out/burgers_nofuse.log | python -c "$S" burgers_nofuse || true
tools/gpu_check.sh 300 $out/burgers_b.log $B --workload burgers
grep -h '^{' $out/burgers_b.log | python -c "$S" burgers_b || true
tools/gpu_check.sh 300 $out/gbm.log $B --workload gbm
grep -h '^{' $out/gbm.log | python -c "$S" gbm || true
cd $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_burgers -o burgers --output-format csv -- python ../../bench.py --steps 20 --warmup 3 --no-cpu-baseline > prof_burgers.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_hjb -o hjb --output-format csv -- python ../../bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > prof_hjb.log 2>&1
