#!/bin/bash
# r04g: the prepared rollout split between the prepare stream (DPI_PIS_PREP_FRAC of the path sets,
# one wave per SIMD beside k_pis_net) and the prepared call's head; GPU tests touching PISGradNet.
out=gpurun_out/${1:-r04g}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
B="python bench.py --workload hjb --steps 20 --warmup 3 --no-cpu-baseline"
for fr in 0.92 0.85 1.0 0.92 0.88; do
  DPI_PIS_PREP_FRAC=$fr tools/gpu_check.sh 300 $out/hjb_f$fr.log $B
  grep -h '^{' $out/hjb_f$fr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('frac $fr', round(d['ms_per_step'],4), '%.3e' % d['value'], d['config']['rel_l2_vs_ref']['grad'])" || true
done
tools/gpu_check.sh 300 $out/hjb_one.log $B --no-prepare
grep -h '^{' $out/hjb_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('one', round(d['ms_per_step'],4))" || true
cd $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_prep -o hjb_prep --output-format csv -- python ../../bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > prof_prep.log 2>&1
