#!/bin/bash
# Round-end check: GPU tests, smoke(), default bench and every workload's bench line.
out=gpurun_out/${1:-final}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -1 $out/gpu_tests.log
tools/gpu_check.sh 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $out/smoke.log
tools/gpu_check.sh 300 $out/bench_default.log python bench.py
tools/gpu_check.sh 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
tools/gpu_check.sh 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
tools/gpu_check.sh 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 10 --warmup 2
for f in $out/bench_*.log; do grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['ms_per_step'], '%.3e' % d['value'], d['roofline']['bound'], round(d['roofline']['frac'], 3))"; done
