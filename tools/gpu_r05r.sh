#!/bin/bash
# round 5, call r: the final check again after the last rebuild (stamp-variant hooks only)
# default bench line (as the driver runs them)
set -e
out=gpurun_out/r05r; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run 300 $out/bench_default.log python bench.py
run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 30 --warmup 3
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 50 --warmup 5
echo done
