#!/bin/bash
# round 5, call e: the whole GPU suite after the train fix; default bench lines
set -e
out=gpurun_out/r05e; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run 300 $out/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 $out/bench_burgers.log python bench.py
run 300 $out/bench_gbm.log python bench.py --workload gbm --no-cpu-baseline
echo done
