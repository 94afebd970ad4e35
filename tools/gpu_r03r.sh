#!/bin/bash
# r03r: round-end check of the committed binary — the whole -m gpu suite and the
# bench line of every workload.
set -e
out=gpurun_out/r03r
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory" "$2"; then echo "fault in $2"; exit 3; fi; }
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run 300 $out/bench_burgers.log python bench.py
run 300 $out/bench_burgers_cfg3.log python bench.py --workload burgers_cfg3
run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
run 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 10 --warmup 2
echo done
