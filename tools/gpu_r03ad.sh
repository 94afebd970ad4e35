#!/bin/bash
# r03ad: (1) HJB baseline rows' chain beside the rollout (DPI_PIS_BASE_SIDE), (2) the 4-wave
# per-point baseline (DPI_BASELINE_W4) — full GPU tests, same-box A/B bench lines, kernel traces.
set -e
out=gpurun_out/${OUT:-r03ad}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
run 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
for rep in 1 2; do
  for s in 1 0; do
    DPI_PIS_BASE_SIDE=$s run 300 $out/bench_hjb_side${s}_rep$rep.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
    DPI_BASELINE_W4=$s run 300 $out/bench_burgers_w4${s}_rep$rep.log python bench.py --no-cpu-baseline
  done
done
run 300 $out/trace_hjb.log timeout -k 10 280 rocprofv3 --kernel-trace --stats -d $out/trace_hjb -o trace --output-format csv -- python3 bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
run 300 $out/trace_burgers.log timeout -k 10 280 rocprofv3 --kernel-trace --stats -d $out/trace_burgers -o trace --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
echo done
