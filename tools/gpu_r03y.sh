#!/bin/bash
# r03y: k_pis_net with / without the non-temporal hint on its row traffic, L2 hit rate of each.
set -e
out=gpurun_out/${OUT:-r03y}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
run 300 $out/fused_test.log python -u -m pytest -v -s --timeout 250 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "fused"
run 200 $out/bench_hjb_fused_onestream.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare
DPI_PIS_NT=0 run 200 $out/bench_hjb_fused_nt0.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare
run 200 $out/bench_hjb_fused_onestream2.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare
run 120 $out/pmc_nt1.log timeout -s KILL 100 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/pmc_nt1 -o p -- python3 bench.py --workload hjb --steps 3 --warmup 1 --no-cpu-baseline --no-prepare --prewarm-s 0
DPI_PIS_NT=0 run 120 $out/pmc_nt0.log timeout -s KILL 100 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/pmc_nt0 -o p -- python3 bench.py --workload hjb --steps 3 --warmup 1 --no-cpu-baseline --no-prepare --prewarm-s 0
echo done
