#!/bin/bash
# r03z: HJB with k_pis_net — bench line, one-stream kernel trace, FETCH / WRITE PMC passes
# (tools/make_profiles.py <dir> r03z condenses them into profiles/).
set -e
out=gpurun_out/${OUT:-r03z}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
run 300 $out/trace_hjb_onestream.log timeout -k 10 280 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- python3 bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
for c in FETCH_SIZE WRITE_SIZE; do
  run 300 $out/pmc_hjb_$c.log timeout -s KILL 280 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce" -d $out/pmc_hjb_$c -o pmc --output-format csv -- python3 bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
done
echo done
