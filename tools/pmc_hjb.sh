#!/bin/bash
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce" -d $out/pmc_hjb_$c -o pmc \
    --output-format csv -- python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_hjb_$c.log 2>&1 || echo "pass $c rc=$?"
done
echo done
