#!/bin/bash
# r03g: buffer-form LDS-DMA in k_gemm_x3h — microbenchmark (bitwise vs the 256-row kernel, incl. a
# 2,304-word row stride), the PISGradNet GPU tests, the HJB bench and a one-stream kernel trace.
set -e
out=gpurun_out/r03g
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory" "$2"; then echo "fault in $2"; exit 3; fi; }
run 240 $out/ubench_x3h.txt tools/ubench_x3h 262144 20
run 900 $out/pis_tests.log python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_range.py tests/test_gpu_train.py -k "pis or hjb or PIS or HJB or ou"
run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 20 --warmup 3
run 300 $out/bench_hjb_onestream.log python bench.py --workload hjb --steps 20 --warmup 3 --no-prepare --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb1 -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-prepare --no-cpu-baseline > $out/trace_hjb1.log 2>&1
echo done
