#!/bin/bash
# r03v: k_pis_net (the fused PISGradNet VJP chain) — bitwise equality with the layer-wise chain,
# the HJB full-size oracle test, M > 65,536 label calls, and HJB bench lines fused / layer-wise,
# prepare / one stream, plus a one-stream kernel trace of the fused chain.
set -e
out=gpurun_out/${OUT:-r03v}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
run 300 $out/fused_test.log python -u -m pytest -v -s --timeout 250 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "fused or hjb_config2"
run 300 $out/paths_test.log python -u -m pytest -v -s --timeout 250 --timeout-method thread -m gpu tests/test_gpu_parity.py -k more_paths
run 200 $out/bench_hjb_fused.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
run 200 $out/bench_hjb_fused_onestream.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare
DPI_PIS_FUSED=0 run 200 $out/bench_hjb_layerwise.log python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline
run 300 $out/trace.log timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o hjb -- python3 bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare
echo done
