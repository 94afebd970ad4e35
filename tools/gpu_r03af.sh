#!/bin/bash
# r03af: host cost of a Burgers bench step (tools/perf_host.py) and a kernel trace of the
# default bench command, to split the step into kernel time and host-induced gaps.
set -e
out=gpurun_out/${OUT:-r03af}
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; if grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" "$2"; then echo "fault in $2"; exit 3; fi; }
run 200 $out/perf_host_burgers.log python tools/perf_host.py burgers
run 300 $out/bench_burgers.log python bench.py
run 300 $out/trace_burgers.log timeout -k 10 280 rocprofv3 --kernel-trace --stats -d $out/trace_burgers -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
echo done
