#!/bin/bash
# Kernel trace of the HJB bench under the prepare-stream schedule (timeline analysis: tools/trace_timeline.py).
out=gpurun_out/${1:-prep}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/trace_hjb_prep -o trace --output-format csv -- \
  python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb_prep.log 2>&1
echo rc=$?
