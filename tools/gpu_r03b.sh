#!/bin/bash
# r03b: fp16-split range probe + the new data-module / full-size / train GPU tests.
set -e
out=gpurun_out/r03b
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 900 $out/new_tests.log python -u -m pytest -v --timeout 600 --timeout-method thread \
  tests/test_gpu_dataset.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -m gpu
run 800 $out/probe_range.jsonl python tools/probe_range.py
echo done
