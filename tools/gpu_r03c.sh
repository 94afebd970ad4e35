#!/bin/bash
# r03c: the whole GPU suite (range guard, weight-scaled goldens, HJB train, data module), printed output kept.
set -e
out=gpurun_out/r03c
mkdir -p $out
export TMPDIR=/tmp
tools/gpu_check.sh 1100 $out/gpu_tests.log python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread
echo done
