set -e
out=gpurun_out/r06b; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_check.sh 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
grep -E "passed|failed" $out/gpu_tests.log | tail -1
tools/ab_bench.sh r06b/ab burgers hjb gbm gbm_hess
