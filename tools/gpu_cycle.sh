set -e
mkdir -p gpurun_out
tools/gpu_check.sh 600 gpurun_out/gpu_tests.log python -m pytest tests -m gpu -q -x -s
tools/gpu_check.sh 300 gpurun_out/bench.log python bench.py --steps 20 --warmup 3
cd gpurun_out && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof -o r01b --output-format csv -- python ../bench.py --steps 20 --warmup 3 > prof.log 2>&1
