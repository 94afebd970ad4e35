set -o pipefail
mkdir -p gpurun_out
tools/ab_probe_small.sh probe_r06c "" homog,all && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_range.py tests/test_gpu_fullsize.py -k "down_scaled or unequal" > gpurun_out/t_r06c_new.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_range.py tests/test_gpu_tanh.py > gpurun_out/t_r06c_parity.txt 2>&1
