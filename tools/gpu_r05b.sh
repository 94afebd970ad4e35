#!/bin/bash
# round 5, call b: Tanh kernels + canaries + new train test, the whole suite, range-check A/B at 100
# steps, and the k_pis_net L2 PMC passes (measure first)
set -e
out=gpurun_out/r05b; mkdir -p $out; export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
run 600 $out/new_tests.log python -u -m pytest tests/test_gpu_tanh.py tests/test_gpu_canary.py tests/test_gpu_train.py -m gpu -x -v --timeout 300 --timeout-method thread
run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
for i in 1 2; do
  for m in off step region; do
    run 200 $out/bench_burgers_${m}_$i.log python bench.py --no-cpu-baseline --no-fp32-pass --steps 100 --range-check $m
  done
done
run 180 $out/nccl_smoke.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/nccl_smoke.py
tools/rehearsal_n2.sh r05b
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_pis_net|k_pis_rollout" -d $out/pmc_pis_a -o pmc --output-format csv -- \
  python bench.py --workload hjb --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-pass --no-prepare > $out/pmc_pis_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY \
  --kernel-include-regex "k_pis_net" -d $out/pmc_pis_b -o pmc --output-format csv -- \
  python bench.py --workload hjb --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-pass --no-prepare > $out/pmc_pis_b.log 2>&1
echo done
