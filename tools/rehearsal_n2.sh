#!/bin/bash
# N=2 rehearsals of the bench's N > 1 path (gloo, two ranks on one shared GPU) for every workload.  usage: tools/rehearsal_n2.sh <tag>
out=gpurun_out/${1:-r04q}; mkdir -p $out; export TMPDIR=/tmp
set -e
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
export DPI_BENCH_BACKEND=gloo DPI_BENCH_SHARE_GPU=1
tools/gpu_check.sh 300 $out/rehearsal_burgers_cfg3_n2.log $R --master-port 29522 bench.py --gpus 2 --workload burgers_cfg3 --steps 10 --warmup 2
tools/gpu_check.sh 300 $out/rehearsal_hjb_n2.log $R --master-port 29523 bench.py --gpus 2 --workload hjb --steps 6 --warmup 2
tools/gpu_check.sh 300 $out/rehearsal_gbm_n2.log $R --master-port 29524 bench.py --gpus 2 --workload gbm --steps 10 --warmup 2
tools/gpu_check.sh 300 $out/rehearsal_gbm_hess_n2.log $R --master-port 29525 bench.py --gpus 2 --workload gbm_hess --steps 6 --warmup 2
unset DPI_BENCH_BACKEND DPI_BENCH_SHARE_GPU
grep -h '^{' $out/rehearsal_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); p = d['config'].get('rel_l2_vs_ref', {})
    print(d['workload_key'], d['n_gpus'], d['config'].get('mc_paths_per_gpu'), round(d['ms_per_step'], 4), p.get('bit_identical_to_single_call'), p.get('grad'))
"
