#!/bin/bash
# r04y: GBM u = 0 / H = 16 instances back under 80 KB of LDS: GBM tests, bench, VALU pass.
out=gpurun_out/${1:-r04y}; mkdir -p $out; export TMPDIR=/tmp
set -e
tools/gpu_check.sh 600 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "gbm or GBM or sdgd or SDGD or hess or zero"
tail -1 $out/gpu_tests.log
S='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), "%.3e" % d["value"], round(d["roofline"]["kernel_ms"],4), d["config"]["rel_l2_vs_ref"]["grad"], d["roofline"].get("noise_floor"))'
tools/gpu_check.sh 300 $out/gbm.log python bench.py --workload gbm --steps 20 --warmup 3 --no-cpu-baseline
grep -h '^{' $out/gbm.log | python -c "$S" gbm || true
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex k_paths -d $out/pmc_valu_gbm -o pmc --output-format csv -- \
  python bench.py --workload gbm --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_valu_gbm.log 2>&1
