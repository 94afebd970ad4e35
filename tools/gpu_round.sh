#!/bin/bash
# One GPU call of a round, by stages: GPU tests, bench lines for every workload, kernel traces (one
# stream for HJB), the counter list, the VALU / HBM PMC passes, same-box A/B against the round-5
# package (ab, probe: tools/variants/r05pkg), the N = 2 gloo rehearsals and the RCCL smoke.
# usage: tools/gpu_round.sh <tag> [tests|fused|fbab|bench|wide|gbmlong|hessab|hjbfrac|trace|traceb|hjb|hjbprep|counters|pmc|ab|probe|rehearsal|nccl ...]
#        outputs under gpurun_out/<tag>/
set -e
tag=${1:-r02}; shift || true
what=${*:-tests bench trace pmc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
run() { tools/gpu_check.sh "$@"; }
for w in $what; do
  case $w in
  tests)
    run 900 $out/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
  bench)
    run 300 $out/bench_burgers.log python bench.py
    run 300 $out/bench_burgers_cfg3.log python bench.py --workload burgers_cfg3
    run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
    run 300 $out/bench_gbm.log python bench.py --workload gbm --steps 20 --warmup 3
    run 300 $out/bench_gbm_hess.log python bench.py --workload gbm_hess --steps 10 --warmup 2 ;;
  trace)
    for wl in burgers burgers_cfg3 gbm gbm_hess; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$wl -o trace --output-format csv -- \
        python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_$wl.log 2>&1
    done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- \
      python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_hjb_onestream.log 2>&1 ;;
  traceb)  # the Burgers bench line's kernels only, one-launch and two-launch sample_with_gradients
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_burgers -o trace --output-format csv -- \
      python bench.py --workload burgers --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_burgers.log 2>&1
    DPI_FUSED_BASE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_burgers_fb0 -o trace \
      --output-format csv -- python bench.py --workload burgers --steps 10 --warmup 2 --no-cpu-baseline \
      > $out/trace_burgers_fb0.log 2>&1 ;;
  wide)  # not a BASELINE config: the configs[1] network at nx = 256
    run 300 $out/bench_burgers_nx256.log python bench.py --workload burgers_nx256 --no-cpu-baseline ;;
  gbmlong)  # GBM over 60 steps (15 timed launches for kernel_ms)
    run 300 $out/bench_gbm_60.log python bench.py --workload gbm --steps 60 --warmup 3 --no-cpu-baseline ;;
  hessab)  # Hessian labels: the prepare schedule against one stream, interleaved
    for r in 1 2; do
      run 300 $out/bench_gbm_hess_prep_$r.log python bench.py --workload gbm_hess --steps 40 --warmup 3 --no-cpu-baseline --no-fp32-pass --prepare
      run 300 $out/bench_gbm_hess_plain_$r.log python bench.py --workload gbm_hess --steps 40 --warmup 3 --no-cpu-baseline --no-fp32-pass
    done ;;
  hjbfrac)  # HJB: the prepared share of the rollout (DPI_PIS_PREP_FRAC), interleaved
    for r in 1 2; do
      for f in ${HJB_FRACS:-0.88 0.92 0.96 1.0}; do
        DPI_PIS_PREP_FRAC=$f run 300 $out/bench_hjb_f${f}_$r.log python bench.py --workload hjb --steps 60 --warmup 3 --no-cpu-baseline --no-fp32-pass
      done
    done ;;
  hjb)
    run 300 $out/bench_hjb.log python bench.py --workload hjb --steps 10 --warmup 2
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_onestream -o trace --output-format csv -- \
      python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline --no-prepare > $out/trace_hjb_onestream.log 2>&1 ;;
  hjbprep)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_hjb_prepare -o trace --output-format csv -- \
      python bench.py --workload hjb --steps 10 --warmup 2 --no-cpu-baseline > $out/trace_hjb_prepare.log 2>&1 ;;
  fused)
    run 900 $out/gpu_fused.log python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_canary.py -v --timeout 300 \
      --timeout-method thread ;;
  fbab)  # Burgers: the one-launch sample_with_gradients against the two-launch form, interleaved
    for r in 1 2; do
      DPI_FUSED_BASE=1 run 300 $out/bench_burgers_fb1_$r.log python bench.py
      DPI_FUSED_BASE=0 run 300 $out/bench_burgers_fb0_$r.log python bench.py
    done ;;
  ab)
    tools/ab_bench.sh $tag/ab burgers hjb gbm gbm_hess ;;
  probe)
    tools/ab_probe_small.sh $tag/probe_small "" homog,all ;;
  rehearsal)
    tools/rehearsal_n2.sh $tag ;;
  nccl)
    run 180 $out/nccl_smoke.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 tools/nccl_smoke.py ;;
  counters)
    timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1 ;;
  pmcgbm)  # the GBM VALU pass alone (network launch + the prepare stream's k_noise_shared)
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      --kernel-include-regex "k_paths|k_noise" -d $out/pmc_valu_gbm -o pmc --output-format csv -- \
      python bench.py --workload gbm --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_valu_gbm.log 2>&1 ;;
  pmc)
    for wl in burgers burgers_cfg3 gbm gbm_hess; do
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        --kernel-include-regex "k_paths|k_noise" -d $out/pmc_valu_$wl -o pmc --output-format csv -- \
        python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $out/pmc_valu_$wl.log 2>&1
    done
    for wl in burgers burgers_cfg3 hjb gbm gbm_hess; do
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_paths|k_pis|k_gemm|k_reduce|k_noise" -d $out/pmc_${wl}_$c -o pmc \
          --output-format csv -- python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-pass > $out/pmc_${wl}_$c.log 2>&1
      done
    done ;;
  esac
done
