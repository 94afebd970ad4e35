# PMC passes over the HJB bench (k_gemm_x3 only); csv -> gpurun_out/pmcg*/
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex k_gemm_x3 -d gpurun_out/pmcg1 -o pmc --output-format csv -- python bench.py --workload hjb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcg1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM --kernel-include-regex k_gemm_x3 -d gpurun_out/pmcg2 -o pmc --output-format csv -- python bench.py --workload hjb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcg2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gemm_x3 -d gpurun_out/pmcg3 -o pmc --output-format csv -- python bench.py --workload hjb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcg3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_gemm_x3 -d gpurun_out/pmcg4 -o pmc --output-format csv -- python bench.py --workload hjb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcg4.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_gemm_x3 -d gpurun_out/pmcg5 -o pmc --output-format csv -- python bench.py --workload hjb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcg5.log 2>&1
