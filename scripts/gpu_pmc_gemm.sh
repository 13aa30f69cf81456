#!/bin/bash
# PMC counters for the 8-wave GEMM on the GPT-2 fc / LM-head shapes (kernel trace only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_gemm -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA \
  -- python3 benchmarks/gemm_bench.py --only fc --reps 3 > gpurun_out/pmc_gemm.log 2>&1
echo "PMC1 EXIT $?"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_gemm2 -o run \
  --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_WAVES \
  -- python3 benchmarks/gemm_bench.py --only fc --reps 3 > gpurun_out/pmc_gemm2.log 2>&1
echo "PMC2 EXIT $?"
