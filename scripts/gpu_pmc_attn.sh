#!/bin/bash
# PMC counters for the flash-attention kernels (GPT-2 shape); counters only with kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA \
  -- python3 benchmarks/attn_bench.py --only gpt2 --reps 3 > gpurun_out/pmc_attn.log 2>&1
echo "PMC EXIT $?"
