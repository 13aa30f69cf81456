#!/bin/bash
# per-kernel clock / MFMA-busy / wait% of the final round-5 GPT-2 step (scripts/pmc_clock.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
d=gpurun_out/pmc_clock_gpt2_r5; rm -rf "$d"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  -- python3 bench.py --steps 2 --warmup 1 --no-ckpt --sweep 0 > gpurun_out/pmc_clock_gpt2_r5.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_clock_gpt2_r5.log; exit 1; }
python3 scripts/pmc_clock.py "$d" > gpurun_out/pmc_clock_gpt2_r5.txt
find "$d" -name '*.csv' -size +20M -delete
head -30 gpurun_out/pmc_clock_gpt2_r5.txt
