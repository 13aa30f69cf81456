#!/bin/bash
# GPT-2 plain dgrads (qkv / attn_proj / fc1 / LM head, M = 16384) on hipBLASLt (RTDC_DGRAD_BLASLT=1)
# vs the auto rule (native for M > 4096), then one kernel trace of the hipBLASLt arm
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for arm in auto 1; do
  RTDC_DGRAD_BLASLT=$arm timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/ab_bench_${arm}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "DGRAD_BLASLT=$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bench_${arm}_$r.log)"
done; done
RTDC_DGRAD_BLASLT=1 TAG=gpt2_dgblaslt STEPS=5 WARMUP=3 bash scripts/gpu.sh prof
