#!/bin/bash
# Llama-3-8B: plain forwards (RTDC_FWD_BLASLT) and plain dgrads (RTDC_DGRAD_BLASLT) on hipBLASLt vs the native GEMMs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in "X=0" "RTDC_FWD_BLASLT=1" "RTDC_FWD_BLASLT=1 RTDC_DGRAD_BLASLT=1"; do
  env $v timeout -k 10 400 python bench.py --model llama3-8b --steps 5 --warmup 2 --no-ckpt > gpurun_out/y_bench.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/y_bench.log; exit 1; }
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/y_bench.log)"
done; done
