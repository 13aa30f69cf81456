#!/bin/bash
# Round-3 pass AA: Llama-3-8B on one GPU - AdamW over 8B fp32 parameters (~240 GB of optimizer
# traffic, ~40 ms) overlapped with backward (--overlap-opt 1) vs the plain step, alternating.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 1 0; do
    timeout -k 10 400 python -u bench.py --model llama3-8b --steps 6 --warmup 2 --no-ckpt --overlap-opt $v > gpurun_out/llama_aa_ov${v}_r$r.log 2>&1
    rc=$?; echo "LLAMA OVERLAP=$v r$r EXIT $rc $(tail -n 1 gpurun_out/llama_aa_ov${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
