#!/bin/bash
# Round-3 pass JJ: grouped weight-gradient capacity (RTDC_WGRAD_ROUND 256 / 216 / 160 / 128) on GPT-2,
# alternating, two rounds.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 256 216 160 128; do
    RTDC_WGRAD_ROUND=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_jj_${v}_r$r.log 2>&1
    rc=$?; echo "GPT2 WGRAD_ROUND=$v r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_jj_${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
