#!/bin/bash
# Round-3 pass T: optimizer updates overlapped with backward (--overlap-opt 1) now that weight
# gradients arrive in grouped bursts on the side stream - GPT-2 interleaved 1,0,1,0.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for o in 1 0; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt --overlap-opt $o > gpurun_out/gpt2_ov${o}_r$r.log 2>&1
    rc=$?; echo "GPT2 OVERLAP=$o r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_ov${o}_r$r.log | grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
  done
done
