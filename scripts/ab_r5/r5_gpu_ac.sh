#!/bin/bash
# flash forward: s_setprio(1) around the S = K.Q and P.V MFMA groups (abv/_C_faprio.so, built with
# VAR=attn_flash scripts/build_variant.sh faprio -DRTDC_FA_PRIO=1) vs the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/dump
timeout -k 10 120 python scripts/ab_r5/attn_dump.py /tmp/dump/attn_base.pt > gpurun_out/ac_dump1.log 2>&1 || { echo dump1 failed; tail gpurun_out/ac_dump1.log; exit 1; }
RTDC_EXT_SO=abv/_C_faprio.so timeout -k 10 120 python scripts/ab_r5/attn_dump.py /tmp/dump/attn_prio.pt > gpurun_out/ac_dump2.log 2>&1 || { echo dump2 failed; exit 1; }
python3 -c "
import torch
a=torch.load('/tmp/dump/attn_base.pt', weights_only=True); b=torch.load('/tmp/dump/attn_prio.pt', weights_only=True)
for k in a: print(k, 'fwd bitwise', torch.equal(a[k][0], b[k][0]), 'bwd bitwise', torch.equal(a[k][1], b[k][1]))
"
for r in 1 2 3; do for arm in base prio; do
  if [ $arm = prio ]; then e="RTDC_EXT_SO=abv/_C_faprio.so"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 120 python benchmarks/attn_bench.py --reps 30 > gpurun_out/ac_attn_${arm}_$r.log 2>&1 || { echo "attn $arm failed"; exit 1; }
  echo "$arm $r $(python3 -c "
import json
for l in open('gpurun_out/ac_attn_${arm}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['kernel_fwd_us'], d['kernel_bwd_us'], end=' | ')
")"
done; done
