#!/bin/bash
# Llama attention backward knobs (benchmarks/attn_bench.py, llama8b / llama8b_b4 shapes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in "X=0" "RTDC_FA_QS=1" "RTDC_FA_QS=2" "RTDC_FA_QS=4" "RTDC_FA_DQ=1" "RTDC_FA_XCD=1" "RTDC_FA_DKDV=2"; do
  env $v timeout -k 10 120 python benchmarks/attn_bench.py --reps 20 > gpurun_out/x_attn.log 2>&1 || { echo "attn $v failed"; exit 1; }
  echo "$v $r $(python3 -c "
import json
for l in open('gpurun_out/x_attn.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if d['shape'] != 'gpt2': print(d['shape'], d['kernel_fwd_us'], d['kernel_bwd_us'], d['kernel_bwd_TF'], end=' | ')
")"
done; done
