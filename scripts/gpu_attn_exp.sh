#!/bin/bash
# attention experiments: fwd variant 2 at Dh=64, then PMC counters of the current kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RTDC_FA_FWD=2 timeout -k 10 200 python benchmarks/attn_bench.py --only gpt2 > gpurun_out/attn_fwd2.jsonl 2>&1
rc=$?; echo "FWD2 EXIT $rc"; grep shape gpurun_out/attn_fwd2.jsonl
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_attn.sh
