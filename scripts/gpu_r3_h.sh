#!/bin/bash
# Round-3 pass H: kernel trace of the GPT-2 step (native LM head + native embedding sort),
# then the 2-rank gloo rehearsal (async-save step time vs clean step with the per-node writer
# budget).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash scripts/gpu_prof_gpt2.sh && bash scripts/gpu_multirank.sh
