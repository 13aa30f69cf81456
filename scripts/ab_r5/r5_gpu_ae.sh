#!/bin/bash
# (the RTDC_XENT_NT512 switch was removed after this A/B: profiles/xent_nt512_ab_r5.txt)
# cross-entropy over GPT-2 logits (16384 x 50304 bf16): 256 threads x 25 chunks per row (shipped) vs
# 512 x 13 (RTDC_XENT_NT512=1) in the step, then the kernel's time under rocprofv3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for arm in 0 1; do
  if [ $arm = 1 ]; then export RTDC_XENT_NT512=1; else unset RTDC_XENT_NT512; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/ae_bench_${arm}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "NT512=$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ae_bench_${arm}_$r.log) loss $(grep -o '"final_loss": [0-9.]*' gpurun_out/ae_bench_${arm}_$r.log)"
done; done
unset RTDC_XENT_NT512
d=gpurun_out/ae_prof; rm -rf $d
RTDC_XENT_NT512=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt --sweep 0 > gpurun_out/ae_prof.log 2>&1 || { echo "prof failed"; exit 1; }
grep -h "xent" $(find $d -name '*kernel_stats.csv') | cut -c1-160
find $d -name '*trace.csv' -delete
