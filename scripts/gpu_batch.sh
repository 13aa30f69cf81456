#!/bin/bash
# One gpurun batch (edit the step list per call): each GPU step runs under its own timeout and
# the batch stops at the first step that ends by signal / timeout (rc > 1); test failures
# (rc 1) do not stop it.  Logs: gpurun_out/<step>.log.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] EXIT $rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
}
L=fwd_bias_res,fwd_bias_gelu,dgrad_gelu_cs
W4=$PWD/abv/_C_w4.so
step kt_w4 600 env RTDC_EXT_SO=$W4 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm or linear or mlp" --timeout 120 --timeout-method thread
step gemm_w4 400 env RTDC_EXT_SO=$W4 python -u benchmarks/gemm_bench.py --set gpt2 --layouts $L --reps 20
step gemm_head 400 python -u benchmarks/gemm_bench.py --set gpt2 --layouts $L --reps 20
step gemm_w4b 400 env RTDC_EXT_SO=$W4 python -u benchmarks/gemm_bench.py --set gpt2 --layouts $L --reps 20
step gemm_headb 400 python -u benchmarks/gemm_bench.py --set gpt2 --layouts $L --reps 20
bash scripts/gpu.sh envab TAG=w4 ROUNDS=3 STEPS=30 ENVA=RTDC_GELU_SAVE_GRAD=0 ENVB=RTDC_EXT_SO=$W4
bash scripts/gpu.sh envab TAG=gsg ROUNDS=3 STEPS=30 ENVA=RTDC_GELU_SAVE_GRAD=0 ENVB=RTDC_GELU_SAVE_GRAD=1
