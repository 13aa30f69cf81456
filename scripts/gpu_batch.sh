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
  echo "[$name] EXIT $rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step kmaj_tests 300 python -u -m pytest tests/test_kmajor_gpu.py tests/test_kernels_gpu.py -m gpu -k "kmajor or transpose" -v --timeout 200 --timeout-method thread
bash scripts/gpu.sh envab ENVA="RTDC_DGRAD_KMAJOR=0" ENVB="RTDC_DGRAD_KMAJOR=auto" ROUNDS=3 TAG=kmajor2
RTDC_DGRAD_KMAJOR=auto step prof_kmaj2 700 bash scripts/gpu.sh prof STEPS=10 TAG=gpt2_kmaj2
