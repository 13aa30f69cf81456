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
RTDC_NORM_FWD2R=1 step ln2r_tests 300 python -u -m pytest tests -m gpu -k "norm or layer" -v --timeout 200 --timeout-method thread
for r in 1 2; do
  for v in 0 1; do
    RTDC_NORM_FWD2R=$v step norm_bench_${v}_$r 200 python -u benchmarks/norm_bench.py
    grep '"ours_fwd_us"' gpurun_out/norm_bench_${v}_$r.log | cut -c1-200
  done
done
bash scripts/gpu.sh envab ENVA="RTDC_NORM_FWD2R=0" ENVB="RTDC_NORM_FWD2R=1" ROUNDS=3 TAG=ln2r
