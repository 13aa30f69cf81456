#!/bin/bash
# timing-only GEMM builds (ab/_C_diag{1,2,4,7}.so, RTDC_G8_DIAG bits) vs the in-tree build,
# non-persistent 8-wave kernel on the fc and 4096^3 shapes
set -o pipefail
cd /root/repo
export TMPDIR=/tmp RTDC_GEMM_PERSIST=0
mkdir -p gpurun_out
for v in base diag1 diag2 diag4 diag7; do
  if [ $v = base ]; then unset RTDC_EXT_SO; else export RTDC_EXT_SO=/root/repo/ab/_C_$v.so; fi
  for sh in fc sq4096; do
    timeout -k 10 120 python benchmarks/gemm_bench.py --only $sh > gpurun_out/diag_${v}_$sh.jsonl 2>&1
    rc=$?; echo "$v $sh EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
