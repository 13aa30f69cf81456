#!/bin/bash
# GEMM stagers with 32-bit per-lane offsets (abv/_C_s32.so, -DRTDC_STAGER32=1) vs 64-bit pointers (in-tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=abv/_C_s32.so
RTDC_EXT_SO=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm or epilogue or gelu or wgrad" > gpurun_out/v_tests.log 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/v_tests.log; exit 1; }
tail -n 1 gpurun_out/v_tests.log
for r in 1 2; do for arm in base s32; do
  if [ $arm = s32 ]; then e="RTDC_EXT_SO=$V"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 300 python benchmarks/gemm_bench.py --set all --reps 10 > gpurun_out/v_gemm_${arm}_$r.log 2>&1 || { echo "gemm $arm failed"; tail -5 gpurun_out/v_gemm_${arm}_$r.log; exit 1; }
  echo "$arm $r"; python3 - "$arm" "$r" <<'PY'
import json, sys
for l in open(f"gpurun_out/v_gemm_{sys.argv[1]}_{sys.argv[2]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"  {d['shape']:10s} fwd {d['fwd']['ours_us']:8.1f} gelu {d['fwd_bias_gelu']['ours_us']:8.1f} dgrad {d['dgrad']['ours_us']:8.1f} dgg {d['dgrad_gelu']['ours_us']:8.1f} wgrad {d['wgrad']['ours_us']:8.1f}")
PY
done; done
for r in 1 2; do for arm in base s32; do
  if [ $arm = s32 ]; then e="RTDC_EXT_SO=$V"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/v_bench_${arm}_$r.log 2>&1 || { echo "bench $arm failed"; exit 1; }
  echo "$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/v_bench_${arm}_$r.log)"
done; done
