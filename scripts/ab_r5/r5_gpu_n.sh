#!/bin/bash
# epilogue-input touch prefetch (abv/_C_touch.so, -DRTDC_G8_TOUCH=1) vs the in-tree build:
# GEMM epilogue tests on the variant, GPT-2 GEMM products, then the GPT-2 step, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=abv/_C_touch.so
RTDC_EXT_SO=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm or epilogue or gelu" > gpurun_out/n_tests.log 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/n_tests.log; exit 1; }
tail -n 1 gpurun_out/n_tests.log
for r in 1 2; do for arm in base touch; do
  if [ $arm = touch ]; then e="RTDC_EXT_SO=$V"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 200 python benchmarks/gemm_bench.py --set gpt2 --reps 20 > gpurun_out/n_gemm_${arm}_$r.log 2>&1 || { echo "gemm $arm failed"; tail -5 gpurun_out/n_gemm_${arm}_$r.log; exit 1; }
  echo "$arm $r"; python3 - "$arm" "$r" <<'PY'
import json, sys
for l in open(f"gpurun_out/n_gemm_{sys.argv[1]}_{sys.argv[2]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"  {d['shape']:10s} dgrad_gelu {d['dgrad_gelu']['ours_us']:7.1f} us  fwd_bias_res {d['fwd_bias_res']['ours_us']:7.1f} us  dgrad {d['dgrad']['ours_us']:7.1f} us")
PY
done; done
for r in 1 2; do for arm in base touch; do
  if [ $arm = touch ]; then e="RTDC_EXT_SO=$V"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/n_bench_${arm}_$r.log 2>&1 || { echo "bench $arm failed"; exit 1; }
  echo "$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/n_bench_${arm}_$r.log)"
done; done
