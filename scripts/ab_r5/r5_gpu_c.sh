# Round-5 GPU session C: LayerNorm forward variants, GEMM tail test, env A/Bs of dgrad K-major / LM-head hipBLASLt.
set -e
export TMPDIR=/tmp
O=gpurun_out/c; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "norm or tail_split or layer" > $O/tests.log 2>&1
for v in "RTDC_NORM_FWD4=0" "RTDC_NORM_FWD_BPC=2" "RTDC_NORM_FWD_BPC=4" "RTDC_NORM_FWD_BPC=8" "RTDC_NORM_FWD_BPC=16"; do
  env $v timeout -k 10 120 python benchmarks/norm_bench.py > $O/norm_${v}.jsonl 2>&1
done
bash scripts/gpu.sh envab TAG=kmaj ENVA="RTDC_DGRAD_KMAJOR=0" ENVB="RTDC_DGRAD_KMAJOR=1" ROUNDS=2 > $O/envab_kmaj.txt 2>&1
bash scripts/gpu.sh envab TAG=blaslt ENVA="RTDC_LMHEAD_BLASLT=0" ENVB="RTDC_LMHEAD_BLASLT=1" ROUNDS=2 > $O/envab_blaslt.txt 2>&1
