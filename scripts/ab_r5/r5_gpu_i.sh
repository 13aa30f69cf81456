# Round-5 GPU session I: bf16 GEMM epilogue lookahead W = 2 (shipped) / 4 / 8 (abv/ builds).
set -e
export TMPDIR=/tmp
for so in "" /root/repo/abv/_C_w4.so /root/repo/abv/_C_w8.so; do
  RTDC_EXT_SO=$so timeout -k 10 300 python benchmarks/gemm_bench.py --only mlp_proj --reps 20 >> gpurun_out/i_gemm.jsonl 2>/dev/null
  RTDC_EXT_SO=$so timeout -k 10 300 python benchmarks/gemm_bench.py --only fc --reps 20 >> gpurun_out/i_gemm.jsonl 2>/dev/null
done
bash scripts/gpu.sh envab TAG=w4 ENVA="X=0" ENVB="RTDC_EXT_SO=/root/repo/abv/_C_w4.so" ROUNDS=2 > gpurun_out/i_w4.txt 2>&1
bash scripts/gpu.sh envab TAG=w8 ENVA="X=0" ENVB="RTDC_EXT_SO=/root/repo/abv/_C_w8.so" ROUNDS=2 > gpurun_out/i_w8.txt 2>&1
