# Round-5 GPU session B: grouped wgrad microbench (persistent vs per-tile), bench overlap window.
set -e
export TMPDIR=/tmp
O=gpurun_out/b; mkdir -p $O
RTDC_G8G_PERSIST=0 timeout -k 10 200 python benchmarks/gemm_bench.py --wgrad-group llama > $O/wg_llama_g8g.jsonl 2> $O/wg.err
timeout -k 10 200 python benchmarks/gemm_bench.py --wgrad-group llama > $O/wg_llama_g8gp.jsonl 2>> $O/wg.err
RTDC_G8G_PERSIST=0 timeout -k 10 200 python benchmarks/gemm_bench.py --wgrad-group gpt2 > $O/wg_gpt2_g8g.jsonl 2>> $O/wg.err
timeout -k 10 200 python benchmarks/gemm_bench.py --wgrad-group gpt2 > $O/wg_gpt2_g8gp.jsonl 2>> $O/wg.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
RTDC_G8G_PERSIST=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_g8g.json 2> $O/bench_g8g.err
