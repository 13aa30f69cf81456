# Round-5 GPU session E2: AdamW variants at GPT-2 size, interleaved x3.
set -e
O=gpurun_out/e2; mkdir -p $O
for r in 1 2 3; do
for v in "X=0" "RTDC_ADAMW_U=2" "RTDC_ADAMW_GRID=1" "RTDC_ADAMW_U=2 RTDC_ADAMW_GRID=1" "RTDC_OPT_CHUNK=65536" "RTDC_ADAMW_U=2 RTDC_OPT_CHUNK=65536"; do
  env $v timeout -k 10 100 python benchmarks/optim_bench.py --params 124.4e6 --reps 20 >> $O/optim.jsonl 2>> $O/optim.err
done
done
