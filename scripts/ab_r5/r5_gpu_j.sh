# Round-5 GPU session J2: Llama-3-8B, fused AdamW overlapped with backward with a capped update grid.
set -e
export TMPDIR=/tmp
for r in 1 2; do
  for v in "RTDC_X=0 OV=0" "RTDC_OVERLAP_GRID=256 OV=1" "RTDC_OVERLAP_GRID=512 OV=1" "RTDC_OVERLAP_GRID=128 OV=1" "RTDC_OVERLAP_GRID=256 RTDC_OVERLAP_PRIO=-1 OV=1"; do
    ov=${v##*OV=}; tag=$(echo $v | tr ' =' '__')
    env ${v% OV=*} timeout -k 10 400 python bench.py --model llama3-8b --steps 6 --warmup 2 --no-ckpt --overlap-opt $ov > gpurun_out/j2_${r}_$tag.log 2>&1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/j2_${r}_$tag.log)"
  done
done
