# Round-5 GPU session G: kernel + memory-copy trace of the async-save window (SDMA drain vs HIP copy stream).
set -e
export TMPDIR=/tmp
for mode in sdma hip; do
  d=gpurun_out/g_$mode; rm -rf $d
  RTDC_CKPT_D2H=$mode timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $d -o run -- \
    python3 bench.py --steps 10 --warmup 3 > gpurun_out/g_$mode.log 2>&1
done
