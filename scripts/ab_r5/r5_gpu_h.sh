# Round-5 GPU session H: re-check of older opt-in switches on the round-5 build (GPT-2-small step).
set -e
export TMPDIR=/tmp
bash scripts/gpu.sh envab TAG=gsg ENVA="RTDC_GELU_SAVE_GRAD=0" ENVB="RTDC_GELU_SAVE_GRAD=1" ROUNDS=2 > gpurun_out/h_gsg.txt 2>&1
bash scripts/gpu.sh envab TAG=g4b ENVA="RTDC_GEMM4B_AUTO=2" ENVB="RTDC_GEMM4B_AUTO=1" ROUNDS=2 > gpurun_out/h_g4b.txt 2>&1
bash scripts/gpu.sh envab TAG=wside ENVA="RTDC_WGRAD_SIDE=0" ENVB="RTDC_WGRAD_SIDE=1" ROUNDS=2 > gpurun_out/h_wside.txt 2>&1
bash scripts/gpu.sh envab TAG=kmaj2 ENVA="RTDC_DGRAD_KMAJOR=0" ENVB="RTDC_DGRAD_KMAJOR=1 RTDC_GELU_SAVE_GRAD=1" ROUNDS=2 > gpurun_out/h_kmaj2.txt 2>&1
