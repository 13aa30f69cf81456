# Round-5 GPU session D: full GPU test suite + smoke, then the dgrad-on-hipBLASLt A/B.
set -e
export TMPDIR=/tmp
bash scripts/gpu.sh tests,smoke
bash scripts/gpu.sh envab TAG=dgblaslt ENVA="RTDC_DGRAD_BLASLT=0" ENVB="RTDC_DGRAD_BLASLT=1" ROUNDS=2 > gpurun_out/envab_dgblaslt.txt 2>&1
