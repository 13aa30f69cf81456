#!/bin/bash
# One parametrised runner for gpurun calls (replaces the per-experiment wrappers).
#
#   bash scripts/gpu.sh <task>[,<task>...] [KEY=VALUE ...]
#
# tasks (run in order, the call stops at the first failure):
#   tests      GPU test suite            (TESTS="tests" selection, -k via K=...)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py                  (MODEL, STEPS, WARMUP, ARGS="extra flags", TAG)
#   prof       rocprofv3 kernel trace of bench.py --no-ckpt: stats + one step's kernels (MODEL, STEPS, ARGS, TAG)
#   pmc        rocprofv3 PMC pass of bench.py (MODEL, PMC="counters", ARGS, TAG)
#   gemm       benchmarks/gemm_bench.py  (ARGS)
#   attn       benchmarks/attn_bench.py  (ARGS)
#   norm       benchmarks/norm_bench.py  (ARGS)
#   ab         alternating bench runs of ab/_C_old.so vs the in-tree _C (MODEL, STEPS, ROUNDS)
#   envab      alternating bench runs under ENVA vs ENVB ("K=V ..."; MODEL, STEPS, ROUNDS, TAG)
#   multirank  2-rank gloo rehearsal of the multi-GPU bench path on one GPU
#   roundend   tests + smoke + bench + multirank (what the driver runs)
#   py         python3 $PY (a script path with args)
# Every GPU step runs under its own timeout; logs go to gpurun_out/<task>[_TAG].log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TASKS="$1"; shift || true
for kv in "$@"; do export "$kv"; done
MODEL=${MODEL:-gpt2-small}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
TAG=${TAG:-$MODEL}
ROUNDS=${ROUNDS:-2}

run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] EXIT $rc"
  tail -n "${TAILN:-3}" "gpurun_out/$name.log"
  return $rc
}

for task in ${TASKS//,/ }; do
  case $task in
    tests)
      sel=${TESTS:-tests}
      kflag=(); [ -n "$K" ] && kflag=(-k "$K")
      run tests 900 python -u -m pytest $sel -x -v -m gpu --timeout 200 --timeout-method thread "${kflag[@]}" || exit $?
      grep -E "passed|failed|skipped" gpurun_out/tests.log | tail -n 1 ;;
    smoke)
      run smoke 240 python -c 'import __graft_entry__ as g; g.smoke()' || exit $? ;;
    bench)
      TAILN=1 run "bench_$TAG" 500 python bench.py --model "$MODEL" --steps "$STEPS" --warmup "$WARMUP" $ARGS || exit $? ;;
    prof)
      d=gpurun_out/prof_$TAG; rm -rf "$d"
      run "prof_$TAG" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
        python3 bench.py --model "$MODEL" --steps "$STEPS" --warmup "$WARMUP" --no-ckpt $ARGS || exit $?
      f=$(find "$d" -name '*kernel_stats.csv' | head -n 1)
      t=$(find "$d" -name '*kernel_trace.csv' | head -n 1)
      python3 scripts/kstats.py "$f" "$((STEPS + WARMUP + 3))" 45 > "gpurun_out/prof_${TAG}_summary.txt"
      python3 scripts/ktimeline.py "$t" --last-ms 100 >> "gpurun_out/prof_${TAG}_summary.txt"
      python3 scripts/kstep.py "$t" ${MARKER:+--marker $MARKER} > "gpurun_out/prof_${TAG}_step.txt"
      head -n 30 "gpurun_out/prof_${TAG}_summary.txt"; tail -n 1 "gpurun_out/prof_${TAG}_step.txt" ;;
    pmc)
      # one counter set per pass (rocprofv3 does not split passes): SQ set, then FETCH_SIZE
      d=gpurun_out/pmc_$TAG; rm -rf "$d" "${d}2"
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
        --pmc ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE} \
        -- python3 bench.py --model "$MODEL" --steps 2 --warmup 1 --no-ckpt --sweep 0 $ARGS > "gpurun_out/pmc_$TAG.log" 2>&1
      rc=$?; echo "[pmc_$TAG] EXIT $rc"; [ $rc -eq 0 ] || exit $rc
      timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "${d}2" -o run --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
        -- python3 bench.py --model "$MODEL" --steps 2 --warmup 1 --no-ckpt --sweep 0 $ARGS > "gpurun_out/pmc2_$TAG.log" 2>&1
      rc=$?; echo "[pmc2_$TAG] EXIT $rc"; [ $rc -eq 0 ] || exit $rc
      f1=$(find "$d" -name '*counter_collection.csv' | head -n 1)
      f2=$(find "${d}2" -name '*counter_collection.csv' | head -n 1)
      python3 scripts/pmc_util.py "$f1" "$f2" > "gpurun_out/pmc_${TAG}_summary.txt"
      head -n 40 "gpurun_out/pmc_${TAG}_summary.txt" ;;
    gemm)
      TAILN=40 run "gemm_$TAG" 600 python3 benchmarks/gemm_bench.py $ARGS || exit $? ;;
    attn)
      TAILN=40 run "attn_$TAG" 600 python3 benchmarks/attn_bench.py $ARGS || exit $? ;;
    norm)
      TAILN=40 run "norm_$TAG" 300 python3 benchmarks/norm_bench.py $ARGS || exit $? ;;
    ab)
      OLD=$PWD/abv/_C_old.so
      for r in $(seq "$ROUNDS"); do
        for arm in old new; do
          if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
          TAILN=0 run "ab_${TAG}_${arm}_$r" 300 python bench.py --model "$MODEL" --steps "$STEPS" --warmup "$WARMUP" --no-ckpt --sweep 0 $ARGS || exit $?
          echo "  $arm $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_${TAG}_${arm}_$r.log")"
        done
      done
      unset RTDC_EXT_SO ;;
    envab)
      # alternating bench runs under two environment settings (ENVA / ENVB: "K=V K2=V2"), ROUNDS each
      for r in $(seq "$ROUNDS"); do
        for arm in A B; do
          if [ $arm = A ]; then envs=$ENVA; else envs=$ENVB; fi
          TAILN=0 run "envab_${TAG}_${arm}_$r" 300 env $envs python bench.py --model "$MODEL" --steps "$STEPS" --warmup "$WARMUP" --no-ckpt --sweep 0 $ARGS || exit $?
          echo "  $arm [$envs] $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/envab_${TAG}_${arm}_$r.log")"
        done
      done ;;
    multirank)
      # both ranks share cuda:0 over gloo (RCCL refuses two ranks on one device): DDP bucket
      # engine, BatchNorm buffer broadcast, sharded DCP save dedup + restore, bf16/ZeRO/P2P modes
      mr() { local name=$1 port=$2; shift 2
        TAILN=1 run "mr_$name" 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port "$port" bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo "$@"; }
      # one HIP hardware queue per process: two processes on one device with gloo's priority
      # streams plus the checkpoint engine's stream oversubscribe the device's queue slots and the
      # scheduler time-slices them (kernels 1000x their length; profiles/multiproc_slowdown_r6.md)
      export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-1}
      export RTDC_SWEEP_CELLS=fp32:32,bf16:64
      mr gpt2 29533 --batch 4 --sweep-budget-s 420 || exit $?
      mr resnet 29534 --model resnet18 --batch 32 --sweep-budget-s 420 || exit $?
      unset RTDC_SWEEP_CELLS
      mr gpt2_zero 29535 --batch 4 --zero 1 --grad-comm-dtype bf16 || exit $?
      mr gpt2_p2p 29536 --batch 4 --p2p-kb 4096 --no-ckpt || exit $?
      unset GPU_MAX_HW_QUEUES ;;
    roundend)
      bash "$0" tests,smoke,bench,multirank || exit $? ;;
    py)
      TAILN=${TAILN:-20} run "py_$TAG" 600 python3 $PY || exit $? ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
