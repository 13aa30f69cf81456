#!/bin/bash
# Product path at production size on one MI355X (VERDICT r2 "next" #3): GPT-2-small through
# train_flow.py (TorchTrainer + async sharded DCP checkpoints every 50 steps), then an exact
# --from-run resume, against an uninterrupted run of the same length, and bench.py on the
# same box for the throughput comparison.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/product_r3}
mkdir -p $OUT
export RTDC_HOME=/tmp/rtdc_home
STEPS=${STEPS:-200}
MORE=${MORE:-250}
MODEL=${MODEL:-gpt2-small}
timeout -k 10 400 python -u train_flow.py run --model $MODEL --steps $STEPS --ckpt_every_n_steps 50 \
  --num_workers 1 --report_every_n_steps 10 > $OUT/run_a.log 2>&1
rc=$?; echo "RUN A EXIT $rc"; tail -n 3 $OUT/run_a.log
[ $rc -eq 0 ] || exit $rc
RID=$(sed -n 's/.*RayTorchTrain\/\([^ ]*\) starting.*/\1/p' $OUT/run_a.log | head -n 1)
echo "run A id: $RID"
timeout -k 10 400 python -u train_flow.py run --model $MODEL --steps $MORE --ckpt_every_n_steps 50 \
  --num_workers 1 --from-run RayTorchTrain/$RID --resume_mode exact > $OUT/run_b.log 2>&1
rc=$?; echo "RUN B EXIT $rc"; tail -n 3 $OUT/run_b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u train_flow.py run --model $MODEL --steps $MORE --ckpt_every_n_steps 50 \
  --num_workers 1 --report_every_n_steps 10 > $OUT/run_c.log 2>&1
rc=$?; echo "RUN C EXIT $rc"; tail -n 3 $OUT/run_c.log
[ $rc -eq 0 ] || exit $rc
# collect the trial logs (result.json rows) of the three runs
for f in $(find $RTDC_HOME -name result.json); do
  d=$(echo $f | sed 's/[^A-Za-z0-9_.-]/_/g'); cp $f $OUT/$d
done
timeout -k 10 300 python -u bench.py --model $MODEL --steps 50 --warmup 10 > $OUT/bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 $OUT/bench.log
