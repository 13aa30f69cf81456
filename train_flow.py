"""RayTorchTrain - the reference training flow (R/train_flow.py) on the MI355X-native framework.

    python train_flow.py [--environment=fast-bakery] run [--epochs 3] [--batch_size 32]
        [--learning_rate 1e-3] [--from-run RayTorchTrain/<id>] [--from-task F/R/S/T]
    python train_flow.py argo-workflows create | trigger

Same flags, defaults and step graph (start -> train (gang of N_PARALLEL) -> join -> end) as
the reference.  `current.ray_storage_path` is the per-task checkpoint root handed to
RunConfig(storage_path=...); `--from-task` takes precedence over `--from-run`; the string
"null" means unset.  Added (optional): --resume_mode best_weights|exact, --num_workers,
--max_failures, and the bf16 DDP workloads of BASELINE.json (configs 2-5) through the same
trainer / storage layout / --from-run path:
    python train_flow.py run --model gpt2-small --steps 200 --ckpt_every_n_steps 50
    python train_flow.py run --model gpt2-small --steps 400 --from-run RayTorchTrain/<id> --resume_mode exact
(--model resnet18 | llama3-8b | *-tiny; sharded DCP checkpoints every N steps, async.)
"""
from ray_torch_distributed_checkpoint_amd.flow import (FlowSpec, Parameter, current, gpu_profile, kubernetes,
                                                       metaflow_ray, pypi, retry, schedule, step, upstream_checkpoint)

N_PARALLEL = 2
N_GPU_PER_WORKER = 1


@schedule(cron="*/5 * * * *")
class RayTorchTrain(FlowSpec):

    epochs = Parameter("epochs", default=3)
    global_batch_size = Parameter("batch_size", default=32)
    learning_rate = Parameter("learning_rate", default=1e-3)
    upstream_task_pathspec = Parameter(
        "from-task",
        default=None,
        help="A task pathspec like flow_name/run_id/step_name/task_id containing a .results artifact with a checkpoint.",
    )
    upstream_run_pathspec = Parameter(
        "from-run",
        default=None,
        help="A run pathspec like flow_name/run_id containing a .results artifact with a checkpoint.",
    )
    resume_mode = Parameter("resume_mode", default="best_weights",
                            help="best_weights (reference warm start) or exact (optimizer/epoch/RNG/sampler).")
    num_workers = Parameter("num_workers", default=0, help="0 = N_PARALLEL*N_GPU_PER_WORKER capped by visible GPUs")
    max_failures = Parameter("max_failures", default=0, help="in-trainer restarts from the latest checkpoint")
    model = Parameter("model", default="mlp",
                      help="mlp (the reference workload) | gpt2-small | resnet18 | llama3-8b | gpt2-tiny | ...")
    steps = Parameter("steps", default=100, help="optimizer steps (bf16 workloads)")
    ckpt_every_n_steps = Parameter("ckpt_every_n_steps", default=25, help="sharded async checkpoint interval")
    report_every_n_steps = Parameter("report_every_n_steps", default=0,
                                     help="metrics rows between checkpoints (0: one row per checkpoint)")
    grad_comm_dtype = Parameter("grad_comm_dtype", default="fp32", help="fp32 | bf16 gradient all-reduce")
    zero_stage = Parameter("zero_stage", default=-1,
                           help="1: ZeRO-1 sharded optimizer step, 0: replicated; -1 (default): ZeRO-1 for llama* "
                                "at more than one worker (bf16 workloads)")
    batch_size_per_worker = Parameter("batch_size_per_worker", default=0,
                                      help="bf16 workloads: samples per worker per step (0: the model's default). "
                                           "--batch_size is the reference MLP's global batch")

    @step
    def start(self):
        self.next(self.train, num_parallel=N_PARALLEL)

    @retry(times=3)
    @metaflow_ray(all_nodes_started_timeout=60 * 5)
    @pypi(packages={})
    @gpu_profile(interval=1)
    @kubernetes(gpu=N_GPU_PER_WORKER, compute_pool="obp-gpu")
    @step
    def train(self):
        import torch

        from my_ray_module import train_fashion_mnist

        from ray_torch_distributed_checkpoint_amd.workloads import train_workload

        use_gpu = torch.cuda.is_available()
        n = int(self.num_workers) or N_PARALLEL * N_GPU_PER_WORKER
        if use_gpu:
            n = min(n, torch.cuda.device_count())
        hyperparameters = dict(
            epochs=int(self.epochs),
            global_batch_size=int(self.global_batch_size),
            learning_rate=float(self.learning_rate),
        )
        args = dict(
            num_workers=n,
            use_gpu=use_gpu,
            checkpoint_storage_path=current.ray_storage_path,
            resume_mode=self.resume_mode,
            max_failures=int(self.max_failures),
            **hyperparameters,
        )
        warm = upstream_checkpoint(self.upstream_task_pathspec, self.upstream_run_pathspec, required=False)
        if warm is not None:  # --from-task wins over --from-run (flow/upstream.py)
            args["checkpoint"] = warm
        else:
            print("Training from newly initialized")

        if self.model == "mlp":
            self.result = train_fashion_mnist(**args)
        else:
            mode = "exact" if self.resume_mode == "exact" else "weights"
            self.result = train_workload(
                model=self.model, steps=int(self.steps), num_workers=n, use_gpu=use_gpu,
                batch_size_per_worker=int(self.batch_size_per_worker) or None,
                lr=None, ckpt_every_n_steps=int(self.ckpt_every_n_steps),
                checkpoint_storage_path=current.ray_storage_path, checkpoint=args.get("checkpoint"),
                resume_mode=mode, max_failures=int(self.max_failures), grad_comm_dtype=self.grad_comm_dtype,
                zero_stage=int(self.zero_stage),
                report_every_n_steps=int(self.report_every_n_steps) or None)
        self.next(self.join)

    @step
    def join(self, inputs):
        for i in inputs:
            try:
                self.result = i.result
            except AttributeError:
                pass
        self.next(self.end)

    @step
    def end(self):
        print(self.result)


if __name__ == "__main__":
    RayTorchTrain()
