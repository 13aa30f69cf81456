"""RayTorchEval - the reference evaluation flow (R/eval_flow.py) on the MI355X-native framework.

    python eval_flow.py run --from-run RayTorchTrain/<id> [--from-task ...] [--batch_size 512]
    python eval_flow.py argo-workflows create     # then every finished RayTorchTrain run triggers it

Checkpoint precedence: triggering run > --from-task > --from-run > error (R/eval_flow.py:40-54).
Batch inference runs the native fp32 MLP through the columnar `data.Dataset.map_batches`
pipeline; the error-analysis card ("Misclassifications X out of Y" + a table of samples with
image / true label / predicted label / logits chart) is written as static HTML in the task
directory.  Fixes of reference quirks: fewer than 50 misclassifications no longer raises
(Appendix B.7), output order is guaranteed (positional join is sound).
"""
from ray_torch_distributed_checkpoint_amd.flow import (FlowSpec, Parameter, card, current, gpu_profile, kubernetes,
                                                       pypi, step, trigger_on_finish, upstream_checkpoint)
from ray_torch_distributed_checkpoint_amd.flow.cards import error_analysis_components

N_GPU = 1


@trigger_on_finish(flow="RayTorchTrain")
class RayTorchEval(FlowSpec):

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
    upstream_namespace = Parameter(
        "from-namespace",
        default=None,
        help="Namespace of the upstream run (the local registry has a single namespace).",
    )
    batch_size = Parameter("batch_size", default=512)
    n_error_samples = 50

    def _get_checkpoint(self):
        # triggering run > --from-task > --from-run > error (flow/upstream.py)
        return upstream_checkpoint(self.upstream_task_pathspec, self.upstream_run_pathspec, use_trigger=True)

    @card(type="blank", id="error_analysis")
    @gpu_profile(interval=1)
    @kubernetes(gpu=N_GPU, compute_pool="obp-gpu")
    @pypi(packages={})
    @step
    def start(self):
        import pandas as pd
        import torch

        from my_ray_module import TorchPredictor, get_dataloaders, get_labels_map

        self.upstream_checkpoint = self._get_checkpoint()
        bs = int(self.batch_size)
        ds = get_dataloaders(batch_size=bs, val_only=True, as_ray_ds=True)
        predictor = TorchPredictor(checkpoint=self.upstream_checkpoint, cpu_only=not torch.cuda.is_available())
        scored = ds.map_batches(predictor, concurrency=N_GPU, batch_size=bs, num_gpus=N_GPU).take_all()
        # map_batches keeps the input order, so the positional join is sound
        self.predictions = pd.concat([ds.to_pandas(), pd.DataFrame(scored)], axis=1)
        wrong = self.predictions.labels != self.predictions.predicted_values
        self.misclassifications = self.predictions.where(wrong).dropna()
        current.card["error_analysis"].extend(
            error_analysis_components(self.predictions, self.misclassifications, get_labels_map(), self.n_error_samples))
        self.accuracy = float((~wrong).mean())
        self.next(self.end)

    @step
    def end(self):
        print(f"[eval] accuracy={self.accuracy:.4f} misclassified={self.misclassifications.shape[0]}")


if __name__ == "__main__":
    RayTorchEval()
