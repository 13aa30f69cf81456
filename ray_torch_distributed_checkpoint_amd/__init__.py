"""MI355X-native distributed training + sharded checkpointing framework.

Capabilities of outerbounds/ray-torch-distributed-checkpoint (Ray Train DDP trainer, report /
Checkpoint / RunConfig(storage_path) / CheckpointConfig(num_to_keep), --from-run resume,
batch-inference eval flow) re-designed for AMD Instinct MI355X (gfx950): process-per-GPU
launcher, RCCL/xGMI bucketed all-reduce on flat gradient buffers, hand-written CDNA4 HIP
kernels (MFMA GEMMs, norms, fused cross-entropy, fused optimizers), and a native
DCP-compatible sharded checkpoint engine (HBM snapshot -> pinned ring -> writer threads).

Subpackages: ops (kernels), models, parallel, optim, checkpoint, train, data, flow, utils.
"""
__version__ = "0.1.0"
