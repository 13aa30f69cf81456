"""Distributed sampler with torch's permutation contract (torch/utils/data/distributed.py:66-146:
seed+epoch randperm, pad to total_size, strided rank slice) plus an exact mid-epoch resume
offset, which the fault-tolerance path checkpoints (BASELINE config 5)."""
from __future__ import annotations

import math

import torch
from torch.utils.data import Sampler


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: int | None = None, rank: int | None = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        import torch.distributed as dist

        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        self.dataset, self.num_replicas, self.rank = dataset, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        self.start_index = 0  # samples of this rank's epoch already consumed (resume)
        n = len(dataset)
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def indices(self) -> list[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(len(self.dataset), generator=g).tolist()
        else:
            idx = list(range(len(self.dataset)))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def __iter__(self):
        return iter(self.indices()[self.start_index:])

    def __len__(self):
        return self.num_samples - self.start_index

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        self.start_index = 0

    def state_dict(self) -> dict:
        return {"epoch": self.epoch, "start_index": self.start_index, "seed": self.seed}

    def load_state_dict(self, sd: dict) -> None:
        self.epoch = int(sd["epoch"])
        self.start_index = int(sd["start_index"])
        self.seed = int(sd.get("seed", self.seed))
