"""Datasets: a synthetic, learnable FashionMNIST-shaped dataset (torchvision is not available
and there is no network - BASELINE "synthetic data"), the label map, and the
`get_dataloaders` entry point of the reference (R/my_ray_module.py:30-91).

Samples are 1x28x28 float32 in [-1, 1] (the range of ToTensor()+Normalize((0.5,),(0.5,)),
R/my_ray_module.py:38): a per-class smooth prototype plus per-sample noise and a random
shift, generated deterministically from (seed, split, index), so the MLP reaches a
meaningful, non-trivial accuracy.  60,000 train / 10,000 test rows like FashionMNIST.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch.utils.data import Dataset

LABELS = {0: "T-Shirt", 1: "Trouser", 2: "Pullover", 3: "Dress", 4: "Coat", 5: "Sandal", 6: "Shirt",
          7: "Sneaker", 8: "Bag", 9: "Ankle Boot"}


def get_labels_map() -> dict:
    return dict(LABELS)


def _prototypes(seed: int = 1234) -> np.ndarray:
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:28, 0:28] / 27.0
    protos = []
    for c in range(10):
        img = np.zeros((28, 28))
        for _ in range(4):
            cx, cy = rng.uniform(0.15, 0.85, 2)
            sx, sy = rng.uniform(0.08, 0.3, 2)
            amp = rng.uniform(0.6, 1.2)
            img += amp * np.exp(-(((xx - cx) / sx) ** 2 + ((yy - cy) / sy) ** 2))
        img = img / img.max() * 2.0 - 1.0
        protos.append(img)
    return np.stack(protos).astype(np.float32)


class SyntheticFashionMNIST(Dataset):
    """Tensor-backed synthetic FashionMNIST: `data` [N,1,28,28] f32, `targets` [N] int64."""

    def __init__(self, train: bool = True, n: int | None = None, seed: int = 0, noise: float = 0.6):
        n = n if n is not None else (60000 if train else 10000)
        rng = np.random.default_rng(seed * 2 + (0 if train else 1))
        protos = _prototypes()
        y = rng.integers(0, 10, size=n)
        x = protos[y]
        shifts = rng.integers(-3, 4, size=(n, 2))
        out = np.empty_like(x)
        for i in range(n):  # vectorised enough: 60k small rolls
            out[i] = np.roll(x[i], tuple(shifts[i]), axis=(0, 1))
        out += rng.normal(0.0, noise, size=out.shape).astype(np.float32)
        np.clip(out, -1.0, 1.0, out=out)
        self.data = torch.from_numpy(out).unsqueeze(1).contiguous()
        self.targets = torch.from_numpy(y.astype(np.int64))
        self.train = train

    def __len__(self):
        return self.targets.shape[0]

    def __getitem__(self, i):
        return self.data[i], self.targets[i]

    def as_tensors(self):
        return self.data, self.targets


_cache: dict = {}


def fashion_mnist(train: bool, n: int | None = None) -> SyntheticFashionMNIST:
    """Cached per process (the reference's FileLock'ed download, D26, has nothing to lock here)."""
    n = n if n is not None else int(os.environ.get("RTDC_FMNIST_TRAIN" if train else "RTDC_FMNIST_TEST",
                                                   60000 if train else 10000))
    key = (train, n)
    if key not in _cache:
        _cache[key] = SyntheticFashionMNIST(train=train, n=n)
    return _cache[key]


def get_dataloaders(batch_size: int, val_only: bool = False, as_ray_ds: bool = False):
    """R/my_ray_module.py:30-76: train DataLoader (shuffle=True) + val DataLoader, or the
    val-only loader, or (as_ray_ds) `data.Dataset`s of {"features", "labels"} rows."""
    from torch.utils.data import DataLoader

    from .dataset import from_items

    test = fashion_mnist(False)
    if val_only:
        if as_ray_ds:
            return from_items(_rows(test))
        return DataLoader(test, batch_size=batch_size)
    train = fashion_mnist(True)
    if as_ray_ds:
        return from_items(_rows(train)), from_items(_rows(test))
    return DataLoader(train, batch_size=batch_size, shuffle=True), DataLoader(test, batch_size=batch_size)


def _rows(ds: SyntheticFashionMNIST):
    x, y = ds.as_tensors()
    # columnar fast path: the Dataset keeps numpy columns, no per-row Python walk (Appendix B.10)
    return {"features": x.numpy(), "labels": y.numpy()}
