"""Datasets and loaders.

The reference trains on torchvision CIFAR-10 downloaded at start-up
(/root/reference/example/main.py:23-29).  torchvision is not installed here and
there is no network, so this module provides

* synthetic CIFAR-/MNIST-/ImageNet-shaped data (deterministic per seed),
* readers for the original on-disk formats (CIFAR-10 ``data_batch_*.bin``,
  MNIST idx) when the files are present locally, and
* :class:`DeviceBatchPool` - batches generated once and kept resident in HBM
  so a throughput run measures the training step, not PCIe.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, TensorDataset

CIFAR_MEAN = (0.5, 0.5, 0.5)   # reference transform: Normalize((.5,.5,.5),(.5,.5,.5)), main.py:35-38
CIFAR_STD = (0.5, 0.5, 0.5)
CIFAR_CLASSES = ("plane", "car", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck")


class SyntheticImages(Dataset):
    """``n`` random images of ``shape`` with labels in ``[0, num_classes)``.

    Each class has a fixed random template (shared by every split and seed);
    an image is ``template[label] * signal + N(0, 1)``, so a model can actually
    fit the data: loss decreasing is a meaningful end-to-end check, and
    time-to-target-loss is measurable.
    """

    def __init__(self, n: int, shape=(3, 32, 32), num_classes: int = 10, seed: int = 0,
                 learnable: bool = True, signal: float = 0.5):
        g = torch.Generator().manual_seed(seed)
        self.y = torch.randint(0, num_classes, (n,), generator=g)
        self.x = torch.randn(n, *shape, generator=g)
        if learnable:
            templates = torch.randn(num_classes, *shape,
                                    generator=torch.Generator().manual_seed(1234))
            self.x += signal * templates[self.y]

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i]


def read_cifar10_binary(root: str, train: bool = True):
    """Read CIFAR-10 binary batches (``data_batch_{1..5}.bin`` / ``test_batch.bin``).

    Returns uint8 images [N,3,32,32] and int64 labels [N].
    """
    root = Path(root)
    sub = root / "cifar-10-batches-bin"
    base = sub if sub.exists() else root
    names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    xs, ys = [], []
    for n in names:
        p = base / n
        if not p.exists():
            continue
        raw = np.fromfile(p, dtype=np.uint8).reshape(-1, 3073)
        ys.append(raw[:, 0].astype(np.int64))
        xs.append(raw[:, 1:].reshape(-1, 3, 32, 32))
    if not xs:
        raise FileNotFoundError(f"no CIFAR-10 binary batches under {root}")
    return torch.from_numpy(np.concatenate(xs)), torch.from_numpy(np.concatenate(ys))


def read_mnist_idx(root: str, train: bool = True):
    root = Path(root)
    pre = "train" if train else "t10k"
    img = root / f"{pre}-images-idx3-ubyte"
    lab = root / f"{pre}-labels-idx1-ubyte"
    if not img.exists() or not lab.exists():
        raise FileNotFoundError(f"no MNIST idx files under {root}")
    x = np.fromfile(img, dtype=np.uint8)[16:].reshape(-1, 1, 28, 28)
    y = np.fromfile(lab, dtype=np.uint8)[8:].astype(np.int64)
    return torch.from_numpy(x.copy()), torch.from_numpy(y.copy())


def normalize_uint8(x: torch.Tensor, mean=CIFAR_MEAN, std=CIFAR_STD) -> torch.Tensor:
    c = x.shape[1]
    m = torch.tensor(mean[:c]).view(1, c, 1, 1)
    s = torch.tensor(std[:c]).view(1, c, 1, 1)
    return (x.float() / 255.0 - m) / s


def get_datasets(name: str, data_dir: str = "./data", input_shape=(3, 32, 32),
                 num_classes: int = 10, n_train: int = 50000, n_test: int = 10000,
                 seed: int = 0):
    """Return ``(train_ds, test_ds, source)``; real files when present, else synthetic."""
    name = name.lower()
    if name == "cifar10":
        try:
            xtr, ytr = read_cifar10_binary(data_dir, True)
            xte, yte = read_cifar10_binary(data_dir, False)
            return (TensorDataset(normalize_uint8(xtr), ytr),
                    TensorDataset(normalize_uint8(xte), yte), "cifar10")
        except FileNotFoundError:
            name = "synthetic"
    if name == "mnist":
        try:
            xtr, ytr = read_mnist_idx(data_dir, True)
            xte, yte = read_mnist_idx(data_dir, False)
            return (TensorDataset(normalize_uint8(xtr, (0.1307,), (0.3081,)), ytr),
                    TensorDataset(normalize_uint8(xte, (0.1307,), (0.3081,)), yte), "mnist")
        except FileNotFoundError:
            name = "synthetic"
    if name != "synthetic":
        raise ValueError(f"unknown dataset {name!r}")
    tr = SyntheticImages(n_train, input_shape, num_classes, seed=seed)
    te = SyntheticImages(n_test, input_shape, num_classes, seed=seed + 1)
    return tr, te, "synthetic"


def make_loaders(train_ds, test_ds, batch_size: int, test_batch_size: int, shuffle_seed=None,
                 workers: int = 0, pin: bool = False):
    g = None
    if shuffle_seed is not None:
        g = torch.Generator().manual_seed(shuffle_seed)
    train = DataLoader(train_ds, batch_size=batch_size, shuffle=True, num_workers=workers,
                       drop_last=True, generator=g, pin_memory=pin)
    test = DataLoader(test_ds, batch_size=test_batch_size, shuffle=False, num_workers=workers,
                      pin_memory=pin)
    return train, test


class DeviceBatchPool:
    """``n_batches`` synthetic batches resident on the device, served round-robin."""

    def __init__(self, batch: int, shape, num_classes: int, device, n_batches: int = 8,
                 dtype=torch.bfloat16, seed: int = 0, channels_last: bool = True,
                 learnable: bool = False, signal: float = 0.5):
        """``learnable``: images are ``signal * template[label] + N(0, 1)`` with
        fixed per-class templates (as :class:`SyntheticImages`), so the loss can
        reach a target; otherwise pure noise with random labels."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.x, self.y = [], []
        mf = torch.channels_last if (channels_last and len(shape) == 3) else torch.contiguous_format
        templates = None
        if learnable:
            templates = torch.randn(num_classes, *shape,
                                    generator=torch.Generator().manual_seed(1234))
        for _ in range(n_batches):
            y = torch.randint(0, num_classes, (batch,), generator=g)
            x = torch.randn(batch, *shape, generator=g)
            if templates is not None:
                x += signal * templates[y]
            self.x.append(x.to(device=device, dtype=dtype).contiguous(memory_format=mf))
            self.y.append(y.to(device))
        self.i = 0

    def next(self):
        x, y = self.x[self.i], self.y[self.i]
        self.i = (self.i + 1) % len(self.x)
        return x, y

    def __iter__(self):
        return self

    def __next__(self):
        return self.next()


TTL_TRAIN_SEED = 100
TTL_HELDOUT_SEED = 100 + 7919


def ttl_pools(batch: int, shape, num_classes: int, device, n_train: int, n_heldout: int,
              dtype=torch.bfloat16, signal: float = 0.05):
    """Train and held-out pools of the time-to-target data.

    Both draw ``signal * template[label] + N(0, 1)`` from the SAME class
    templates (so the held-out split measures generalisation of the same task)
    with different generator seeds, so no held-out sample is a training sample
    (``tests/test_core_cpu.py::test_ttl_heldout_split_is_disjoint``).  The
    reference scores training by its test set the same way
    (/root/reference/example/main.py:83-89,110-131)."""
    train = DeviceBatchPool(batch, shape, num_classes, device, n_batches=n_train, dtype=dtype,
                            seed=TTL_TRAIN_SEED, learnable=True, signal=signal)
    held = DeviceBatchPool(batch, shape, num_classes, device, n_batches=n_heldout, dtype=dtype,
                           seed=TTL_HELDOUT_SEED, learnable=True, signal=signal) \
        if n_heldout > 0 else None
    return train, held


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default
