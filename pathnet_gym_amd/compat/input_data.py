"""``input_data.read_data_sets`` (reference ``input_data.py:16-29`` re-exports TF's MNIST reader).

Reads the four MNIST idx files (optionally ``.gz``) from ``train_dir`` when
they are present.  There is no network access, so nothing is downloaded:
without the files, a synthetic MNIST-shaped set is generated
(``algo/supervised.make_digits('mnist')``, 28x28 gray, 10 classes; say so in
any result you report from it).  Returns ``Datasets(train, validation,
test)`` of ``DataSet`` objects with ``images``, ``labels``, ``num_examples``,
``epochs_completed`` and ``next_batch(batch_size, shuffle=True)``, matching
the TF 1.x ``mnist`` module.
"""
from __future__ import annotations

import collections
import gzip
import os
from typing import Optional

import numpy as np

Datasets = collections.namedtuple("Datasets", ["train", "validation", "test"])

_FILES = {"train_x": "train-images-idx3-ubyte", "train_y": "train-labels-idx1-ubyte",
          "test_x": "t10k-images-idx3-ubyte", "test_y": "t10k-labels-idx1-ubyte"}


def _open(path):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    return None


def _read_idx(f) -> np.ndarray:
    """idx format: magic (0x00 0x00 dtype ndim), big-endian dims, raw uint8 payload."""
    head = f.read(4)
    if head[0] != 0 or head[1] != 0 or head[2] != 0x08:
        raise ValueError("not a uint8 idx file")
    ndim = head[3]
    dims = np.frombuffer(f.read(4 * ndim), dtype=">u4").astype(np.int64)
    data = np.frombuffer(f.read(int(np.prod(dims))), dtype=np.uint8)
    return data.reshape(tuple(dims))


def load_mnist_idx(train_dir: str):
    out = {}
    for k, name in _FILES.items():
        f = _open(os.path.join(train_dir, name))
        if f is None:
            return None
        with f:
            out[k] = _read_idx(f)
    return out


def _synthetic(n: int, seed: int):
    import torch.nn.functional as F
    from ..algo.supervised import make_digits
    X, y = make_digits("mnist", n, seed)
    img = X.view(n, 32, 32, 3)[..., 0]
    img = F.interpolate(img[:, None], size=(28, 28), mode="bilinear", align_corners=False)[:, 0]
    return (img.clamp(0, 1).numpy() * 255).astype(np.uint8), y.numpy().astype(np.uint8)


def dense_to_one_hot(labels_dense: np.ndarray, num_classes: int = 10) -> np.ndarray:
    out = np.zeros((labels_dense.shape[0], num_classes), np.float32)
    out[np.arange(labels_dense.shape[0]), labels_dense.astype(np.int64)] = 1.0
    return out


class DataSet:
    def __init__(self, images: np.ndarray, labels: np.ndarray, one_hot=False, dtype=np.float32, reshape=True,
                 seed: Optional[int] = None):
        images = images.reshape(images.shape[0], images.shape[1], images.shape[2], 1) if images.ndim == 3 else images
        if reshape:
            images = images.reshape(images.shape[0], -1)
        if np.dtype(dtype) == np.float32:
            images = images.astype(np.float32) * (1.0 / 255.0)
        self._images = images
        self._labels = dense_to_one_hot(labels) if one_hot else labels.astype(np.int64)
        self._num_examples = images.shape[0]
        self._epochs_completed = 0
        self._index_in_epoch = 0
        self._rng = np.random.RandomState(seed)

    images = property(lambda self: self._images)
    labels = property(lambda self: self._labels)
    num_examples = property(lambda self: self._num_examples)
    epochs_completed = property(lambda self: self._epochs_completed)

    def next_batch(self, batch_size: int, fake_data=False, shuffle=True):
        start = self._index_in_epoch
        if self._epochs_completed == 0 and start == 0 and shuffle:
            self._perm = self._rng.permutation(self._num_examples)
        elif not hasattr(self, "_perm"):
            self._perm = np.arange(self._num_examples)
        idx = []
        while len(idx) < batch_size:
            take = min(batch_size - len(idx), self._num_examples - self._index_in_epoch)
            idx.extend(self._perm[self._index_in_epoch:self._index_in_epoch + take])
            self._index_in_epoch += take
            if self._index_in_epoch == self._num_examples:
                self._epochs_completed += 1
                self._index_in_epoch = 0
                self._perm = self._rng.permutation(self._num_examples) if shuffle else np.arange(self._num_examples)
        idx = np.asarray(idx)
        return self._images[idx], self._labels[idx]


def read_data_sets(train_dir: str, fake_data=False, one_hot=False, dtype=np.float32, reshape=True,
                   validation_size: int = 5000, seed: Optional[int] = None, synthetic_size=(12000, 2000)):
    raw = None if fake_data else load_mnist_idx(train_dir)
    if raw is None:
        n_train, n_test = synthetic_size
        tx, ty = _synthetic(n_train, 1 if seed is None else seed)
        vx, vy = _synthetic(n_test, 2 if seed is None else seed + 1)
        raw = {"train_x": tx, "train_y": ty, "test_x": vx, "test_y": vy}
        validation_size = min(validation_size, n_train // 6)
    tx, ty = raw["train_x"], raw["train_y"]
    kw = dict(one_hot=one_hot, dtype=dtype, reshape=reshape, seed=seed)
    return Datasets(train=DataSet(tx[validation_size:], ty[validation_size:], **kw),
                    validation=DataSet(tx[:validation_size], ty[:validation_size], **kw),
                    test=DataSet(raw["test_x"], raw["test_y"], **kw))
