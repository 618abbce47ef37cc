"""CPU restatement of the reference's EnvNet-v2 batch source (test infrastructure only: imported by
tests/, never by the package).

* envnet_preprocess / envnet_random_crop / envnet_multi_crop: EnvNetPreprocessor.preprocess,
  .random_crop and .multi_crop_test (reference src/datasets/preprocessing.py:814-855 and 857-884):
  constant-0 padding of int(window * padding_ratio) samples each side, a random crop
  randint(0, total - window) when training (python `random`), the centre crop otherwise, and
  linspace(0, total - window, test_crops).long() starts for the multi-crop test.
* stratified_split: ESC50DataModule.setup's train/val split (reference src/datasets/esc50.py:508-546):
  the sorted fold_k/*.pt files of the four training folds, val size ceil(len * val_split),
  sklearn StratifiedShuffleSplit(n_splits=1, test_size=val_size, random_state=42) over their labels.
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch
import torch.nn.functional as F


def envnet_samples(window_length: float = 5.0, padding_ratio: float = 0.5, sample_rate: int = 44100):
    """(window_samples, padding_samples) -- preprocessing.py:807-809."""
    window = int(window_length * sample_rate)
    return window, int(window * padding_ratio)


def envnet_preprocess(w: torch.Tensor, window_length=5.0, padding_ratio=0.5, sample_rate=44100) -> torch.Tensor:
    """preprocessing.py:814-827 (the clip is already at 44.1 kHz: no resampling)."""
    _, pad = envnet_samples(window_length, padding_ratio, sample_rate)
    return F.pad(w, (pad, pad), mode="constant", value=0)


def envnet_random_crop(w: torch.Tensor, training: bool, window_length=5.0, rng: random.Random | None = None,
                       sample_rate=44100) -> torch.Tensor:
    """preprocessing.py:829-855."""
    window, _ = envnet_samples(window_length, 0.5, sample_rate)
    total = w.shape[-1]
    if total <= window:
        return F.pad(w, (0, window - total), mode="constant", value=0)
    if training:
        start = (rng or random).randint(0, total - window)
    else:
        start = (total - window) // 2
    return w[..., start:start + window]


def envnet_multi_crop(w: torch.Tensor, test_crops: int = 10, window_length=5.0, sample_rate=44100):
    """preprocessing.py:857-884."""
    window, _ = envnet_samples(window_length, 0.5, sample_rate)
    total = w.shape[-1]
    if total <= window:
        return [F.pad(w, (0, window - total), mode="constant", value=0)]
    starts = torch.linspace(0, total - window, test_crops).long()
    return [w[..., int(s):int(s) + window] for s in starts]


def stratified_split(files: list, labels: list, val_split: float):
    """esc50.py:527-536 -> (train_files, val_files)."""
    from sklearn.model_selection import StratifiedShuffleSplit

    val_size = math.ceil(len(files) * val_split)
    splitter = StratifiedShuffleSplit(n_splits=1, test_size=val_size, random_state=42)
    tr, va = next(splitter.split(np.zeros(len(labels)), labels))
    return [files[i] for i in tr], [files[i] for i in va]
