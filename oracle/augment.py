"""CPU restatement of the reference's training-time augmentations (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the product
path (dl-sound-classification_amd/) never imports it.

Restated (each with the reference file:line it follows):
  * BC mixing — ``BCMixingUtils`` (src/datasets/preprocessing.py:395-490) and
    ``BCMixingDataset.apply_bc_mixing`` (preprocessing.py:564-609): different-class partner,
    r ~ U(0,1), RMS "SPL" 20 log10(rms) + 94, perceptual r -> p, (p x1 + (1-p) x2)/sqrt(p^2+(1-p)^2),
    soft label r / 1-r (r, not p).
  * SpecAugment — ``ASTPreprocessor.apply_specaugment`` (preprocessing.py:1075-1104).
  * Mixup — ``MixupDataset.apply_mixup`` (src/datasets/esc50.py:52-76) around
    ``MixupAugmentation.__call__`` (preprocessing.py:935-968), including the same-class label
    overwrite (soft[l2] = 1 - lam written after soft[l1] = lam).
  * Time stretch + gain — ``EnvNetPreprocessor.apply_augmentation`` (preprocessing.py:886-925).
The Python ``random`` draws are replayed in the reference's order so that, seeded alike, the
restatement makes the same choices as the reference; the GPU path draws on the device and is fed
the oracle's choices explicitly by the parity tests.

Pinning: tests/golden/golden.npz (bcmix_*) and tests/golden/golden_aug.npz, both written by
tests/golden/make_golden.py running the reference's own classes.
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------------- BC mixing
def a_weighted_spl(w: torch.Tensor) -> float:
    """preprocessing.py:395-419: float32 RMS -> 20 log10(rms) + 94, or -80 for silence."""
    w = torch.as_tensor(w, dtype=torch.float32)
    rms = torch.sqrt(torch.mean(w ** 2))
    if rms > 0:
        return float(20 * torch.log10(rms) + 94)
    return -80.0


def perceptual_mixing_coefficient(r: float, spl1: float, spl2: float) -> float:
    """preprocessing.py:421-447 (Python double arithmetic, float32 clamp)."""
    d = spl1 - spl2
    if abs(d) > 10:
        adj = min(abs(d) / 40.0, 0.3)
        r = r * (1 - adj) if spl1 > spl2 else r * (1 + adj)
    return float(torch.clamp(torch.tensor(r), 0.0, 1.0))


def mix_waveforms(w1: torch.Tensor, w2: torch.Tensor, p: float) -> torch.Tensor:
    """preprocessing.py:449-471."""
    n = min(w1.shape[-1], w2.shape[-1])
    w1, w2 = w1[..., :n], w2[..., :n]
    return (p * w1 + (1 - p) * w2) / torch.sqrt(torch.tensor(p ** 2 + (1 - p) ** 2))


def soft_labels(r: float, l1: int, l2: int, num_classes: int) -> torch.Tensor:
    """preprocessing.py:473-490 (l2 written last: a same-class pair keeps 1 - r)."""
    y = torch.zeros(num_classes, dtype=torch.float32)
    y[l1] = r
    y[l2] = 1 - r
    return y


def one_hot(label: int, num_classes: int) -> torch.Tensor:
    y = torch.zeros(num_classes, dtype=torch.float32)
    y[label] = 1.0
    return y


def bc_mix_one(wave: torch.Tensor, partner: torch.Tensor, r: float, label: int, partner_label: int,
               num_classes: int):
    """Mix one clip with a given partner and ratio: (mixed, soft label, p)."""
    p = perceptual_mixing_coefficient(r, a_weighted_spl(wave), a_weighted_spl(partner))
    return mix_waveforms(wave, partner, p), soft_labels(r, label, partner_label, num_classes), p


def apply_bc_mixing(wave: torch.Tensor, label: int, pool: list, pool_labels: list, num_classes: int,
                    rng: random.Random):
    """BCMixingDataset.apply_bc_mixing (preprocessing.py:564-609) with the draws replayed from ``rng``:
    returns (mixed, soft label, partner pool index or -1, r or None, p or None)."""
    diff = [i for i, l in enumerate(pool_labels) if l != label]
    if not diff:
        return wave, one_hot(label, num_classes), -1, None, None
    q = rng.choice(diff)          # random.choice(different_class_samples), :591
    r = rng.random()              # :594
    mixed, y, p = bc_mix_one(wave, pool[q], r, label, pool_labels[q], num_classes)
    return mixed, y, q, r, p


def partner_from_uniform(u: float, label: int, pool_labels) -> int:
    """The device partner draw (mia_bc_partner): k = min(floor(u * n_diff), n_diff - 1), the k-th
    different-class clip in pool order — the same element ``random.choice`` over the filtered list
    (preprocessing.py:584-591) returns for that k; -1 when no other class exists."""
    diff = [i for i, l in enumerate(list(pool_labels)) if l != label]
    if not diff:
        return -1
    k = min(int(math.floor(np.float32(u) * np.float32(len(diff)))), len(diff) - 1)
    return diff[k]


# ----------------------------------------------------------------------------------- SpecAugment
def specaugment(spec: torch.Tensor, time_mask: int = 192, freq_mask: int = 48, rng: random.Random | None = None,
                params=None):
    """ASTPreprocessor.apply_specaugment (preprocessing.py:1075-1104) on a (C, F, T) spectrogram.
    Draws replayed from ``rng`` (or taken from ``params`` = (t0, tl, f0, fl)); returns
    (masked spec, (t0, tl, f0, fl)) with tl / fl = 0 where a mask is not applied."""
    spec = spec.clone()
    _, n_mels, n_frames = spec.shape
    t0 = tl = f0 = fl = 0
    if params is not None:
        t0, tl, f0, fl = params
    else:
        if time_mask > 0 and n_frames > time_mask:
            tl = rng.randint(1, min(time_mask, n_frames // 4))
            t0 = rng.randint(0, n_frames - tl)
        if freq_mask > 0 and n_mels > freq_mask:
            fl = rng.randint(1, min(freq_mask, n_mels // 4))
            f0 = rng.randint(0, n_mels - fl)
    if tl:
        spec[:, :, t0:t0 + tl] = 0
    if fl:
        spec[:, f0:f0 + fl, :] = 0
    return spec, (t0, tl, f0, fl)


# ----------------------------------------------------------------------------------- Mixup
def mixup_apply(spec1: torch.Tensor, spec2: torch.Tensor, lam, l1: int, l2: int, num_classes: int):
    """MixupAugmentation.__call__ arithmetic (preprocessing.py:960-968); lam a 0-dim f32 tensor."""
    lam = torch.as_tensor(lam, dtype=torch.float32)
    mixed = lam * spec1 + (1 - lam) * spec2
    y = torch.zeros(num_classes, dtype=torch.float32)
    y[l1] = lam
    y[l2] = 1 - lam
    return mixed, y


def apply_mixup(spec: torch.Tensor, label: int, pool: list, pool_labels: list, num_classes: int, alpha: float,
                rng: random.Random):
    """MixupDataset.apply_mixup (esc50.py:64-76) -> MixupAugmentation(alpha, prob=0.5) (:50,
    preprocessing.py:949-958) with the Python draws replayed from ``rng`` and lam drawn from torch's
    global generator like the reference.  Returns (spec, soft label, partner or -1, lam or None)."""
    if rng.random() > 0.5:                                   # esc50.py:64
        return spec, one_hot(label, num_classes), -1, None
    q = rng.randint(0, len(pool) - 1)                        # esc50.py:70
    if rng.random() > 0.5:                                   # preprocessing.py:949, prob=0.5
        return spec, one_hot(label, num_classes), -1, None
    lam = torch.distributions.Beta(alpha, alpha).sample() if alpha > 0 else torch.tensor(1.0)
    mixed, y = mixup_apply(spec, pool[q], lam, label, pool_labels[q], num_classes)
    return mixed, y, q, float(lam)


# ----------------------------------------------------------------------------------- stretch / gain
def time_stretch(w: torch.Tensor, factor: float) -> torch.Tensor:
    """preprocessing.py:900-915: linear resample (align_corners=False) to int(T / factor) samples."""
    n = w.shape[-1]
    m = int(n / factor)
    if m == n:
        return w
    return F.interpolate(w.reshape(1, 1, n), size=m, mode="linear", align_corners=False).reshape(*w.shape[:-1], m)


def apply_augmentation(w: torch.Tensor, cfg: dict, rng: random.Random):
    """EnvNetPreprocessor.apply_augmentation (preprocessing.py:886-925) with the draws replayed from
    ``rng``: returns (waveform, stretch factor or None, linear gain or None)."""
    factor = gain = None
    if not cfg:
        return w, factor, gain
    if "time_stretch" in cfg and rng.random() < 0.5:
        rngs = cfg["time_stretch"]
        if isinstance(rngs, list) and len(rngs) == 2:
            factor = rng.uniform(rngs[0], rngs[1])
            w = time_stretch(w, factor)
    if "gain_shift" in cfg and rng.random() < 0.5:
        g = cfg["gain_shift"]
        if isinstance(g, list) and len(g) == 2:
            gain = 10 ** (rng.uniform(g[0], g[1]) / 20.0)
            w = w * gain
    return w, factor, gain
