"""On-GPU batch augmentations with the reference's semantics.

* ``bc_mix`` — between-class mixing (BCMixingDataset.apply_bc_mixing,
  src/datasets/preprocessing.py:564-609 + BCMixingUtils :395-490): partner drawn uniformly from
  pool clips of a *different* class, r ~ U(0,1), RMS-"SPL" perceptual adjustment of r -> p, mix
  (p x1 + (1-p) x2) / sqrt(p^2 + (1-p)^2), soft label r / 1-r (uses r, not p).
* ``spec_augment_mixup`` — SpecAugment (preprocessing.py:1075-1104) then Mixup
  (esc50.py:52-76, preprocessing.py:935-968): time mask len U[1, min(T_max, F/4)], freq mask
  len U[1, min(F_max, 128/4)], zero fill; with prob 0.5*0.5 mix with an un-augmented partner drawn
  from the pool (any class), lam ~ Beta(alpha, alpha); labels lam / 1-lam with the same-class
  overwrite to 1-lam.
The pool is the resident training set (or the batch itself).  Random draws use torch generators
(no host synchronisation); the per-element work runs in the fused HIP kernels.  The draws cannot
reproduce Python's ``random`` stream, so augmentation parity is distributional; the arithmetic is
exact (tests/test_gpu_augment.py).
"""
from __future__ import annotations

import torch

from ..miaudio import kernels as K
from ..miaudio import lib as L


def _pool_partner(labels: torch.Tensor, pool_labels: torch.Tensor, gen: torch.Generator | None,
                  rounds: int = 16) -> torch.Tensor:
    """Index into the pool drawn uniformly among clips of a different class (rejection sampling with a
    fixed number of rounds, no host synchronisation)."""
    n = pool_labels.numel()
    B = labels.numel()
    dev = labels.device
    q = torch.randint(0, n, (B,), generator=gen, device=dev)
    for _ in range(rounds):
        bad = pool_labels[q] == labels
        q = torch.where(bad, torch.randint(0, n, (B,), generator=gen, device=dev), q)
    return q


def bc_mix(wav: torch.Tensor, labels: torch.Tensor, num_classes: int, gen: torch.Generator | None = None,
           r: torch.Tensor | None = None, partner: torch.Tensor | None = None,
           pool: torch.Tensor | None = None, pool_labels: torch.Tensor | None = None):
    """wav (B, T) f32 CUDA, labels (B,) int64 -> (mixed (B, T), soft labels (B, C), p (B,))."""
    L.require_device(wav, "bc_mix")
    wav = wav.reshape(wav.shape[0], -1).contiguous().float()
    B, T = wav.shape
    labels = labels.to(torch.int64).contiguous()
    if pool is None:
        pool, pool_labels = wav, labels
    pool = pool.reshape(pool.shape[0], -1).contiguous().float()
    pool_labels = pool_labels.to(torch.int64).contiguous()
    if pool.shape[1] != T:
        raise ValueError(f"pool clips have {pool.shape[1]} samples, batch {T}")
    if partner is None:
        partner = _pool_partner(labels, pool_labels, gen)
    partner = partner.to(torch.int32).contiguous()
    if r is None:
        r = torch.rand(B, generator=gen, device=wav.device)
    r = r.float().contiguous()
    out = torch.empty_like(wav)
    y = torch.empty(B, num_classes, dtype=torch.float32, device=wav.device)
    p = torch.empty(B, dtype=torch.float32, device=wav.device)
    ws = K.workspace(8 * B + 64, wav.device, "bcmix")
    L.check(L.load().mia_bc_mix(wav.data_ptr(), pool.data_ptr(), T, B, partner.data_ptr(), r.data_ptr(),
                                labels.data_ptr(), pool_labels.data_ptr(), num_classes, out.data_ptr(), y.data_ptr(),
                                p.data_ptr(), ws.data_ptr(), L.stream_ptr()), "mia_bc_mix")
    return out, y, p


def spec_augment_mixup(spec: torch.Tensor, labels: torch.Tensor, num_classes: int, time_mask: int = 192,
                       freq_mask: int = 48, mixup_alpha: float = 0.5, mixup_prob: float = 0.25,
                       gen: torch.Generator | None = None, specaug: bool = True, mixup: bool = True,
                       pool: torch.Tensor | None = None, pool_labels: torch.Tensor | None = None):
    """spec (B, F, T) f32 CUDA -> (augmented spec, soft labels (B, C))."""
    L.require_device(spec, "spec_augment_mixup")
    spec = spec.contiguous().float()
    B, Fm, T = spec.shape
    dev = spec.device
    labels = labels.to(torch.int64)
    if pool is None:
        pool, pool_labels = spec, labels
    pool = pool.contiguous().float()
    pool_labels = pool_labels.to(torch.int64)
    z = torch.zeros(B, dtype=torch.int32, device=dev)
    t0 = tl = f0 = fl = z
    if specaug:
        if time_mask > 0 and T > time_mask:
            tl = torch.randint(1, min(time_mask, T // 4) + 1, (B,), generator=gen, device=dev).int()
            t0 = (torch.rand(B, generator=gen, device=dev) * (T - tl + 1).float()).floor().int()
        if freq_mask > 0 and Fm > freq_mask:
            fl = torch.randint(1, min(freq_mask, Fm // 4) + 1, (B,), generator=gen, device=dev).int()
            f0 = (torch.rand(B, generator=gen, device=dev) * (Fm - fl + 1).float()).floor().int()
    partner = None
    lam = torch.ones(B, dtype=torch.float32, device=dev)
    if mixup:
        do = torch.rand(B, generator=gen, device=dev) < mixup_prob
        q = torch.randint(0, pool.shape[0], (B,), generator=gen, device=dev)
        partner = torch.where(do, q, torch.full_like(q, -1)).int().contiguous()
        # Beta(a, a) via two Gamma draws (device generator)
        ga = torch._standard_gamma(torch.full((B,), mixup_alpha, device=dev), generator=gen)
        gb = torch._standard_gamma(torch.full((B,), mixup_alpha, device=dev), generator=gen)
        lam = torch.where(do, (ga / (ga + gb)).float(), lam).contiguous()
    out = torch.empty_like(spec)
    L.check(L.load().mia_spec_augment_mixup(spec.data_ptr(), pool.data_ptr(), out.data_ptr(), B, Fm, T,
                                            t0.data_ptr(), tl.data_ptr(), f0.data_ptr(), fl.data_ptr(),
                                            L.ptr(partner), lam.data_ptr(), L.stream_ptr()), "mia_spec_augment_mixup")
    y = torch.zeros(B, num_classes, dtype=torch.float32, device=dev)
    y.scatter_(1, labels.view(-1, 1), 1.0)
    if partner is not None:
        mixed = (partner >= 0).view(-1, 1)
        pl = pool_labels[partner.clamp_min(0).long()]
        ym = torch.zeros_like(y)
        ym.scatter_(1, labels.view(-1, 1), lam.view(-1, 1))
        ym.scatter_(1, pl.view(-1, 1), (1 - lam).view(-1, 1))  # same class: overwritten to 1-lam
        y = torch.where(mixed, ym, y)
    return out, y
