"""On-GPU batch augmentations with the reference's semantics.

* ``bc_mix`` — between-class mixing (BCMixingDataset.apply_bc_mixing,
  src/datasets/preprocessing.py:564-609 + BCMixingUtils :395-490): partner drawn uniformly from
  clips of a *different* class, r ~ U(0,1), RMS-"SPL" perceptual adjustment of r -> p, mix
  (p x1 + (1-p) x2) / sqrt(p^2 + (1-p)^2), soft label r / 1-r (uses r, not p).
* ``spec_augment_mixup`` — SpecAugment (preprocessing.py:1075-1104) then Mixup
  (esc50.py:52-76, preprocessing.py:935-968): time mask len U[1, min(T_max, F/4)], freq mask
  len U[1, min(F_max, 128/4)], zero fill; with prob 0.5*0.5 mix with an un-augmented partner,
  lam ~ Beta(alpha, alpha); labels lam / 1-lam with same-class overwrite to 1-lam.
The random draws are made with torch generators (host or device); the per-element work runs in
the fused HIP kernels.  Draws cannot reproduce Python's ``random`` stream, so parity is
statistical (distributions), the per-element arithmetic is exact.
"""
from __future__ import annotations

import torch

from ..miaudio import lib as L


def _pool_partner(labels: torch.Tensor, pool_labels: torch.Tensor, gen: torch.Generator | None,
                  rounds: int = 12) -> torch.Tensor:
    """For each clip, an index into the pool drawn uniformly among clips of a different class.
    Rejection sampling with a fixed number of rounds and no host synchronisation; with >= 2
    classes the chance a clip is still unmatched after 12 rounds is < (1 - 1/C)^0 * (B_same/B)^12."""
    n = pool_labels.numel()
    B = labels.numel()
    dev = labels.device
    q = torch.randint(0, n, (B,), generator=gen, device=dev)
    for _ in range(rounds):
        bad = pool_labels[q] == labels
        q = torch.where(bad, torch.randint(0, n, (B,), generator=gen, device=dev), q)
    return q


def bc_mix(wav: torch.Tensor, labels: torch.Tensor, num_classes: int, gen: torch.Generator | None = None,
           r: torch.Tensor | None = None, partner: torch.Tensor | None = None):
    """wav (B, T) f32 CUDA, labels (B,) int64 -> (mixed (B, T), soft labels (B, C), p (B,)).
    Partners are drawn from the batch itself (the batch is the resident clip pool)."""
    L.require_device(wav, "bc_mix")
    wav = wav.reshape(wav.shape[0], -1).contiguous().float()
    B, T = wav.shape
    labels = labels.to(torch.int64).contiguous()
    if partner is None:
        partner = _pool_partner(labels, labels, gen)
    partner = partner.to(torch.int32).contiguous()
    if r is None:
        r = torch.rand(B, generator=gen, device=wav.device)
    r = r.float().contiguous()
    out = torch.empty_like(wav)
    y = torch.empty(B, num_classes, dtype=torch.float32, device=wav.device)
    p = torch.empty(B, dtype=torch.float32, device=wav.device)
    L.check(L.load().mia_bc_mix(wav.data_ptr(), T, B, partner.data_ptr(), r.data_ptr(), labels.data_ptr(),
                                num_classes, out.data_ptr(), y.data_ptr(), p.data_ptr(), L.stream_ptr()), "mia_bc_mix")
    return out, y, p


def spec_augment_mixup(spec: torch.Tensor, labels: torch.Tensor, num_classes: int, time_mask: int = 192,
                       freq_mask: int = 48, mixup_alpha: float = 0.5, mixup_prob: float = 0.25,
                       gen: torch.Generator | None = None, specaug: bool = True, mixup: bool = True):
    """spec (B, F, T) f32 CUDA -> (augmented spec, soft labels (B, C))."""
    L.require_device(spec, "spec_augment_mixup")
    spec = spec.contiguous().float()
    B, Fm, T = spec.shape
    dev = spec.device
    labels = labels.to(torch.int64)
    z = torch.zeros(B, dtype=torch.int32, device=dev)
    t0 = tl = f0 = fl = z
    if specaug:
        if time_mask > 0 and T > time_mask:
            tl = torch.randint(1, min(time_mask, T // 4) + 1, (B,), generator=gen, device=dev).int()
            t0 = (torch.rand(B, generator=gen, device=dev) * (T - tl + 1).float()).floor().int()
        if freq_mask > 0 and Fm > freq_mask:
            fl = torch.randint(1, min(freq_mask, Fm // 4) + 1, (B,), generator=gen, device=dev).int()
            f0 = (torch.rand(B, generator=gen, device=dev) * (Fm - fl + 1).float()).floor().int()
    partner = torch.full((B,), -1, dtype=torch.int32, device=dev)
    lam = torch.ones(B, dtype=torch.float32, device=dev)
    if mixup:
        do = torch.rand(B, generator=gen, device=dev) < mixup_prob
        q = torch.randint(0, B, (B,), generator=gen, device=dev)
        partner = torch.where(do, q, torch.full_like(q, -1)).int()
        beta = torch.distributions.Beta(torch.tensor(mixup_alpha, device=dev), torch.tensor(mixup_alpha, device=dev))
        lam = torch.where(do, beta.sample((B,)).float(), lam)
    out = torch.empty_like(spec)
    L.check(L.load().mia_spec_augment_mixup(spec.data_ptr(), out.data_ptr(), B, Fm, T, t0.data_ptr(), tl.data_ptr(),
                                            f0.data_ptr(), fl.data_ptr(), partner.data_ptr(), lam.data_ptr(),
                                            L.stream_ptr()), "mia_spec_augment_mixup")
    y = torch.zeros(B, num_classes, dtype=torch.float32, device=dev)
    y.scatter_(1, labels.view(-1, 1), 1.0)
    mixed = partner >= 0
    if bool(mixed.any()):
        pl = labels[partner.clamp_min(0).long()]
        ym = torch.zeros_like(y)
        ym.scatter_(1, labels.view(-1, 1), lam.view(-1, 1))
        ym.scatter_(1, pl.view(-1, 1), (1 - lam).view(-1, 1))  # same class: overwritten to 1-lam
        y = torch.where(mixed.view(-1, 1), ym, y)
    return out, y
