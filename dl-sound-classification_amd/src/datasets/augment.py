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
* ``stretch_gain`` — time stretch + gain shift (EnvNetPreprocessor.apply_augmentation,
  preprocessing.py:886-925), each with probability 0.5.
The pool is the resident training set (or the batch itself).  Random draws use torch generators on
the device (no host synchronisation); the per-element work and the partner search run in HIP
kernels.  The draws cannot reproduce Python's ``random`` stream, so the *choices* match the
reference in distribution; given the same choices (partner, r, masks, lam, factor, gain) the outputs
match the reference's golden vectors (tests/test_gpu_augment.py, tests/golden/golden_aug.npz).
"""
from __future__ import annotations

import torch

from ..miaudio import kernels as K
from ..miaudio import lib as L


def bc_partner(labels: torch.Tensor, pool_labels: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """Partner index per clip, uniform among the pool clips of a different class (mia_bc_partner;
    preprocessing.py:584-591), from uniforms u (B,) f32; -1 where the pool has no other class."""
    labels = labels.to(torch.int64).contiguous()
    pool_labels = pool_labels.to(torch.int64).contiguous()
    u = u.float().contiguous()
    out = torch.empty(labels.numel(), dtype=torch.int32, device=labels.device)
    L.check(L.load().mia_bc_partner(labels.data_ptr(), labels.numel(), pool_labels.data_ptr(), pool_labels.numel(),
                                    u.data_ptr(), out.data_ptr(), L.stream_ptr()), "mia_bc_partner")
    return out


def bc_mix_cpu(wav: torch.Tensor, labels: torch.Tensor, num_classes: int, pool: torch.Tensor,
               pool_labels: torch.Tensor, gen: torch.Generator | None = None):
    """BC mixing with torch CPU ops — ONLY for ``trainer.accelerator=cpu`` runs (BASELINE config 1, the
    reference's CPU plumbing configuration), where the batch never reaches a GPU.  Same formulas and
    partner rule as mia_bc_mix / mia_bc_partner (preprocessing.py:395-490,564-609)."""
    wav = wav.reshape(wav.shape[0], -1).float()
    pool = pool.reshape(pool.shape[0], -1).float()
    B = wav.shape[0]
    u = torch.rand(B, generator=gen)
    r = torch.rand(B, generator=gen)
    diff = pool_labels.view(1, -1) != labels.view(-1, 1)                    # (B, N)
    nd = diff.sum(1)
    k = torch.minimum((u * nd.float()).floor().long(), (nd - 1).clamp_min(0))
    q = torch.argmax(((diff.cumsum(1) == (k + 1).view(-1, 1)) & diff).int(), dim=1)  # k-th other-class clip
    has = nd > 0

    def spl(x):
        rms = torch.sqrt(torch.mean(x ** 2, dim=1))
        return torch.where(rms > 0, 20 * torch.log10(rms) + 94, torch.full_like(rms, -80.0)).double()

    d = spl(wav) - spl(pool[q])
    adj = torch.clamp(d.abs() / 40.0, max=0.3)
    rd = r.double()
    pd = torch.where(d.abs() > 10, torch.where(d > 0, rd * (1 - adj), rd * (1 + adj)), rd)
    p = pd.float().clamp(0.0, 1.0)
    norm = torch.sqrt((p.double() ** 2 + (1 - p.double()) ** 2).float())
    mixed = (p.view(-1, 1) * wav + (1 - p).view(-1, 1) * pool[q]) / norm.view(-1, 1)
    out = torch.where(has.view(-1, 1), mixed, wav)
    y = torch.zeros(B, num_classes)
    y.scatter_(1, labels.view(-1, 1), torch.where(has, r, torch.ones_like(r)).view(-1, 1))
    yq = torch.zeros(B, num_classes)
    yq.scatter_(1, pool_labels[q].view(-1, 1), (1 - r).view(-1, 1))
    y = torch.where(has.view(-1, 1) & (yq > 0), yq, y)
    return out, y, torch.where(has, p, torch.ones_like(p))


def bc_mix(wav: torch.Tensor, labels: torch.Tensor, num_classes: int, gen: torch.Generator | None = None,
           r: torch.Tensor | None = None, partner: torch.Tensor | None = None,
           pool: torch.Tensor | None = None, pool_labels: torch.Tensor | None = None):
    """wav (B, T) f32 CUDA, labels (B,) int64 -> (mixed (B, T), soft labels (B, C), p (B,))."""
    L.require_device(wav, "bc_mix")
    wav = wav.reshape(wav.shape[0], -1).contiguous().float()
    B, T = wav.shape
    labels = labels.to(device=wav.device, dtype=torch.int64).contiguous()
    if pool is None:
        pool, pool_labels = wav, labels
    pool = pool.reshape(pool.shape[0], -1).contiguous().float()
    pool_labels = pool_labels.to(torch.int64).contiguous()
    if pool.shape[1] != T:
        raise ValueError(f"pool clips have {pool.shape[1]} samples, batch {T}")
    if partner is None:
        partner = bc_partner(labels, pool_labels, torch.rand(B, generator=gen, device=wav.device))
    partner = partner.to(device=wav.device, dtype=torch.int32).contiguous()
    if r is None:
        r = torch.rand(B, generator=gen, device=wav.device)
    r = r.to(device=wav.device, dtype=torch.float32).contiguous()
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
                       pool: torch.Tensor | None = None, pool_labels: torch.Tensor | None = None,
                       masks=None, partner: torch.Tensor | None = None, lam: torch.Tensor | None = None):
    """spec (B, F, T) f32 CUDA -> (augmented spec, soft labels (B, C)).  ``masks`` = (t0, tl, f0, fl)
    int (B,) tensors and ``partner`` (int, -1 = no mixup) / ``lam`` (f32) override the draws."""
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
    if masks is not None:
        t0, tl, f0, fl = (torch.as_tensor(m, device=dev).int().contiguous() for m in masks)
    elif specaug:
        if time_mask > 0 and T > time_mask:
            tl = torch.randint(1, min(time_mask, T // 4) + 1, (B,), generator=gen, device=dev).int()
            t0 = (torch.rand(B, generator=gen, device=dev) * (T - tl + 1).float()).floor().int()
        if freq_mask > 0 and Fm > freq_mask:
            fl = torch.randint(1, min(freq_mask, Fm // 4) + 1, (B,), generator=gen, device=dev).int()
            f0 = (torch.rand(B, generator=gen, device=dev) * (Fm - fl + 1).float()).floor().int()
    if partner is not None:
        partner = partner.to(dev).int().contiguous()
        lam = lam.to(dev).float().contiguous()
    elif mixup:
        do = torch.rand(B, generator=gen, device=dev) < mixup_prob
        q = torch.randint(0, pool.shape[0], (B,), generator=gen, device=dev)
        partner = torch.where(do, q, torch.full_like(q, -1)).int().contiguous()
        # Beta(a, a) via two Gamma draws (device generator)
        ga = torch._standard_gamma(torch.full((B,), mixup_alpha, device=dev), generator=gen)
        gb = torch._standard_gamma(torch.full((B,), mixup_alpha, device=dev), generator=gen)
        lam = torch.where(do, (ga / (ga + gb)).float(), torch.ones_like(ga)).contiguous()
    else:
        lam = torch.ones(B, dtype=torch.float32, device=dev)
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


def stretch_gain(wav: torch.Tensor, time_stretch=None, gain_shift=None, gen: torch.Generator | None = None,
                 factor: torch.Tensor | None = None, gain: torch.Tensor | None = None) -> torch.Tensor:
    """wav (B, T) f32 CUDA -> (B, T).  Per clip, with probability 0.5 each (preprocessing.py:900,918):
    stretch by factor ~ U(time_stretch) (linear resample to int(T / factor) samples, kept in the
    T-sample window) and scale by 10^(U(gain_shift)/20).  ``factor`` (f64, <= 0: none) / ``gain``
    (f32) override the draws."""
    L.require_device(wav, "stretch_gain")
    wav = wav.reshape(wav.shape[0], -1).contiguous().float()
    B, T = wav.shape
    dev = wav.device
    if factor is None and isinstance(time_stretch, (list, tuple)) and len(time_stretch) == 2:
        lo, hi = float(time_stretch[0]), float(time_stretch[1])
        on = torch.rand(B, generator=gen, device=dev, dtype=torch.float64) < 0.5
        f = lo + (hi - lo) * torch.rand(B, generator=gen, device=dev, dtype=torch.float64)
        factor = torch.where(on, f, torch.zeros_like(f))
    if gain is None and isinstance(gain_shift, (list, tuple)) and len(gain_shift) == 2:
        lo, hi = float(gain_shift[0]), float(gain_shift[1])
        on = torch.rand(B, generator=gen, device=dev) < 0.5
        db = lo + (hi - lo) * torch.rand(B, generator=gen, device=dev, dtype=torch.float64)
        gain = torch.where(on, torch.pow(10.0, db / 20.0), torch.ones_like(db)).float()
    if factor is None and gain is None:
        return wav
    factor = None if factor is None else factor.to(device=dev, dtype=torch.float64).contiguous()
    gain = None if gain is None else gain.to(device=dev, dtype=torch.float32).contiguous()
    out = torch.empty_like(wav)
    L.check(L.load().mia_stretch_gain(wav.data_ptr(), T, B, L.ptr(factor), L.ptr(gain), out.data_ptr(),
                                      L.stream_ptr()), "mia_stretch_gain")
    return out
