"""GPU: the on-device augmentation kernels against the reference's golden vectors and the oracle.

Given the same choices (partner, r, masks, lam, stretch factor, gain) the HIP kernels reproduce the
reference's outputs: BC mixing (mia_bc_mix; preprocessing.py:395-490,564-609) and Mixup
(mia_spec_augment_mixup; preprocessing.py:935-968, esc50.py:52-76) are computed op by op in IEEE
f32 like the reference; SpecAugment masking is exact; the time-stretch resample follows
F.interpolate(linear, align_corners=False) (preprocessing.py:886-925).  The device partner draw
(mia_bc_partner) is exact against the oracle's mapping and never returns a same-class clip."""
import random

import numpy as np
import pytest
import torch

from oracle import augment as oaug
from oracle.synth import synth_waveform
from tests._aug_inputs import (AUG_BC_LABELS, AUG_MIX_LABELS, AUG_SPEC_CASES, AUG_STRETCH_CFG, aug_bc_pool,
                               aug_mix_pool, aug_spec_input, aug_stretch_input)

pytestmark = pytest.mark.gpu


def _cs(a, g, prefix, atol, rel=1e-6):
    a = np.asarray(a, np.float64).ravel()
    np.testing.assert_allclose(a[g[f"{prefix}__idx"]], g[f"{prefix}__vals"], atol=atol, rtol=0)
    np.testing.assert_allclose(a.sum(), g[f"{prefix}__sum"], rtol=rel, atol=1e-3)
    np.testing.assert_allclose((a * a).sum(), g[f"{prefix}__sumsq"], rtol=rel)


def test_bc_mix_matches_reference_utils(cuda, golden):
    """golden.npz bcmix_*: BCMixingUtils on two full clips (one ~26 dB quieter: perceptual branch)."""
    from src.datasets.augment import bc_mix
    w1 = synth_waveform(41, 1, 220_500)
    w2 = synth_waveform(42, 1, 220_500) * np.float32(0.05)
    pairs = [(w1, w2), (w2, w1), (w1, w1 * np.float32(0.9))]
    k = 0
    for r in golden["bcmix_r"]:
        x = torch.from_numpy(np.concatenate([a for a, _ in pairs])).to(cuda)
        pool = torch.from_numpy(np.concatenate([b for _, b in pairs])).to(cuda)
        out, y, p = bc_mix(x, torch.tensor([3, 3, 3], device=cuda), 50, r=torch.full((3,), float(r), device=cuda),
                           partner=torch.arange(3, device=cuda), pool=pool,
                           pool_labels=torch.tensor([17, 17, 17], device=cuda))
        out, p = out.cpu().numpy().astype(np.float64), p.cpu().numpy()
        for j in range(3):
            ref_p = golden["bcmix_spl_p"][k][2]
            assert abs(p[j] - ref_p) <= 1e-7, (k, p[j], ref_p)
            cs = golden["bcmix_mix_cs"][k]
            assert out[j].sum() == pytest.approx(cs[0], rel=1e-5, abs=1e-3)
            assert (out[j] ** 2).sum() == pytest.approx(cs[1], rel=1e-6)
            assert abs(out[j, 1234] - cs[2]) <= 1e-7 and abs(out[j, 99999] - cs[3]) <= 1e-7
            k += 1
        yc = y.cpu().numpy()
        assert yc[0, 3] == np.float32(r) and yc[0, 17] == np.float32(1 - np.float32(r)) and yc[0].sum() == pytest.approx(1)
    lab = golden["bcmix_soft_label"]
    assert lab[3] == np.float32(0.37) and lab[17] == np.float32(1 - 0.37)


def test_bc_mix_dataset_cases(cuda, golden_aug):
    """golden_aug aug_bc*: apply_bc_mixing with the reference's own draws (replayed by the oracle)."""
    from src.datasets.augment import bc_mix
    pool_np = np.concatenate(aug_bc_pool())
    pool = torch.from_numpy(pool_np).to(cuda)
    pool_labels = torch.tensor(AUG_BC_LABELS, device=cuda)
    tp = [torch.from_numpy(w) for w in aug_bc_pool()]
    for s in range(8):
        i = s % len(tp)
        _, _, q, r, p_ref = oaug.apply_bc_mixing(tp[i], AUG_BC_LABELS[i], tp, list(AUG_BC_LABELS), 4,
                                                 random.Random(1000 + s))
        out, y, p = bc_mix(pool[i:i + 1], pool_labels[i:i + 1], 4, r=torch.tensor([r], device=cuda),
                           partner=torch.tensor([q], device=cuda), pool=pool, pool_labels=pool_labels)
        # r reaches the kernel as f32 (the reference keeps Python's double): p within 1 f32 ulp
        assert abs(float(p[0]) - p_ref) <= 1.2e-7, (s, float(p[0]), p_ref)
        _cs(out.cpu().numpy(), golden_aug, f"aug_bc{s}", 2e-7, rel=1e-5)
        np.testing.assert_allclose(y.cpu().numpy()[0], golden_aug[f"aug_bc{s}__y"], atol=1e-7, rtol=0)


def test_bc_mix_same_class_pool_keeps_clip(cuda, golden_aug):
    from src.datasets.augment import bc_mix
    pool = torch.from_numpy(np.concatenate(aug_bc_pool()[:2])).to(cuda)
    g = torch.Generator(device=cuda).manual_seed(0)
    out, y, p = bc_mix(pool[:1], torch.tensor([0], device=cuda), 4, gen=g, pool=pool,
                       pool_labels=torch.tensor([0, 0], device=cuda))
    assert torch.equal(out, pool[:1]) and bool(golden_aug["aug_bc_sameclass__equal"])
    np.testing.assert_array_equal(y.cpu().numpy()[0], golden_aug["aug_bc_sameclass__y"])


def test_bc_partner_exact_and_never_same_class(cuda):
    from src.datasets.augment import bc_partner
    g = torch.Generator().manual_seed(5)
    N, B, C = 1440, 256, 50
    pool_labels = torch.randint(0, C, (N,), generator=g)
    labels = torch.randint(0, C, (B,), generator=g)
    u = torch.rand(B, generator=g)
    u[:4] = torch.tensor([0.0, 0.999999, 0.5, 1e-9])
    q = bc_partner(labels.to(cuda), pool_labels.to(cuda), u.to(cuda)).cpu()
    ref = [oaug.partner_from_uniform(float(u[b]), int(labels[b]), pool_labels.tolist()) for b in range(B)]
    assert q.tolist() == ref
    assert bool((pool_labels[q.long()] != labels).all())
    # a pool without another class -> -1 (reference: unmixed clip, one-hot label)
    q = bc_partner(torch.tensor([2, 3], device=cuda), torch.tensor([2, 2, 2], device=cuda),
                   torch.tensor([0.3, 0.3], device=cuda)).cpu()
    assert q.tolist() == [-1, 0]


def test_bc_partner_uniform_over_other_classes(cuda):
    """random.choice over the different-class clips: each candidate equally likely."""
    from src.datasets.augment import bc_partner
    pool_labels = torch.tensor([0, 1, 1, 2, 0, 3, 1, 0, 2, 2], device=cuda)
    B = 200_000
    labels = torch.zeros(B, dtype=torch.int64, device=cuda)
    u = torch.rand(B, generator=torch.Generator(device=cuda).manual_seed(1), device=cuda)
    q = bc_partner(labels, pool_labels, u)
    counts = torch.bincount(q.long(), minlength=10).cpu().double()
    cand = (pool_labels != 0).cpu()
    assert counts[~cand].sum() == 0
    exp = B / int(cand.sum())
    chi2 = float(((counts[cand] - exp) ** 2 / exp).sum())
    assert chi2 < 30.0, chi2  # 6 dof: p < 1e-4


def test_bc_mix_default_draws(cuda):
    """End to end with device draws: every mixed clip has a different-class partner, labels sum to 1."""
    from src.datasets.augment import bc_mix
    g = torch.Generator(device=cuda).manual_seed(3)
    B, T = 64, 4096
    wav = torch.rand(B, T, generator=g, device=cuda) - 0.5
    labels = torch.randint(0, 3, (B,), generator=g, device=cuda)
    out, y, p = bc_mix(wav, labels, 3, gen=g)
    assert torch.isfinite(out).all() and ((p >= 0) & (p <= 1)).all()
    torch.testing.assert_close(y.sum(1), torch.ones(B, device=cuda))
    assert (y.gt(0).sum(1) <= 2).all() and (y[torch.arange(B), labels] > 0).all()


def test_specaugment_exact(cuda, golden_aug):
    from src.datasets.augment import spec_augment_mixup
    for s, (shape, tm, fm) in enumerate(AUG_SPEC_CASES):
        spec = torch.from_numpy(aug_spec_input(s))
        _, (t0, tl, f0, fl) = oaug.specaugment(spec, tm, fm, random.Random(2000 + s))
        x = spec.to(cuda)  # (1, F, T): C = 1 as the reference, B = 1 here
        out, y = spec_augment_mixup(x, torch.tensor([1], device=cuda), 10, mixup=False,
                                    masks=([t0], [tl], [f0], [fl]))
        o = out.cpu().numpy()
        _cs(o, golden_aug, f"aug_spec{s}", 0, rel=1e-12)
        assert int((o == 0).sum()) == int(golden_aug[f"aug_spec{s}__zeros"])
        assert torch.equal(y.cpu()[0], oaug.one_hot(1, 10))


def test_mixup_exact(cuda, golden_aug):
    from src.datasets.augment import spec_augment_mixup
    pool_t = [torch.from_numpy(x) for x in aug_mix_pool()]
    pool = torch.cat(pool_t).to(cuda)
    pool_labels = torch.tensor(AUG_MIX_LABELS, device=cuda)
    mixed = 0
    for s in range(12):
        i = s % len(pool_t)
        torch.manual_seed(3000 + s)
        _, _, q, lam = oaug.apply_mixup(pool_t[i], AUG_MIX_LABELS[i], pool_t, list(AUG_MIX_LABELS), 10, 0.5,
                                        random.Random(3000 + s))
        out, y = spec_augment_mixup(pool[i:i + 1], pool_labels[i:i + 1], 10, specaug=False, pool=pool,
                                    pool_labels=pool_labels, partner=torch.tensor([q]),
                                    lam=torch.tensor([lam if lam is not None else 1.0]))
        _cs(out.cpu().numpy(), golden_aug, f"aug_mix{s}", 0, rel=1e-12)
        np.testing.assert_array_equal(y.cpu().numpy()[0], golden_aug[f"aug_mix{s}__y"])
        mixed += q >= 0
    assert mixed >= 3  # includes a same-class pair (label overwrite to 1 - lam)


def test_specaug_mixup_default_draws(cuda):
    from src.datasets.augment import spec_augment_mixup
    g = torch.Generator(device=cuda).manual_seed(9)
    B = 512
    spec = torch.rand(B, 128, 1379, generator=g, device=cuda) + 1.0  # strictly positive
    labels = torch.randint(0, 50, (B,), generator=g, device=cuda)
    out, y = spec_augment_mixup(spec, labels, 50, gen=g)
    zf = (out == 0).float()
    tmask = zf.amin(dim=1).sum(1)   # fully zero frames
    fmask = zf.amin(dim=2).sum(1)   # fully zero mel rows
    mixed = (y.gt(0).sum(1) > 1) | (y.amax(1) < 1)
    unmixed = ~mixed
    assert (tmask[unmixed] >= 1).all() and (tmask <= 344).all()       # randint(1, min(192, 1379//4))
    assert (fmask[unmixed] >= 1).all() and (fmask[unmixed] <= 32).all()  # randint(1, min(48, 128//4))
    frac = float(mixed.float().mean())
    assert 0.15 < frac < 0.35, frac                                   # 0.5 * 0.5 (esc50.py:64, :949)
    two = y.gt(0).sum(1) == 2                                           # different-class partner
    assert (y[two].sum(1) - 1).abs().max() <= 1e-6 and (y[unmixed].sum(1) == 1).all()


def test_time_stretch_gain(cuda, golden_aug):
    from src.datasets.augment import stretch_gain
    w = torch.from_numpy(aug_stretch_input())
    T = w.shape[-1]
    seen = 0
    for s in range(10):
        o_ref, fac, gain = oaug.apply_augmentation(w, AUG_STRETCH_CFG, random.Random(4000 + s))
        out = stretch_gain(w.to(cuda), factor=torch.tensor([fac or 0.0], dtype=torch.float64),
                           gain=torch.tensor([gain or 1.0])).cpu()[0]
        m = o_ref.shape[-1]
        assert m == int(golden_aug[f"aug_tsg{s}__len"])
        n = min(m, T)
        np.testing.assert_allclose(out[:n].numpy(), o_ref[0, :n].numpy(), atol=2e-7, rtol=0)
        assert bool((out[n:] == 0).all())
        idx = golden_aug[f"aug_tsg{s}__idx"]
        keep = idx < n
        np.testing.assert_allclose(out.numpy()[idx[keep]], golden_aug[f"aug_tsg{s}__vals"][keep], atol=2e-7, rtol=0)
        seen += fac is not None
    assert seen >= 3
