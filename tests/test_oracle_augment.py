"""CPU: the augmentation restatement (oracle/augment.py) reproduces the reference's own outputs
(tests/golden/golden.npz bcmix_* and golden_aug.npz, written by tests/golden/make_golden.py running
BCMixingUtils / BCMixingDataset / ASTPreprocessor.apply_specaugment / MixupDataset /
EnvNetPreprocessor.apply_augmentation / ESC50Dataset with Python's `random` seeded per case), and
the product ESC50Dataset's pad + crop (CPU host code) draws the same crops as the reference."""
import random
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import augment as oaug
from oracle.synth import synth_waveform
from tests._aug_inputs import (AUG_BC_LABELS, AUG_MIX_LABELS, AUG_SPEC_CASES, AUG_STRETCH_CFG, aug_bc_pool,
                               aug_crop_clip, aug_mix_pool, aug_spec_input, aug_stretch_input)


def _check(a, g, prefix, atol):
    a = np.asarray(a, np.float64).ravel()
    np.testing.assert_allclose(a[g[f"{prefix}__idx"]], g[f"{prefix}__vals"], atol=atol, rtol=0)
    np.testing.assert_allclose(a.sum(), g[f"{prefix}__sum"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose((a * a).sum(), g[f"{prefix}__sumsq"], rtol=1e-5)


def test_bcmix_utils_match_reference(golden):
    w1 = torch.from_numpy(synth_waveform(41, 1, 220_500))
    w2 = torch.from_numpy(synth_waveform(42, 1, 220_500) * np.float32(0.05))
    k = 0
    for r in golden["bcmix_r"]:
        for a, b in ((w1, w2), (w2, w1), (w1, w1 * np.float32(0.9))):
            s1, s2 = oaug.a_weighted_spl(a), oaug.a_weighted_spl(b)
            p = oaug.perceptual_mixing_coefficient(float(r), s1, s2)
            assert [s1, s2, p] == list(golden["bcmix_spl_p"][k])
            mix = oaug.mix_waveforms(a, b, p).numpy().astype(np.float64)
            cs = golden["bcmix_mix_cs"][k]
            assert mix.sum() == pytest.approx(cs[0], rel=1e-6) and (mix ** 2).sum() == pytest.approx(cs[1], rel=1e-6)
            assert mix[0, 1234] == cs[2] and mix[0, 99999] == cs[3]
            k += 1
    assert torch.equal(oaug.soft_labels(0.37, 3, 17, 50), torch.from_numpy(golden["bcmix_soft_label"]))


def test_bc_mixing_dataset_draws(golden_aug):
    pool = [torch.from_numpy(w) for w in aug_bc_pool()]
    for s in range(8):
        i = s % len(pool)
        m, y, q, r, p = oaug.apply_bc_mixing(pool[i], AUG_BC_LABELS[i], pool, list(AUG_BC_LABELS), 4,
                                             random.Random(1000 + s))
        assert AUG_BC_LABELS[q] != AUG_BC_LABELS[i]
        _check(m.numpy(), golden_aug, f"aug_bc{s}", 0)
        assert np.array_equal(y.numpy(), golden_aug[f"aug_bc{s}__y"])
    m, y, q, _, _ = oaug.apply_bc_mixing(pool[0], 0, [pool[1], pool[0]], [0, 0], 4, random.Random(1099))
    assert q == -1 and torch.equal(m, pool[0]) and bool(golden_aug["aug_bc_sameclass__equal"])
    assert np.array_equal(y.numpy(), golden_aug["aug_bc_sameclass__y"])


def test_partner_mapping_is_random_choice_over_different_class():
    labels = [3, 1, 3, 3, 2, 1, 0, 3]
    diff = [i for i, l in enumerate(labels) if l != 3]
    got = [oaug.partner_from_uniform(k / len(diff) + 1e-6, 3, labels) for k in range(len(diff))]
    assert got == diff
    assert oaug.partner_from_uniform(0.999999, 3, labels) == diff[-1]
    assert oaug.partner_from_uniform(0.5, 7, [7, 7]) == -1


def test_specaugment_draws(golden_aug):
    for s, (shape, tm, fm) in enumerate(AUG_SPEC_CASES):
        o, prm = oaug.specaugment(torch.from_numpy(aug_spec_input(s)), tm, fm, random.Random(2000 + s))
        assert o.shape == shape
        _check(o.numpy(), golden_aug, f"aug_spec{s}", 0)
        assert int((o == 0).sum()) == int(golden_aug[f"aug_spec{s}__zeros"])
    # n_frames <= time_mask: time mask skipped (preprocessing.py:1093)
    assert oaug.specaugment(torch.from_numpy(aug_spec_input(6)), 8, 2, random.Random(2006))[1][1] == 0


def test_mixup_draws(golden_aug):
    pool = [torch.from_numpy(x) for x in aug_mix_pool()]
    mixed = 0
    for s in range(12):
        i = s % len(pool)
        torch.manual_seed(3000 + s)
        o, y, q, lam = oaug.apply_mixup(pool[i], AUG_MIX_LABELS[i], pool, list(AUG_MIX_LABELS), 10, 0.5,
                                        random.Random(3000 + s))
        _check(o.numpy(), golden_aug, f"aug_mix{s}", 0)
        assert np.array_equal(y.numpy(), golden_aug[f"aug_mix{s}__y"])
        mixed += q >= 0
    assert mixed >= 2
    # same-class partner: the second write wins (preprocessing.py:965-966)
    _, y = oaug.mixup_apply(pool[0], pool[2], torch.tensor(0.3), 5, 5, 10)
    assert float(y[5]) == pytest.approx(0.7) and float(y.sum()) == pytest.approx(0.7)


def test_time_stretch_gain_draws(golden_aug):
    w = torch.from_numpy(aug_stretch_input())
    for s in range(10):
        o, fac, gain = oaug.apply_augmentation(w, AUG_STRETCH_CFG, random.Random(4000 + s))
        assert o.shape[-1] == int(golden_aug[f"aug_tsg{s}__len"])
        _check(o.numpy(), golden_aug, f"aug_tsg{s}", 0)


def test_product_dataset_pad_crop_matches_reference(tmp_path, golden_aug):
    """Product host code: ESC50Dataset (envnet_v2, no BC mixing) pads T/2 each side and crops with
    random.randint like the reference (preprocessing.py:814-855); seeded alike -> identical crops."""
    from src.datasets.esc50 import ESC50Dataset
    files = []
    for i in range(3):
        f = tmp_path / f"clip{i}.pt"
        torch.save({"waveform": torch.from_numpy(aug_crop_clip(i)), "label": i}, f)
        files.append(f)
    for training in (True, False):
        ds = ESC50Dataset(tmp_path, files=files, mode="envnet_v2", pad_crop=True, window_length=0.5,
                          padding_ratio=0.5, training=training)
        for s in range(6 if training else 3):
            random.seed(5000 + s)
            x, label = ds[s % 3]
            tag = f"aug_crop{'T' if training else 'E'}{s}"
            assert tuple(x.shape) == tuple(golden_aug[f"{tag}__shape"])
            _check(x.numpy(), golden_aug, tag, 0)
            assert int(np.argmax(golden_aug[f"{tag}__y"])) == label


# ------------------------------------------------------------------ data split + multi-crop (reference-pinned)
GOLDEN_SPLIT = np.load(Path(__file__).resolve().parent / "golden" / "golden_split.npz")


def test_esc50_split_matches_reference_setup(tmp_path):
    """ESC50DataModule.setup reproduces the reference's own split (tests/golden/golden_split.npz, written
    by running reference esc50.py:501-592 on the same synthetic five-fold layout): identical train /
    validation / test file lists, in the same order."""
    from src.datasets.esc50 import ESC50DataModule
    from tests.golden._layout import SPLIT_CLASSES, SPLIT_FOLD_CLIPS, SPLIT_TEST_FOLD, split_label
    root = tmp_path / "esc50"
    for f in range(5):
        (root / f"fold_{f}").mkdir(parents=True)
        for i in range(SPLIT_FOLD_CLIPS):
            torch.save({"waveform": torch.zeros(1, 64), "label": split_label(f, i)}, root / f"fold_{f}" / f"c{i:03d}.pt")
    dm = ESC50DataModule(root=str(root), fold=SPLIT_TEST_FOLD, val_split=0.1, batch_size=4, num_workers=0,
                         num_classes=SPLIT_CLASSES, preprocessing_config={"window_length": 0.001})
    dm.setup("fit")

    def names(ds):
        return [f"{Path(f).parent.name}/{Path(f).name}" for f in ds.files]

    assert names(dm._train_set) == list(GOLDEN_SPLIT["split_train"])
    assert names(dm._val_set) == list(GOLDEN_SPLIT["split_val"])
    assert names(dm._test_set) == list(GOLDEN_SPLIT["split_test"])


@pytest.mark.parametrize("s", [0, 1, 2])
def test_multi_crop_matches_reference(tmp_path, s):
    """Multi-crop test items = the reference's EnvNetPreprocessor.multi_crop_test of the T/2-padded clip
    (preprocessing.py:814-827,857-884): crop count, shapes and contents (checksums of the reference's
    crops).  The reference's dataset path (esc50.py:208-214) applies multi_crop_test BEFORE the
    padding, which turns every 5 s ESC-50 clip into one 10 s crop the model cannot take; the padded
    order pinned here is the one that yields `test_crops` window-length crops."""
    from src.datasets.esc50 import ESC50Dataset
    from tests.golden._layout import MCROP_CASES, checksum, mcrop_clip
    win, n, crops = MCROP_CASES[s]
    w = torch.from_numpy(mcrop_clip(s))
    f = tmp_path / "clip.pt"
    torch.save({"waveform": w, "label": 0}, f)
    ds = ESC50Dataset(tmp_path, files=[f], window_length=win, pad_crop=True, training=False, multi_crop_test=True,
                      test_crops=crops)
    got, _ = ds[0]
    assert len(got) == int(GOLDEN_SPLIT[f"mcrop{s}__n"])
    for k, c in enumerate(got):
        assert tuple(c.shape) == tuple(GOLDEN_SPLIT[f"mcrop{s}_{k}__shape"])
        cs = checksum(c.numpy(), 32)
        assert cs["sum"] == GOLDEN_SPLIT[f"mcrop{s}_{k}__sum"] and cs["sumsq"] == GOLDEN_SPLIT[f"mcrop{s}_{k}__sumsq"]
        assert np.array_equal(cs["vals"], GOLDEN_SPLIT[f"mcrop{s}_{k}__vals"])
