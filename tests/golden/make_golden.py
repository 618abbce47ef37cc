#!/usr/bin/env python
"""Generate the golden parity fixtures by running the REFERENCE's own Python here.

Run in this container only (the reference is not present on the GPU box):
    python tests/golden/make_golden.py        # golden.npz
    python tests/golden/make_golden.py aug    # golden_aug.npz (augmentations + pad/crop)
    python tests/golden/make_golden.py split  # golden_split.npz (DataModule split + multi-crop)

What runs from /root/reference (imported as-is, never copied):
  * src/models/envnet_v2.py::EnvNetV2                    (needs only torch)
  * src/datasets/preprocessing.py::ASTPreprocessor.preprocess, BCMixingUtils
        through tests/golden/_stubs/torchaudio (restates torchaudio 2.7.1)
  * src/models/ast.py::ASTModel through tests/golden/_stubs/timm (restates timm 1.0.16,
        synthetic weights because the pretrained DeiT checkpoint needs the network)
  * src/datasets/preprocessing.py::BCMixingDataset, ASTPreprocessor.apply_specaugment,
        EnvNetPreprocessor.apply_augmentation, and src/datasets/esc50.py::MixupDataset /
        ESC50Dataset (through a small lightning stub), with Python's `random` seeded per case
  * src/datasets/esc50.py::ESC50DataModule.setup (the fold / stratified validation split) and
        EnvNetPreprocessor.multi_crop_test
Inputs/weights come from oracle/synth.py (splitmix64 counters) so the GPU tests can
regenerate them bit-identically; only outputs and checksums are committed.
The script also cross-checks oracle/ against these outputs and prints the errors.
"""
from __future__ import annotations

import os
import random
import sys
import time
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path(os.environ.get("REFERENCE_DIR", "/root/reference"))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(HERE / "_stubs"))
sys.path.insert(1, str(REF))
sys.dont_write_bytecode = True

from oracle import ast as oast  # noqa: E402
from oracle import envnet as oenv  # noqa: E402
from oracle import logmel as olog  # noqa: E402
from oracle.synth import hash_labels, hash_uniform, synth_waveform  # noqa: E402

torch.set_num_threads(os.cpu_count() or 8)
SAMPLE_IDX_SEED = 555


def sample_idx(n, k, seed=SAMPLE_IDX_SEED):
    return (hash_uniform(seed, (k,), 0.0, 1.0) * n).astype(np.int64).clip(0, n - 1)


def checksum(a: np.ndarray, k: int = 64, seed: int = SAMPLE_IDX_SEED):
    a = np.asarray(a, dtype=np.float64).ravel()
    idx = sample_idx(a.size, k, seed)
    return {"sum": a.sum(), "sumsq": (a * a).sum(), "idx": idx, "vals": a[idx]}


def pack(prefix, cs, out):
    for k, v in cs.items():
        out[f"{prefix}__{k}"] = np.asarray(v)


# --------------------------------------------------------------------------- logmel
def golden_logmel(out):
    from src.datasets.preprocessing import ASTPreprocessor, PreprocessingConfig
    cfg = PreprocessingConfig(sample_rate=44100, n_mels=128, normalize=True,
                              target_mean=0.0, target_std=0.5)
    pre = ASTPreprocessor(cfg)
    short = synth_waveform(11, 2, 16_000)
    ys = np.stack([pre.preprocess(torch.from_numpy(short[i:i + 1]), 44100)[0].numpy()
                   for i in range(2)])
    out["logmel_short"] = ys.astype(np.float32)                      # (2,128,101)
    full = synth_waveform(12, 2, 220_500)
    yf = np.stack([pre.preprocess(torch.from_numpy(full[i:i + 1]), 44100)[0].numpy()
                   for i in range(2)])                                # (2,128,1379)
    for b in range(2):
        pack(f"logmel_full{b}", checksum(yf[b], 2048), out)
        out[f"logmel_full{b}__rowmean"] = yf[b].mean(axis=1)
        out[f"logmel_full{b}__colmean"] = yf[b].mean(axis=0)
    # raw (unnormalised) dB path too
    cfg2 = PreprocessingConfig(sample_rate=44100, n_mels=128, normalize=False)
    y2 = ASTPreprocessor(cfg2).preprocess(torch.from_numpy(short[:1]), 44100)[0].numpy()
    out["logmel_short_db"] = y2.astype(np.float32)
    # oracle cross-check
    e1 = np.abs(olog.logmel(short).numpy() - ys).max()
    e2 = np.abs(olog.logmel(full).numpy() - yf).max()
    e3 = np.abs(olog.logmel(short[:1], normalize=False).numpy()[0] - y2).max()
    print(f"[logmel] oracle vs reference max|err| short={e1:.3g} full={e2:.3g} db={e3:.3g}")
    assert e1 < 1e-4 and e2 < 1e-4 and e3 < 1e-3


# --------------------------------------------------------------------------- envnet
def golden_envnet(out):
    from src.models.envnet_v2 import EnvNetV2
    params = oenv.hash_params(100)
    x = synth_waveform(21, 2, 220_500)[:, None, :]
    labels = hash_labels(22, 2, 50)
    r = np.array([0.3, 0.8], np.float32)
    y = np.zeros((2, 50), np.float32)
    y[0, labels[0]] = 1.0                       # one-hot row
    y[1, labels[1]] = r[1]                      # BC-mix style soft row
    y[1, (labels[1] + 7) % 50] = 1 - r[1]
    out["envnet_x_seed"] = np.array(21)
    out["envnet_y"] = y

    def build(dropout):
        m = EnvNetV2(num_classes=50, dropout=dropout)
        sd = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not unexpected and all(k.endswith("num_batches_tracked") for k in missing), (missing, unexpected)
        return m

    xt = torch.from_numpy(x)
    m = build(0.5).eval()
    with torch.no_grad():
        z_eval = m(xt).numpy()
    out["envnet_logits_eval"] = z_eval
    m = build(0.0).train()
    z_train = m(xt)
    loss = -torch.sum(torch.from_numpy(y) * torch.log(torch.softmax(z_train, 1) + 1e-8), 1).mean()
    loss.backward()
    out["envnet_logits_train"] = z_train.detach().numpy()
    out["envnet_loss"] = np.array(loss.item())
    for name, t in m.state_dict().items():
        if name.endswith("running_mean") or name.endswith("running_var"):
            out[f"envnet_after__{name}"] = t.numpy().copy()
    names = [n for n, _ in m.named_parameters()]
    for n, p in m.named_parameters():
        pack(f"envnet_grad__{n}", checksum(p.grad.numpy(), 64), out)
    total = torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    out["envnet_gradnorm"] = np.array(float(total))
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, weight_decay=1e-4)
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    opt.step()
    for n, p in m.named_parameters():
        pack(f"envnet_delta__{n}", checksum((p.detach() - before[n]).numpy(), 64), out)
    out["envnet_param_names"] = np.array(names)
    # margins for argmax well-definedness
    for tag, z in (("eval", z_eval), ("train", out["envnet_logits_train"])):
        s = np.sort(z, axis=1)
        print(f"[envnet] {tag} top2 margin rel:", (s[:, -1] - s[:, -2]) / np.abs(s[:, -1]))
    # oracle cross-check
    tp = oenv.to_torch(params)
    with torch.no_grad():
        ze = oenv.forward(tp, xt, training=False).numpy()
        zt = oenv.forward(oenv.to_torch(params), xt, training=True, dropout_p=0.0).numpy()
    print(f"[envnet] oracle vs reference eval={np.abs(ze - z_eval).max():.3g} "
          f"train={np.abs(zt - out['envnet_logits_train']).max():.3g} (|z|max {np.abs(z_eval).max():.3g})")


# --------------------------------------------------------------------------- ast
def golden_ast(out):
    import timm
    timm.STATE_HOOK = lambda: oast.deit_hash_state(300)
    from src.models.ast import ASTModel
    m = ASTModel(num_classes=50)
    hw, hb = oast.head_hash(900, 50)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    m.eval()
    x = hash_uniform(31, (2, 128, 1379))
    t0 = time.time()
    with torch.no_grad():
        probs = m(torch.from_numpy(x)).numpy()
    print(f"[ast] reference forward {time.time() - t0:.1f}s")
    out["ast_probs"] = probs
    out["ast_pos_embed_cs"] = np.asarray([m.pos_embed.detach().double().sum().item(),
                                          m.pos_embed.detach().double().pow(2).sum().item()])
    out["ast_nparams"] = np.array(sum(p.numel() for p in m.parameters()))
    p = oast.model_params(oast.deit_hash_state(300), hw, hb)
    with torch.no_grad():
        po = oast.forward(p, torch.from_numpy(x)).numpy()
    s = np.sort(probs, axis=1)
    print("[ast] top2 margin:", s[:, -1] - s[:, -2])
    print(f"[ast] oracle vs reference max|err|={np.abs(po - probs).max():.3g}; "
          f"nparams={int(out['ast_nparams'])}")


# --------------------------------------------------------------------------- BC mixing
def golden_bcmix(out):
    from src.datasets.preprocessing import BCMixingUtils
    u = BCMixingUtils()
    w1 = synth_waveform(41, 1, 220_500)
    w2 = synth_waveform(42, 1, 220_500) * np.float32(0.05)   # ~-26 dB -> perceptual branch
    rs = np.array([0.1, 0.37, 0.5, 0.93], np.float32)
    ps, mixes = [], []
    for r in rs:
        for a, b in ((w1, w2), (w2, w1), (w1, w1 * np.float32(0.9))):
            s1 = u.a_weighted_spl(torch.from_numpy(a))
            s2 = u.a_weighted_spl(torch.from_numpy(b))
            p = u.perceptual_mixing_coefficient(float(r), s1, s2)
            mix = u.mix_waveforms(torch.from_numpy(a), torch.from_numpy(b), p).numpy()
            ps.append([s1, s2, p])
            mixes.append([mix.sum(), (mix.astype(np.float64) ** 2).sum(), mix[0, 1234], mix[0, 99999]])
    out["bcmix_r"] = rs
    out["bcmix_spl_p"] = np.array(ps, np.float64)
    out["bcmix_mix_cs"] = np.array(mixes, np.float64)
    lab = u.create_soft_labels(0.37, 3, 17, 50).numpy()
    out["bcmix_soft_label"] = lab


# --------------------------------------------------------------------------- augmentations + batch source
def golden_aug(out):
    """BC mixing, SpecAugment, Mixup, time-stretch/gain and the EnvNet pad + crop, each run through
    the reference's own classes with Python's `random` (and torch's generator for Beta) seeded per
    case; the oracle (oracle/augment.py) replays the same draws and must reproduce every output."""
    import tempfile

    from src.datasets.esc50 import ESC50Dataset, MixupDataset
    from src.datasets.preprocessing import (ASTPreprocessor, BCMixingDataset, EnvNetPreprocessor,
                                            PreprocessingConfig)
    from oracle import augment as oaug
    from tests._aug_inputs import (AUG_BC_LABELS, AUG_MIX_LABELS, AUG_SPEC_CASES, AUG_STRETCH_CFG,
                                   aug_bc_pool, aug_crop_clip, aug_mix_pool, aug_spec_input,
                                   aug_stretch_input)
    # BC mixing through BCMixingDataset.apply_bc_mixing (preprocessing.py:564-609)
    pool = [torch.from_numpy(w) for w in aug_bc_pool()]
    data = list(zip(pool, AUG_BC_LABELS))
    bc = BCMixingDataset(enable_bc_mixing=True, num_classes=4)
    for s in range(8):
        i = s % len(pool)
        random.seed(1000 + s)
        mixed, y = bc.apply_bc_mixing(pool[i], AUG_BC_LABELS[i], data)
        pack(f"aug_bc{s}", checksum(mixed.numpy(), 64), out)
        out[f"aug_bc{s}__y"] = y.numpy()
        m2, y2, q, r, p = oaug.apply_bc_mixing(pool[i], AUG_BC_LABELS[i], pool, list(AUG_BC_LABELS), 4,
                                               random.Random(1000 + s))
        print(f"[aug] bc{s}: partner {q} r {r:.4f} p {p:.4f} oracle err {np.abs(m2.numpy() - mixed.numpy()).max():.3g}")
        assert torch.equal(y, y2)
    random.seed(1099)
    mixed, y = bc.apply_bc_mixing(pool[0], 0, [(pool[1], 0), (pool[0], 0)])  # no other class: unchanged, one-hot
    out["aug_bc_sameclass__y"] = y.numpy()
    out["aug_bc_sameclass__equal"] = np.array(torch.equal(mixed, pool[0]))
    # SpecAugment (preprocessing.py:1075-1104)
    pre = ASTPreprocessor(PreprocessingConfig(sample_rate=44100, n_mels=128))
    for s, (shape, tm, fm) in enumerate(AUG_SPEC_CASES):
        spec = torch.from_numpy(aug_spec_input(s))
        random.seed(2000 + s)
        o = pre.apply_specaugment(spec, time_mask=tm, freq_mask=fm).numpy()
        pack(f"aug_spec{s}", checksum(o, 64), out)
        out[f"aug_spec{s}__zeros"] = np.array((o == 0).sum())
        o2, prm = oaug.specaugment(spec, tm, fm, random.Random(2000 + s))
        print(f"[aug] spec{s}: {prm} oracle equal {np.array_equal(o2.numpy(), o)}")
        assert np.array_equal(o2.numpy(), o)
    # Mixup: MixupDataset.apply_mixup (esc50.py:52-76) -> MixupAugmentation (preprocessing.py:935-968)
    mpool = [torch.from_numpy(x) for x in aug_mix_pool()]
    mdata = list(zip(mpool, AUG_MIX_LABELS))
    md = MixupDataset(enable_mixup=True, mixup_alpha=0.5, num_classes=10)
    for s in range(12):
        i = s % len(mpool)
        random.seed(3000 + s)
        torch.manual_seed(3000 + s)
        o, y = md.apply_mixup(mpool[i], AUG_MIX_LABELS[i], mdata)
        pack(f"aug_mix{s}", checksum(o.numpy(), 64), out)
        out[f"aug_mix{s}__y"] = y.numpy()
        torch.manual_seed(3000 + s)
        o2, y2, q, lam = oaug.apply_mixup(mpool[i], AUG_MIX_LABELS[i], mpool, list(AUG_MIX_LABELS), 10, 0.5,
                                          random.Random(3000 + s))
        print(f"[aug] mix{s}: partner {q} lam {lam} oracle equal {torch.equal(o, o2) and torch.equal(y, y2)}")
        assert torch.equal(o, o2) and torch.equal(y, y2)
    # time stretch + gain (EnvNetPreprocessor.apply_augmentation, preprocessing.py:886-925)
    ep = EnvNetPreprocessor(PreprocessingConfig(sample_rate=44100, window_length=0.5, augment=AUG_STRETCH_CFG))
    w = torch.from_numpy(aug_stretch_input())
    for s in range(10):
        random.seed(4000 + s)
        o = ep.apply_augmentation(w).numpy()
        out[f"aug_tsg{s}__len"] = np.array(o.shape[-1])
        pack(f"aug_tsg{s}", checksum(o, 64), out)
        o2, fac, gain = oaug.apply_augmentation(w, AUG_STRETCH_CFG, random.Random(4000 + s))
        print(f"[aug] tsg{s}: factor {fac} gain {gain} len {o.shape[-1]} oracle err "
              f"{np.abs(o2.numpy() - o).max() if o2.shape == o.shape else 'shape'}")
        assert o2.shape == o.shape and np.abs(o2.numpy() - o).max() == 0
    # ESC50Dataset pad + crop (esc50.py:198-249, preprocessing.py:814-855), envnet_v2 mode, no BC mixing
    with tempfile.TemporaryDirectory() as td:
        root = Path(td) / "esc50"
        (root / "fold_0").mkdir(parents=True)
        files = []
        for i in range(3):
            f = root / "fold_0" / f"clip{i}.pt"
            torch.save({"waveform": torch.from_numpy(aug_crop_clip(i)), "label": i}, f)
            files.append(f)
        pc = {"window_length": 0.5, "padding_ratio": 0.5}
        for training in (True, False):
            ds = ESC50Dataset(root=root, files=files, preprocessing_mode="envnet_v2", preprocessing_config=pc,
                              enable_bc_mixing=False, num_classes=3, training=training)
            for s in range(6 if training else 3):
                random.seed(5000 + s)
                x, y = ds[s % 3]
                tag = f"aug_crop{'T' if training else 'E'}{s}"
                pack(tag, checksum(x.numpy(), 64), out)
                out[f"{tag}__shape"] = np.array(x.shape)
                out[f"{tag}__y"] = y.numpy()


# --------------------------------------------------------------------------- data split + multi-crop
def golden_split(out):
    """The reference's own ESC50DataModule.setup (esc50.py:501-592: four train folds, stratified
    validation split with StratifiedShuffleSplit(random_state=42), held-out test fold) on a synthetic
    five-fold layout, and EnvNetPreprocessor.multi_crop_test (preprocessing.py:857-884) on padded
    clips; the file lists are recorded as fold_k/name strings, the crops as checksums."""
    import tempfile

    from src.datasets.esc50 import ESC50DataModule
    from src.datasets.preprocessing import EnvNetPreprocessor, PreprocessingConfig
    from tests.golden._layout import (MCROP_CASES, SPLIT_CLASSES, SPLIT_FOLD_CLIPS, SPLIT_TEST_FOLD, mcrop_clip,
                                      split_label)
    with tempfile.TemporaryDirectory() as td:
        root = Path(td) / "esc50"
        for f in range(5):
            (root / f"fold_{f}").mkdir(parents=True)
            for i in range(SPLIT_FOLD_CLIPS):
                torch.save({"waveform": torch.zeros(1, 64), "label": split_label(f, i)},
                           root / f"fold_{f}" / f"c{i:03d}.pt")
        dm = ESC50DataModule(root=str(root), fold=SPLIT_TEST_FOLD, val_split=0.1, batch_size=4, num_workers=0,
                             num_classes=SPLIT_CLASSES, preprocessing_config={"window_length": 0.001})
        dm.setup("fit")

        def names(ds):
            return np.array([f"{Path(f).parent.name}/{Path(f).name}" for f in ds.files])

        out["split_train"] = names(dm._train_set)
        out["split_val"] = names(dm._val_set)
        out["split_test"] = names(dm._test_set)
        print(f"[split] train {len(out['split_train'])} val {len(out['split_val'])} test {len(out['split_test'])}")
    # multi-crop: crops of the T/2-padded clip at linspace(0, max_start, test_crops) starts
    for s, (win, n, crops) in enumerate(MCROP_CASES):
        pre = EnvNetPreprocessor(PreprocessingConfig(sample_rate=44100, window_length=win, test_crops=crops,
                                                     multi_crop_test=True))
        w = torch.from_numpy(mcrop_clip(s))
        cs = pre.multi_crop_test(pre.preprocess(w, 44100))
        out[f"mcrop{s}__n"] = np.array(len(cs))
        for k, c in enumerate(cs):
            pack(f"mcrop{s}_{k}", checksum(c.numpy(), 32), out)
            out[f"mcrop{s}_{k}__shape"] = np.array(c.shape)


def main():
    only = sys.argv[1:]
    if only == ["split"]:
        out = {}
        golden_split(out)
        dst = HERE / "golden_split.npz"
        np.savez_compressed(dst, **out)
        print(f"wrote {dst} ({dst.stat().st_size / 1e6:.2f} MB, {len(out)} arrays)")
        return
    if only == ["aug"]:
        out = {}
        golden_aug(out)
        dst = HERE / "golden_aug.npz"
        np.savez_compressed(dst, **out)
        print(f"wrote {dst} ({dst.stat().st_size / 1e6:.2f} MB, {len(out)} arrays)")
        return
    random.seed(0)
    out = {}
    golden_logmel(out)
    golden_bcmix(out)
    golden_envnet(out)
    golden_ast(out)
    dst = HERE / "golden.npz"
    np.savez_compressed(dst, **out)
    print(f"wrote {dst} ({dst.stat().st_size / 1e6:.2f} MB, {len(out)} arrays)")


if __name__ == "__main__":
    main()
