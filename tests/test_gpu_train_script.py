"""GPU: the drop-in under scripts/train.py (reference train.py:173-201) with the real models.

dataset=synthetic -> ESC50 DataModule API -> build_from_cfg -> LitClassifier -> lite.Trainer.fit ->
test(ckpt_path="best"), trainer.precision=bf16-mixed, 2 epochs, for EnvNetV2 (on-GPU BC mixing and
time-stretch/gain in gpu_transform) and ASTModel (on-GPU log-mel + SpecAugment + Mixup); then a
resume from the best checkpoint (+ckpt_path, callbacks.py:32-56) for one more epoch."""
import importlib.util
import math
from pathlib import Path

import pytest

from src.utils.config import compose

pytestmark = pytest.mark.gpu
PKG = Path(__file__).resolve().parents[1] / "dl-sound-classification_amd"


def _script():
    spec = importlib.util.spec_from_file_location("train_script", PKG / "scripts" / "train.py")
    ts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ts)
    return ts


@pytest.mark.parametrize("model", ["envnet_v2", "ast"])
def test_train_script_fit_test_resume(cuda, tmp_path, monkeypatch, model):
    import torch
    ts = _script()
    monkeypatch.chdir(tmp_path)
    over = ["dataset=synthetic", "dataset.num_clips=40", f"model={model}", "trainer.precision=bf16-mixed",
            "batch_size=8", "num_workers=0", f"checkpoint.dirpath={tmp_path}/ck", "checkpoint.monitor=val/loss",
            "checkpoint.mode=min"]

    def cfg_for(epochs, extra=()):
        cfg = compose(PKG / "configs", "training", over + [f"trainer.max_epochs={epochs}", *extra])
        if model == "envnet_v2":  # exercise the on-GPU time stretch + gain (preprocessing.py:886-925)
            cfg.model.dataset_overrides.preprocessing_config.augment = {"time_stretch": [0.8, 1.25],
                                                                        "gain_shift": [-6, 6]}
        return cfg

    out = ts.train(cfg_for(2))
    assert {"test/acc", "test/f1", "test/auroc", "test/loss"} <= set(out)
    assert all(math.isfinite(v) for v in out.values()), out
    ck = sorted((tmp_path / "ck").glob("*.ckpt"))
    assert len(ck) == 1
    saved = torch.load(ck[0], map_location="cpu", weights_only=True)
    assert saved["lr_schedulers"] and saved["optimizer_states"]
    out2 = ts.train(cfg_for(3, [f"+ckpt_path={ck[0]}"]))
    assert all(math.isfinite(v) for v in out2.values()), out2


def _us8k_tree(root):
    """Ten folds of .pt bundles, 10 classes, 4 s clips (the reference has no UrbanSound8K loader --
    download_data.py:84-87 only -- so the file layout is the ESC-50 one)."""
    import torch
    for f in range(10):
        d = root / "us8k" / f"fold_{f}"
        d.mkdir(parents=True)
        for i in range(12):  # >= 10 clips per class: the stratified val split needs one per class
            g = torch.Generator().manual_seed(100 * f + i)
            w = 0.1 * torch.randn(1, 176_400, generator=g)
            torch.save({"waveform": w / w.abs().max(), "label": (f + i) % 10}, d / f"{i}.pt")


def test_train_script_urbansound8k_envnet_bf16(cuda, tmp_path, monkeypatch):
    """BASELINE config 4's workload on the GPU: EnvNetV2 through scripts/train.py with
    dataset=urbansound8k (ten folds of .pt bundles, 10 classes, 4 s clips zero-padded into the 5 s
    window by the pad + crop, BC mixing on the device), bf16, fit + test("best")."""
    import torch
    _us8k_tree(tmp_path)
    ts = _script()
    monkeypatch.chdir(tmp_path)
    cfg = compose(PKG / "configs", "training", [
        "dataset=urbansound8k", f"dataset.root={tmp_path}/us8k", "dataset.fold=9", "model=envnet_v2",
        "trainer.precision=bf16-mixed", "trainer.max_epochs=1", "batch_size=8", "num_workers=0",
        f"checkpoint.dirpath={tmp_path}/ck", "checkpoint.monitor=val/loss", "checkpoint.mode=min"])
    out = ts.train(cfg)
    assert {"test/acc", "test/f1", "test/auroc", "test/loss"} <= set(out)
    assert all(math.isfinite(v) for v in out.values()), out
    ck = sorted((tmp_path / "ck").glob("*.ckpt"))
    saved = torch.load(ck[0], map_location="cpu", weights_only=True)
    assert saved["state_dict"]["model.classifier.7.weight"].shape == (10, 4096)  # replace_head(10)


def test_train_script_config5_ast_fp8_urbansound8k(cuda, tmp_path, monkeypatch):
    """BASELINE config 5's workload through the drop-in (reference train.py:188-201): model=ast with
    trainer.precision=fp8-mixed (the block linears' forward GEMMs on MX-fp8 operands) on
    dataset=urbansound8k, Mixup + SpecAugment on the device (configs/model/ast.yaml), fit ->
    test("best") -> resume from the best checkpoint for one more epoch."""
    import os

    import torch
    os.environ["MIA_QUIET"] = "1"
    _us8k_tree(tmp_path)
    ts = _script()
    monkeypatch.chdir(tmp_path)
    over = ["dataset=urbansound8k", f"dataset.root={tmp_path}/us8k", "dataset.fold=3", "model=ast",
            "trainer.precision=fp8-mixed", "batch_size=8", "num_workers=0", f"checkpoint.dirpath={tmp_path}/ck",
            "checkpoint.monitor=val/loss", "checkpoint.mode=min"]
    cfg = compose(PKG / "configs", "training", over + ["trainer.max_epochs=1"])
    assert cfg.model.dataset_overrides.enable_mixup and cfg.model.dataset_overrides.augment.time_mask > 0
    out = ts.train(cfg)
    assert {"test/acc", "test/f1", "test/auroc", "test/loss"} <= set(out)
    assert all(math.isfinite(v) for v in out.values()), out
    ck = sorted((tmp_path / "ck").glob("*.ckpt"))
    assert len(ck) == 1
    saved = torch.load(ck[0], map_location="cpu", weights_only=True)
    assert saved["state_dict"]["model.head.weight"].shape == (10, 768)
    assert saved["optimizer_states"]
    out2 = ts.train(compose(PKG / "configs", "training", over + ["trainer.max_epochs=2", f"+ckpt_path={ck[0]}"]))
    assert all(math.isfinite(v) for v in out2.values()), out2
