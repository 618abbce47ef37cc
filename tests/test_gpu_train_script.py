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
