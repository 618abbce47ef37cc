"""LightningModule wrapper — drop-in for the reference ``src.training.engine`` (LitClassifier,
build_from_cfg; reference src/training/engine.py:32-325).

Same constructor (model_cfg, optim_cfg, sched_cfg, loss_cfg, metric_cfg), same ``_step`` semantics:
soft labels (B, C) f32 -> ``-(y * log(softmax(z) + 1e-8)).sum(1).mean()`` (engine.py:175-176; the
configured CrossEntropyLoss is bypassed for one-hot / mixed labels exactly as in the reference),
KL branch when the loss class name contains "KL", hard labels -> the configured criterion (multi-crop
test), accuracy on ``argmax(y)``.  Differences, all MI355X-motivated:
  * the soft-label loss and its gradient run in one fused kernel (mia_soft_ce);
  * the batch's feature transform / augmentation (BC mixing for EnvNet; log-mel + SpecAugment +
    Mixup for AST) runs on the GPU inside the step (``datamodule.gpu_transform``) instead of in CPU
    DataLoader workers;
  * ``configure_optimizers`` maps torch.optim.Adam to the fused clip+Adam kernel (FusedAdam) when the
    parameters live on the GPU (the clip value comes from ``trainer.gradient_clip_val``).
Lightning is not installed in this image; ``src.training.lite`` provides the LightningModule/Trainer
surface this class uses (log, current_epoch, hparams, fit/test loop, DDP over RCCL).
"""
from __future__ import annotations

from typing import Any

import torch
import torch.nn as nn

from ..utils.config import instantiate
from . import metrics as M
from .lite import LightningModule


def _adapt_head_if_possible(model: nn.Module, num_classes: int) -> None:
    """Resize the classification head when the backbone exposes one (engine.py:32-46)."""
    if hasattr(model, "replace_head") and callable(model.replace_head):
        model.replace_head(num_classes)
    elif hasattr(model, "classifier") and isinstance(model.classifier, nn.Linear):
        model.classifier = nn.Linear(model.classifier.in_features, num_classes)
    elif hasattr(model, "fc") and isinstance(model.fc, nn.Linear):
        model.fc = nn.Linear(model.fc.in_features, num_classes)


class LitClassifier(LightningModule):
    def __init__(self, model_cfg, optim_cfg, sched_cfg=None, loss_cfg=None, metric_cfg=None) -> None:
        super().__init__()
        self.model: nn.Module = instantiate(model_cfg)
        if "num_classes" in model_cfg and isinstance(model_cfg["num_classes"], (int, float)):
            _adapt_head_if_possible(self.model, int(model_cfg["num_classes"]))
        self.num_classes = int(model_cfg.get("num_classes", 50) or 50)
        self.criterion: nn.Module = instantiate(loss_cfg) if loss_cfg is not None else nn.CrossEntropyLoss()
        self._is_kl_loss = "KL" in self.criterion.__class__.__name__
        C = self.num_classes
        self.train_acc, self.val_acc, self.test_acc = M.Accuracy(C), M.Accuracy(C), M.Accuracy(C)
        self.test_f1, self.test_auroc = M.F1Macro(C), M.AUROC(C)
        self.test_confmat, self.test_class_acc = M.ConfusionMatrix(C), M.ClassAccuracy(C)
        self.train_acc_history, self.val_acc_history, self.epoch_history = [], [], []
        self._optim_cfg, self._sched_cfg = optim_cfg, sched_cfg
        self.save_hyperparameters({"optim": dict(optim_cfg) if optim_cfg is not None else None,
                                   "sched": dict(sched_cfg) if sched_cfg is not None else None,
                                   "loss": str(self.criterion)})

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.model(x)

    def _soft_loss(self, logits, y):
        if logits.is_cuda and not self._is_kl_loss and not torch.is_grad_enabled():
            from ..miaudio import kernels as K
            loss, _, _ = K.soft_ce(logits.detach().float().contiguous(), y.float().contiguous(), input_sigmoid=False)
            return loss
        if logits.is_cuda and not self._is_kl_loss:
            return _FusedSoftCE.apply(logits, y)
        if self._is_kl_loss:
            return self.criterion(torch.log_softmax(logits, dim=1), y)
        probs = torch.softmax(logits, dim=1)
        return -torch.sum(y * torch.log(probs + 1e-8), dim=1).mean()

    def _step(self, batch: Any, stage: str) -> torch.Tensor:
        x, y = (batch["inputs"], batch["labels"]) if isinstance(batch, dict) else batch
        dm = getattr(self, "datamodule", None)
        if dm is not None and hasattr(dm, "gpu_transform") and not isinstance(x, (list, tuple)):
            x, y = dm.gpu_transform(x, y, training=(stage == "train"))
        if isinstance(x, (list, tuple)) and stage == "test":
            logits = torch.stack([self(xi) for xi in x], dim=0).mean(dim=0)
        else:
            logits = self(x)
        if y.dtype == torch.float32 and y.dim() > 1:
            loss = self._soft_loss(logits, y)
            hard = torch.argmax(y, dim=1)
        else:
            loss = self.criterion(logits, y)
            hard = y
        self.log(f"{stage}/loss", loss, prog_bar=True, on_step=False, on_epoch=True)
        if stage == "train":
            self.train_acc.update(logits, hard)
        elif stage == "val":
            self.val_acc.update(logits, hard)
        else:
            for m in (self.test_acc, self.test_f1, self.test_auroc, self.test_confmat, self.test_class_acc):
                m.update(logits, hard)
        return loss

    def training_step(self, batch, batch_idx):
        return self._step(batch, "train")

    def validation_step(self, batch, batch_idx):
        self._step(batch, "val")

    def test_step(self, batch, batch_idx):
        self._step(batch, "test")

    def on_train_epoch_end(self) -> None:
        acc = self.train_acc.compute()
        self.log("train/acc", acc, prog_bar=True)
        self.train_acc.reset()
        self.train_acc_history.append(float(acc))
        self.epoch_history.append(self.current_epoch)

    def on_validation_epoch_end(self) -> None:
        acc = self.val_acc.compute()
        self.log("val/acc", acc, prog_bar=True)
        self.val_acc.reset()
        self.val_acc_history.append(float(acc))

    def on_test_epoch_end(self) -> None:
        self.log("test/acc", self.test_acc.compute(), prog_bar=True)
        self.log("test/f1", self.test_f1.compute(), prog_bar=True)
        self.log("test/auroc", self.test_auroc.compute(), prog_bar=True)
        self.test_confmat_result = self.test_confmat.compute()
        self.test_class_acc_result = self.test_class_acc.compute()
        if self.logger is not None and hasattr(self.logger, "save_tensor"):
            self.logger.save_tensor("test_confmat.pt", self.test_confmat_result)
            self.logger.save_tensor("test_class_acc.pt", self.test_class_acc_result)
        for m in (self.test_acc, self.test_f1, self.test_auroc, self.test_confmat, self.test_class_acc):
            m.reset()

    def configure_optimizers(self):
        params = list(self.parameters())
        target = str(self._optim_cfg.get("_target_", "")) if self._optim_cfg is not None else ""
        optim = None
        if params and params[0].is_cuda and target in ("torch.optim.Adam", "src.training.optim.FusedAdam"):
            from .optim import FusedAdam
            kw = {k: v for k, v in self._optim_cfg.items() if k != "_target_"}
            clip = getattr(getattr(self, "trainer", None), "gradient_clip_val", 0.0) or 0.0
            try:
                optim = FusedAdam(params, clip=clip, **kw)
                optim.handles_clipping = True
            except ValueError as e:  # an Adam option the fused kernel does not implement
                if target != "torch.optim.Adam":
                    raise
                print(f"[engine] {e}; running torch.optim.Adam", flush=True)
        if optim is None:
            optim = instantiate(self._optim_cfg, params=params)
        if self._sched_cfg is None:
            return optim
        sched = instantiate(self._sched_cfg, optimizer=optim)
        return {"optimizer": optim, "lr_scheduler": sched if isinstance(sched, dict) else {"scheduler": sched}}


class _FusedSoftCE(torch.autograd.Function):
    """Soft-label loss of engine.py:175-176 with its gradient from one fused kernel."""

    @staticmethod
    def forward(ctx, logits, y):
        from ..miaudio import kernels as K
        loss, dlogits, _ = K.soft_ce(logits.detach().float().contiguous(), y.float().contiguous(),
                                     input_sigmoid=False)
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dlogits,) = ctx.saved_tensors
        return dlogits * g, None


def build_from_cfg(cfg) -> LitClassifier:
    return LitClassifier(model_cfg=cfg.model, optim_cfg=cfg.optimizer, sched_cfg=cfg.get("scheduler"),
                         loss_cfg=cfg.get("loss"), metric_cfg=cfg.get("metric"))
