"""Epoch metrics used by LitClassifier (the torchmetrics MulticlassAccuracy / F1 / AUROC /
ConfusionMatrix / per-class accuracy of reference engine.py:104-111; torchmetrics is not installed).
States are small device tensors; ``compute()`` all-reduces them across data-parallel ranks
(torchmetrics syncs at compute the same way)."""
from __future__ import annotations

import torch
import torch.distributed as dist


def _sync(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = t.clone()
        dist.all_reduce(t)
    return t


class _Confusion:
    def __init__(self, num_classes: int):
        self.C = num_classes
        self.cm = None

    def reset(self):
        self.cm = None

    def update(self, logits: torch.Tensor, target: torch.Tensor):
        pred = logits.detach().argmax(dim=1)
        idx = target.long().view(-1) * self.C + pred.view(-1)
        cm = torch.bincount(idx, minlength=self.C * self.C).view(self.C, self.C)
        self.cm = cm if self.cm is None else self.cm + cm

    def confusion(self):
        if self.cm is None:
            return torch.zeros(self.C, self.C, dtype=torch.long)
        return _sync(self.cm)


class Accuracy(_Confusion):
    """MulticlassAccuracy with torchmetrics' default average='macro' over classes present."""

    def compute(self):
        cm = self.confusion().double()
        support = cm.sum(1)
        per = torch.where(support > 0, cm.diag() / support.clamp_min(1), torch.zeros_like(support))
        present = support > 0
        return (per[present].mean() if present.any() else per.sum() * 0).float()


class ClassAccuracy(_Confusion):
    def compute(self):
        cm = self.confusion().double()
        return (cm.diag() / cm.sum(1).clamp_min(1)).float()


class ConfusionMatrix(_Confusion):
    def compute(self):
        return self.confusion()


class F1Macro(_Confusion):
    def compute(self):
        cm = self.confusion().double()
        tp = cm.diag()
        prec = tp / cm.sum(0).clamp_min(1)
        rec = tp / cm.sum(1).clamp_min(1)
        f1 = torch.where(prec + rec > 0, 2 * prec * rec / (prec + rec), torch.zeros_like(tp))
        return f1.mean().float()


class AUROC:
    """Macro one-vs-rest AUROC from softmax scores (rank statistic), accumulated on the host."""

    def __init__(self, num_classes: int):
        self.C = num_classes
        self.reset()

    def reset(self):
        self.scores, self.targets = [], []

    def update(self, logits, target):
        self.scores.append(torch.softmax(logits.detach().float(), dim=1).cpu())
        self.targets.append(target.detach().long().cpu())

    def compute(self):
        if not self.scores:
            return torch.tensor(0.0)
        s = torch.cat(self.scores)
        t = torch.cat(self.targets)
        aucs = []
        for c in range(self.C):
            pos = t == c
            npos, nneg = int(pos.sum()), int((~pos).sum())
            if npos == 0 or nneg == 0:
                continue
            ranks = torch.empty_like(s[:, c])
            ranks[s[:, c].argsort()] = torch.arange(1, len(t) + 1, dtype=ranks.dtype)
            aucs.append((ranks[pos].sum() - npos * (npos + 1) / 2) / (npos * nneg))
        return torch.stack(aucs).mean() if aucs else torch.tensor(0.0)
