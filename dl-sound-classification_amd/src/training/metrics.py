"""Epoch metrics used by LitClassifier (the torchmetrics 1.7 MulticlassAccuracy / F1 / AUROC /
ConfusionMatrix / per-class accuracy of reference engine.py:104-111; torchmetrics is not installed).
States are small device tensors; ``compute()`` all-reduces (AUROC: all-gathers) them across
data-parallel ranks, as torchmetrics syncs at compute.  Macro averages weight a class in when
tp + fp + fn > 0 (torchmetrics ``_adjust_weights_safe_divide``): a class never present but predicted
counts with score 0, a class neither present nor predicted is left out."""
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


def _macro(score: torch.Tensor, cm: torch.Tensor) -> torch.Tensor:
    tp = cm.diag()
    w = ((cm.sum(0) + cm.sum(1) - tp) > 0).double()  # tp + fp + fn > 0
    return ((score * w).sum() / w.sum()).float() if w.sum() > 0 else score.sum().float() * 0


class Accuracy(_Confusion):
    """MulticlassAccuracy, average='macro' (per-class recall, torchmetrics class weighting)."""

    def compute(self):
        cm = self.confusion().double()
        return _macro(cm.diag() / cm.sum(1).clamp_min(1), cm)


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
        denom = 2 * tp + (cm.sum(0) - tp) + (cm.sum(1) - tp)  # 2tp + fp + fn
        return _macro(torch.where(denom > 0, 2 * tp / denom.clamp_min(1), torch.zeros_like(tp)), cm)


def _avg_ranks(v: torch.Tensor) -> torch.Tensor:
    """1-based ranks with ties sharing their average rank (Mann-Whitney form of the ROC area)."""
    order = v.argsort()
    sv = v[order]
    _, inv, counts = torch.unique_consecutive(sv, return_inverse=True, return_counts=True)
    ends = counts.cumsum(0).double()
    avg = ends - (counts.double() - 1) / 2
    ranks = torch.empty(v.numel(), dtype=torch.float64)
    ranks[order] = avg[inv]
    return ranks


class AUROC:
    """MulticlassAUROC, average='macro', one-vs-rest.  Scores are softmaxed per update unless already in
    [0, 1] (torchmetrics' rule: AST's sigmoid outputs are used as they are); a class without positives
    (or without negatives) scores 0 and counts in the mean, as in torchmetrics 1.7 (parity unpinned:
    torchmetrics is not importable here); ties get average ranks (= the trapezoidal ROC area).  Scores are gathered from every
    rank at compute()."""

    def __init__(self, num_classes: int):
        self.C = num_classes
        self.reset()

    def reset(self):
        self.scores, self.targets = [], []

    def update(self, logits, target):
        s = logits.detach().float()
        if not bool(((s >= 0) & (s <= 1)).all()):
            s = torch.softmax(s, dim=1)
        self.scores.append(s.cpu())
        self.targets.append(target.detach().long().cpu())

    def compute(self):
        s = torch.cat(self.scores) if self.scores else torch.zeros(0, self.C)
        t = torch.cat(self.targets) if self.targets else torch.zeros(0, dtype=torch.long)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            parts = [None] * dist.get_world_size()
            dist.all_gather_object(parts, (s, t))
            s = torch.cat([p[0] for p in parts])
            t = torch.cat([p[1] for p in parts])
        aucs = []
        for c in range(self.C):
            pos = t == c
            npos, nneg = int(pos.sum()), int((~pos).sum())
            if npos == 0 or nneg == 0:
                # torchmetrics 1.7 (_binary_roc_compute) returns an all-zero TPR (no positives) or FPR (no
                # negatives) curve here, whose area 0 enters the macro mean (it drops only NaN)
                aucs.append(torch.tensor(0.0, dtype=torch.float64))
                continue
            r = _avg_ranks(s[:, c].double())
            aucs.append((r[pos].sum() - npos * (npos + 1) / 2) / (npos * nneg))
        return torch.stack(aucs).mean().float() if aucs else torch.tensor(0.0)
