"""CPU restatement of the reference training step (TEST INFRASTRUCTURE).

LitClassifier._step soft-label loss (src/training/engine.py:164-179), Lightning's
``gradient_clip_val: 1.0`` (configs/base_training.yaml:51 -> torch
clip_grad_norm_(max_norm=1.0, norm_type=2)) and ``torch.optim.Adam(lr, weight_decay)``
(base_training.yaml:56-59; L2-style decay added to the gradient), restated as
plain tensor arithmetic so every intermediate can be compared.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import torch


def soft_ce(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    probs = torch.softmax(logits, dim=1)
    return -torch.sum(y * torch.log(probs + 1e-8), dim=1).mean()


def clip_grad_norm(grads, max_norm: float = 1.0):
    """torch.nn.utils.clip_grad_norm_: coef = max_norm / (total + 1e-6), clamped to 1."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return [g * coef for g in grads], float(total)


def adam_step(p, g, m, v, step: int, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-4):
    """torch.optim.Adam single-tensor update (non-amsgrad, non-maximize)."""
    g = g + weight_decay * p
    m = m * beta1 + (1 - beta1) * g
    v = v * beta2 + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = v.sqrt() / (bc2 ** 0.5) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v
