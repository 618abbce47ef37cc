"""CPU restatement of the reference EnvNet-v2 (TEST INFRASTRUCTURE).

Follows src/models/envnet_v2.py:10-90 op-for-op as plain ``torch.nn.functional``
calls over an explicit parameter dict (reference parameter names and layouts), so
the checker is independent of the product's module classes.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .synth import hash_uniform

# (name, in_ch, out_ch, kernel, stride)   envnet_v2.py:14-45
CONVS = [
    ("frontend.0", 1, 32, (1, 64), (1, 2)),
    ("frontend.3", 32, 64, (1, 16), (1, 2)),
    ("trunk.0.0", 1, 32, (8, 8), (1, 1)),
    ("trunk.0.3", 32, 32, (8, 8), (1, 1)),
    ("trunk.1.0", 32, 64, (1, 4), (1, 1)),
    ("trunk.1.3", 64, 64, (1, 4), (1, 1)),
    ("trunk.2.0", 64, 128, (1, 2), (1, 1)),
    ("trunk.2.3", 128, 128, (1, 2), (1, 1)),
    ("trunk.3.0", 128, 256, (1, 2), (1, 1)),
    ("trunk.3.3", 256, 256, (1, 2), (1, 1)),
]
# BN follows each conv at index+1 (envnet_v2.py:16,20,32,35)
POOLS = {  # pool after the block, envnet_v2.py:23,41-44
    "frontend": ((1, 64), (1, 64)),
    "trunk.0": ((5, 3), (5, 3)),
    "trunk.1": ((1, 2), (1, 2)),
    "trunk.2": ((1, 2), (1, 2)),
    "trunk.3": ((1, 2), (1, 2)),
}
FCS = [("classifier.1", 84480, 4096), ("classifier.4", 4096, 4096), ("classifier.7", 4096, None)]


def bn_name(conv_name: str) -> str:
    pre, idx = conv_name.rsplit(".", 1)
    return f"{pre}.{int(idx) + 1}"


def param_shapes(num_classes: int = 50):
    shapes = {}
    for name, cin, cout, k, _ in CONVS:
        shapes[f"{name}.weight"] = (cout, cin, *k)
        shapes[f"{name}.bias"] = (cout,)
        b = bn_name(name)
        shapes[f"{b}.weight"] = (cout,)
        shapes[f"{b}.bias"] = (cout,)
    for name, fin, fout in FCS:
        fout = fout or num_classes
        shapes[f"{name}.weight"] = (fout, fin)
        shapes[f"{name}.bias"] = (fout,)
    return shapes


def buffer_shapes():
    out = {}
    for name, _, cout, _, _ in CONVS:
        b = bn_name(name)
        out[f"{b}.running_mean"] = (cout,)
        out[f"{b}.running_var"] = (cout,)
    return out


def hash_params(seed: int = 100, num_classes: int = 50):
    """Deterministic synthetic parameters + BN buffers (reference layout), numpy float32."""
    p = {}
    for i, (name, shape) in enumerate(sorted(param_shapes(num_classes).items())):
        s = seed + 7919 * i
        if name.endswith(".weight") and len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            bound = math.sqrt(6.0 / fan_in)
            p[name] = hash_uniform(s, shape) * np.float32(bound)
        elif name.endswith(".weight"):  # BN gamma
            p[name] = (1.0 + 0.1 * hash_uniform(s, shape)).astype(np.float32)
        else:
            p[name] = (0.05 * hash_uniform(s, shape)).astype(np.float32)
    for i, (name, shape) in enumerate(sorted(buffer_shapes().items())):
        s = seed + 104729 + 31 * i
        if name.endswith("running_var"):
            p[name] = (1.0 + 0.5 * hash_uniform(s, shape, 0.0, 1.0)).astype(np.float32)
        else:
            p[name] = (0.1 * hash_uniform(s, shape)).astype(np.float32)
    return p


def forward(params, x, training: bool, dropout_p: float = 0.5, momentum: float = 0.1,
            eps: float = 1e-5, dropout_masks=None):
    """EnvNetV2.forward (envnet_v2.py:76-85). ``params`` holds torch tensors.
    In training mode BN running stats in ``params`` are updated in place (momentum 0.1,
    unbiased running_var) exactly as nn.BatchNorm2d does."""
    if x.dim() == 2:
        x = x.unsqueeze(1)
    if x.dim() == 3:
        x = x.unsqueeze(2)

    def cbr(h, name, stride):
        h = F.conv2d(h, params[f"{name}.weight"], params[f"{name}.bias"], stride=stride)
        b = bn_name(name)
        h = F.batch_norm(h, params[f"{b}.running_mean"], params[f"{b}.running_var"],
                         params[f"{b}.weight"], params[f"{b}.bias"], training, momentum, eps)
        return F.relu(h)

    convs = {c[0]: c for c in CONVS}
    h = cbr(x, "frontend.0", (1, 2))
    h = cbr(h, "frontend.3", (1, 2))
    k, s = POOLS["frontend"]
    h = F.max_pool2d(h, k, s)
    h = h.transpose(1, 2)
    for blk in range(4):
        pre = f"trunk.{blk}"
        h = cbr(h, f"{pre}.0", convs[f"{pre}.0"][4])
        h = cbr(h, f"{pre}.3", convs[f"{pre}.3"][4])
        k, s = POOLS[pre]
        h = F.max_pool2d(h, k, s)
    h = h.flatten(1)
    for i, (name, _, _) in enumerate(FCS):
        h = F.linear(h, params[f"{name}.weight"], params[f"{name}.bias"])
        if i < 2:
            h = F.relu(h)
            if dropout_masks is not None:
                h = h * dropout_masks[i]
            else:
                h = F.dropout(h, dropout_p, training)
    return h


def soft_ce(logits, y):
    """engine.py:175-176: -(y * log(softmax(z) + 1e-8)).sum(1).mean()"""
    probs = torch.softmax(logits, dim=1)
    return -torch.sum(y * torch.log(probs + 1e-8), dim=1).mean()


def to_torch(params, requires_grad=False):
    out = {}
    for k, v in params.items():
        t = torch.from_numpy(np.ascontiguousarray(v)).float()
        if requires_grad and not (k.endswith("running_mean") or k.endswith("running_var")):
            t.requires_grad_(True)
        out[k] = t
    return out


def trainable_names(params):
    return [k for k in sorted(params) if not (k.endswith("running_mean") or k.endswith("running_var"))]
