"""CPU restatement of the reference AST model (TEST INFRASTRUCTURE).

Follows src/models/ast.py:8-63 and the timm 1.0.16 VisionTransformer pieces it
reuses (uv.lock:2136; timm is absent here, its published Block is restated):
  patch_embed = Conv2d(1, 768, 16, stride 10), weight = RGB-mean of DeiT's (ast.py:30-33)
  pos_embed   = cls + bilinear(24x24 -> 12x275, align_corners=False)     (ast.py:42-48)
  x = cat(cls, patches) + pos_embed[:, :N]  (flat-index quirk, ast.py:59)
  12 x [x + proj(SDPA(qkv(LN1 x))); x + fc2(GELU_erf(fc1(LN2 x)))], LN eps 1e-6
  out = sigmoid(head(LN(x)[:, 0]))                                          (ast.py:63)

``deit_hash_state`` is the synthetic stand-in for the pretrained DeiT-B/384 weights
that the reference downloads (unavailable offline).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .synth import hash_uniform

EMBED = 768
DEPTH = 12
HEADS = 12
MLP = 3072
OLD_GRID = (24, 24)


def new_grid(sample_rate=44100, patch_size=16, overlap=6, f_dim=128):
    t_dim = int((sample_rate * 10) / 160) + 1
    return ((f_dim - patch_size) // (patch_size - overlap) + 1,
            (t_dim - patch_size) // (patch_size - overlap) + 1)


def deit_state_shapes(depth: int = DEPTH):
    s = {
        "patch_embed.proj.weight": (EMBED, 3, 16, 16),
        "patch_embed.proj.bias": (EMBED,),
        "cls_token": (1, 1, EMBED),
        "pos_embed": (1, OLD_GRID[0] * OLD_GRID[1] + 1, EMBED),
        "norm.weight": (EMBED,),
        "norm.bias": (EMBED,),
    }
    for i in range(depth):
        p = f"blocks.{i}."
        s[p + "norm1.weight"] = (EMBED,)
        s[p + "norm1.bias"] = (EMBED,)
        s[p + "attn.qkv.weight"] = (3 * EMBED, EMBED)
        s[p + "attn.qkv.bias"] = (3 * EMBED,)
        s[p + "attn.proj.weight"] = (EMBED, EMBED)
        s[p + "attn.proj.bias"] = (EMBED,)
        s[p + "norm2.weight"] = (EMBED,)
        s[p + "norm2.bias"] = (EMBED,)
        s[p + "mlp.fc1.weight"] = (MLP, EMBED)
        s[p + "mlp.fc1.bias"] = (MLP,)
        s[p + "mlp.fc2.weight"] = (EMBED, MLP)
        s[p + "mlp.fc2.bias"] = (EMBED,)
    return s


def deit_hash_state(seed: int = 300, depth: int = DEPTH):
    out = {}
    for i, (name, shape) in enumerate(sorted(deit_state_shapes(depth).items())):
        s = seed + 7919 * i
        if name in ("cls_token", "pos_embed"):
            out[name] = (0.02 * hash_uniform(s, shape)).astype(np.float32)
        elif name.endswith("norm.weight") or name.endswith("norm1.weight") or name.endswith("norm2.weight"):
            out[name] = (1.0 + 0.1 * hash_uniform(s, shape)).astype(np.float32)
        elif name.endswith(".weight"):
            fan_in = int(np.prod(shape[1:]))
            out[name] = (hash_uniform(s, shape) * math.sqrt(3.0 / fan_in)).astype(np.float32)
        else:
            out[name] = (0.02 * hash_uniform(s, shape)).astype(np.float32)
    return out


def head_hash(seed: int = 900, num_classes: int = 50):
    w = (hash_uniform(seed, (num_classes, EMBED)) * math.sqrt(3.0 / EMBED)).astype(np.float32)
    b = (0.02 * hash_uniform(seed + 1, (num_classes,))).astype(np.float32)
    return w, b


def interpolate_pos_embed(pos_embed: torch.Tensor, grid=None) -> torch.Tensor:
    grid = grid or new_grid()
    cls = pos_embed[:, :1]
    patch = pos_embed[:, 1:].reshape(1, *OLD_GRID, -1).permute(0, 3, 1, 2)
    patch = F.interpolate(patch, size=grid, mode="bilinear", align_corners=False)
    patch = patch.permute(0, 2, 3, 1).reshape(1, -1, pos_embed.shape[-1])
    return torch.cat((cls, patch), dim=1)


def model_params(deit_state, head_w, head_b, depth: int = DEPTH):
    """Apply the reference's __init__ transforms (ast.py:30-40) -> AST parameter dict."""
    t = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in deit_state.items()}
    p = {
        "patch_embed.weight": t["patch_embed.proj.weight"].mean(dim=1, keepdim=True),
        "patch_embed.bias": t["patch_embed.proj.bias"].clone(),
        "cls_token": t["cls_token"].clone(),
        "pos_embed": interpolate_pos_embed(t["pos_embed"]),
        "norm.weight": t["norm.weight"], "norm.bias": t["norm.bias"],
        "head.weight": torch.from_numpy(head_w), "head.bias": torch.from_numpy(head_b),
    }
    for i in range(depth):
        for k in ("norm1.weight", "norm1.bias", "attn.qkv.weight", "attn.qkv.bias",
                  "attn.proj.weight", "attn.proj.bias", "norm2.weight", "norm2.bias",
                  "mlp.fc1.weight", "mlp.fc1.bias", "mlp.fc2.weight", "mlp.fc2.bias"):
            p[f"transformer.{i}.{k}"] = t[f"blocks.{i}.{k}"]
    return p


def block(p, pre, x, lin=F.linear):
    """timm Block; ``lin`` replaces the four block linears (tests: an MX-fp8 emulation for fp8-mixed)."""
    B, N, C = x.shape
    h = F.layer_norm(x, (C,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], 1e-6)
    qkv = lin(h, p[pre + "attn.qkv.weight"], p[pre + "attn.qkv.bias"])
    qkv = qkv.reshape(B, N, 3, HEADS, C // HEADS).permute(2, 0, 3, 1, 4)
    q, k, v = qkv.unbind(0)
    scale = (C // HEADS) ** -0.5
    a = torch.softmax((q * scale) @ k.transpose(-2, -1), dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, N, C)
    x = x + lin(a, p[pre + "attn.proj.weight"], p[pre + "attn.proj.bias"])
    h = F.layer_norm(x, (C,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], 1e-6)
    h = F.gelu(lin(h, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"]))
    return x + lin(h, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])


def forward(p, x, depth: int = DEPTH, return_logits: bool = False, lin=F.linear):
    """ASTModel.forward (ast.py:50-63). x: (B, 128, F) or (B, 1, 128, F)."""
    if x.dim() == 3:
        x = x.unsqueeze(1)
    x = F.conv2d(x, p["patch_embed.weight"], p["patch_embed.bias"], stride=10)
    x = x.flatten(2).transpose(1, 2)
    cls = p["cls_token"].expand(x.shape[0], -1, -1)
    x = torch.cat((cls, x), dim=1)
    x = x + p["pos_embed"][:, :x.size(1)]
    for i in range(depth):
        x = block(p, f"transformer.{i}.", x, lin)
    x = F.layer_norm(x, (x.shape[-1],), p["norm.weight"], p["norm.bias"], 1e-6)
    z = F.linear(x[:, 0], p["head.weight"], p["head.bias"])
    return z if return_logits else torch.sigmoid(z)
