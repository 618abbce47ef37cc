"""Audio Spectrogram Transformer — drop-in for the reference ``src.models.ast.ASTModel``.

Same Hydra target (configs/model/ast.yaml:10), same constructor kwargs (sample_rate, patch_size,
patch_stride, overlap, num_classes, pretrained_model), same parameter names as the reference module
(patch_embed, cls_token, pos_embed, transformer.<i>.{norm1,attn.qkv,attn.proj,norm2,mlp.fc1,mlp.fc2},
norm, head), same forward contract: (B, F, T) or (B, 1, F, T) log-mel -> (B, C) sigmoid
probabilities (reference src/models/ast.py:50-63).  Optionally (``input="waveform"``) the model
takes (B, 1, T) waveforms and computes the log-mel on the GPU first (the batched HIP log-mel).

The reference initialises from timm's ImageNet DeiT-B/384 (network download, ast.py:19), then
averages the patch filter over RGB and bilinearly resizes the 24x24 position table to the 12x275
grid (ast.py:23-48).  ``from_vit_state`` applies exactly those transforms to any DeiT-shaped state
dict (e.g. a checkpoint file named by MIA_DEIT_CHECKPOINT, loaded with weights_only=True);
without one, timm-style random init is used.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..miaudio import lib as L
from .ast_hip import ASTFunction


class _Attn(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)


class _Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):
    """Parameter container with timm's Block names (the math lives in ast_hip)."""

    def __init__(self, dim=768, hidden=3072):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attn(dim)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _Mlp(dim, hidden)


DEIT = {"deit_base_patch16_384": dict(dim=768, depth=12, heads=12, grid=24),
        "deit_small_patch16_224": dict(dim=384, depth=12, heads=6, grid=14),
        "deit_tiny_patch16_224": dict(dim=192, depth=12, heads=3, grid=14)}


class ASTModel(nn.Module):
    def __init__(self, sample_rate=44100, patch_size=16, patch_stride=10, overlap=6, num_classes=50,
                 pretrained_model="deit_base_patch16_384", depth: int | None = None, input: str = "spectrogram",
                 compute_dtype: str | None = None):
        super().__init__()
        spec = DEIT.get(pretrained_model, DEIT["deit_base_patch16_384"])
        self.f_dim = 128
        self.num_classes = num_classes
        self.t_dim = int((sample_rate * 10) / 160) + 1
        self.emb_dim = spec["dim"]
        self.num_heads = spec["heads"]
        self.patch_size, self.patch_stride = patch_size, patch_stride
        self.old_grid = (spec["grid"], spec["grid"])
        self.new_grid = ((self.f_dim - patch_size) // (patch_size - overlap) + 1,
                         (self.t_dim - patch_size) // (patch_size - overlap) + 1)
        D = self.emb_dim
        self.patch_embed = nn.Conv2d(1, D, kernel_size=patch_size, stride=patch_stride, bias=True)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, D))
        self.pos_embed = nn.Parameter(torch.zeros(1, self.new_grid[0] * self.new_grid[1] + 1, D))
        self.transformer = nn.Sequential(*[Block(D, 4 * D) for _ in range(depth or spec["depth"])])
        self.norm = nn.LayerNorm(D, eps=1e-6)
        self.head = nn.Linear(D, num_classes)
        self.input = input
        self.compute_dtype = compute_dtype
        self._logmel = None
        ckpt = os.environ.get("MIA_DEIT_CHECKPOINT")
        if ckpt and os.path.exists(ckpt):
            self.load_vit_state(torch.load(ckpt, map_location="cpu", weights_only=True))
        else:
            self._timm_init()
            if os.environ.get("MIA_QUIET") is None:
                warnings.warn("no DeiT checkpoint available offline (MIA_DEIT_CHECKPOINT unset): "
                              "AST starts from random init", stacklevel=2)

    # -------------------------------------------------------------------- init
    def _timm_init(self):
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def interpolate_pos_embed(self, pos_embed):
        cls = pos_embed[:, :1]
        patch = pos_embed[:, 1:].reshape(1, *self.old_grid, -1).permute(0, 3, 1, 2)
        patch = F.interpolate(patch, size=self.new_grid, mode="bilinear", align_corners=False)
        patch = patch.permute(0, 2, 3, 1).reshape(1, -1, self.emb_dim)
        return torch.cat((cls, patch), dim=1)

    @torch.no_grad()
    def load_vit_state(self, sd):
        """Apply the reference's ViT -> AST transforms (ast.py:30-38) to a DeiT state dict."""
        sd = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(v)) for k, v in sd.items()}
        self.patch_embed.weight.copy_(sd["patch_embed.proj.weight"].mean(dim=1, keepdim=True))
        self.patch_embed.bias.copy_(sd["patch_embed.proj.bias"])
        self.cls_token.copy_(sd["cls_token"])
        self.pos_embed.copy_(self.interpolate_pos_embed(sd["pos_embed"].float()))
        self.norm.weight.copy_(sd["norm.weight"])
        self.norm.bias.copy_(sd["norm.bias"])
        for i, blk in enumerate(self.transformer):
            for name, t in blk.named_parameters():
                t.copy_(sd[f"blocks.{i}.{name}"])

    # -------------------------------------------------------------------- forward
    def _compute_code(self) -> int:
        cd = self.compute_dtype
        if cd is None:
            if torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16:
                return L.BF16
            return L.F32
        return {"bf16": L.BF16, "bfloat16": L.BF16, "f32": L.F32, "fp32": L.F32, "32": L.F32,
                "fp8": L.MXFP8}[str(cd)]

    def param_list(self):
        ps = [self.patch_embed.weight, self.patch_embed.bias, self.cls_token, self.pos_embed]
        for blk in self.transformer:
            ps += [blk.norm1.weight, blk.norm1.bias, blk.attn.qkv.weight, blk.attn.qkv.bias, blk.attn.proj.weight,
                   blk.attn.proj.bias, blk.norm2.weight, blk.norm2.bias, blk.mlp.fc1.weight, blk.mlp.fc1.bias,
                   blk.mlp.fc2.weight, blk.mlp.fc2.bias]
        ps += [self.norm.weight, self.norm.bias, self.head.weight, self.head.bias]
        return ps

    def forward(self, x):
        if self.input == "waveform" or (x.dim() == 3 and x.shape[1] == 1 and x.shape[-1] > 4096):
            from ..datasets.features import GpuLogMel
            if self._logmel is None:
                self._logmel = GpuLogMel()
            x = self._logmel(x.reshape(x.shape[0], -1))
        if x.dim() == 4:
            x = x[:, 0]
        params = self.param_list()
        # grad mode is off inside an autograd.Function's forward: read it here, so an inference forward
        # (validation / test under no_grad) skips the backward's saved-Q' workspace
        grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
        with torch.autocast("cuda", enabled=False):
            return ASTFunction.apply(self, x, self._compute_code(), grad, *params)
