"""CPU restatement of OCP MX-fp8 quantisation and the MX GEMM (TEST INFRASTRUCTURE).

North-star config 5 ("AST, fp8 MFMA weights") has no counterpart in the reference (its AST runs bf16 /
fp16 autocast nn.Linear, src/models/ast.py:38,60-61 inside timm's Block), so parity is unpinned beyond
the published format: OCP Microscaling Formats (MX) v1.0, MXFP8 with E4M3 elements --
  * block = 32 consecutive elements along K, one shared E8M0 scale X = 2^e;
  * e = floor(log2(max |x| over the block)) - emax_elem, emax_elem = 8 for E4M3; E8M0 byte = e + 127;
  * elements P_i = x_i / X rounded to nearest-even E4M3 (OCP e4m3fn: bias 7, max normal 448, no inf),
    values beyond +-448 saturated (the spec leaves overflow implementation-defined; this build clamps);
  * value of an element = X * P_i.
torch.float8_e4m3fn is that element format, so its cast (round-to-nearest-even) is the reference rounding.
An all-zero block takes scale byte 0 (e = -127).  Only tests/ use this module.
"""
from __future__ import annotations

import torch

E4M3_MAX = 448.0
EMAX_ELEM = 8


def quantize(x: torch.Tensor):
    """x [rows][cols] (cols % 32 == 0) -> (q uint8 [rows][cols] e4m3fn bytes, scales uint8 [rows][cols/32])."""
    x = x.float()
    rows, cols = x.shape
    blk = x.reshape(rows, cols // 32, 32)
    amax = blk.abs().amax(dim=2)
    # floor(log2(amax)) from the float's exponent field (exact for normal numbers; subnormal/zero -> -127)
    bits = amax.view(torch.int32)
    be = (bits >> 23) & 0xFF
    e = torch.where(be == 0, torch.full_like(be, -127), be - 127 - EMAX_ELEM).clamp(-127, 127)
    scale = torch.pow(2.0, -e.double()).float()
    y = (blk * scale[..., None]).clamp(-E4M3_MAX, E4M3_MAX)
    q = y.to(torch.float8_e4m3fn).view(torch.uint8).reshape(rows, cols)
    return q, (e + 127).to(torch.uint8)


def dequantize(q: torch.Tensor, scales: torch.Tensor) -> torch.Tensor:
    """float64 values X * P of an MX-fp8 tensor."""
    rows, cols = q.shape
    p = q.view(torch.float8_e4m3fn).to(torch.float64).reshape(rows, cols // 32, 32)
    x = torch.pow(2.0, scales.to(torch.float64) - 127.0)
    return (p * x[..., None]).reshape(rows, cols)


def gemm(qa, sa, qb, sb) -> torch.Tensor:
    """float64 A B^T of two MX-fp8 operands (A [M][K], B [N][K])."""
    return dequantize(qa, sa) @ dequantize(qb, sb).T


# the block linears whose backward-data GEMM runs on MX-fp8 operands in the HIP path (src/models/ast_hip.py
# MX_DGRAD): dx = MX(dy) MX(W^T)^T, W^T quantised in blocks of 32 along the output features; the qkv
# backward-data and every weight gradient stay bf16
MX_DGRAD = ("proj", "fc1", "fc2")


def block_linear_kind(w: torch.Tensor) -> str:
    """Which ViT block linear a weight [out][in] is, from its shape (D = embedding width)."""
    o, i = w.shape
    return {(3 * i): "qkv", i: "proj", (4 * i): "fc1"}.get(o, "fc2" if i == 4 * o else "?")


class MXLinear(torch.autograd.Function):
    """Emulation of an fp8-mixed block linear (TEST INFRASTRUCTURE): forward on the MX-fp8 values of the
    bf16-rounded activation (what autocast hands a Linear) and of the f32 weight, bf16 output as autocast's;
    backward: the weight gradient straight through in bf16 (the activations the backward sees are the
    unquantised ones, as in the HIP path, which keeps the bf16 tensors for its backward GEMMs), the
    backward-data product on MX-fp8 operands for the MX_DGRAD linears (MX of the bf16 dy and of W^T, as
    mia_mx_quantize / mia_mx_quantize_t), bf16 otherwise."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        shp = x.shape
        xb = x.detach().to(torch.bfloat16).float().reshape(-1, shp[-1]).cpu()
        xq = dequantize(*quantize(xb)).to(x.device)
        wq = dequantize(*quantize(w.detach().float().cpu())).to(x.device)
        y = (xq @ wq.T).float() + b.detach().float()
        return y.to(torch.bfloat16).reshape(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g = gy.to(torch.bfloat16).float().reshape(-1, gy.shape[-1])
        xb = x.to(torch.bfloat16).float().reshape(-1, x.shape[-1])
        if block_linear_kind(w) in MX_DGRAD:
            gq = dequantize(*quantize(g.cpu()))
            wtq = dequantize(*quantize(w.detach().float().t().contiguous().cpu()))
            gx = (gq @ wtq.T).float().to(torch.bfloat16).to(g.device).to(x.dtype).reshape(x.shape)
        else:
            gx = (g @ w.to(torch.bfloat16).float()).to(x.dtype).reshape(x.shape)
        return gx, (g.T @ xb).to(w.dtype), g.sum(0).to(w.dtype)


def mx_linear(x, w, b):
    return MXLinear.apply(x, w, b)
