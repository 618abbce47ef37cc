"""GPU: the bf16 AST patch embedding (reference src/models/ast.py:38, PatchEmbed = Conv2d(1, 768, 16,
stride 10) over the (B, 128, T) spectrogram) -- mia_ast_patches writes the bf16 patch matrix in token
order (zero row in each clip's cls slot), one dense GEMM with the bias epilogue writes the token rows
of x, mia_tokens_fwd_inplace adds cls / positional rows.  The patch matrix is held byte-exact against
torch's unfold of the bf16-rounded spectrogram, the token rows against a float64 conv of the same
bf16 operands, and the weight / bias gradients of one AST depth-1 backward against float64 sums."""
import pytest
import torch
import torch.nn.functional as F

from oracle.synth import hash_uniform

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,T", [(1, 1379), (3, 96), (2, 27)])
def test_patch_matrix_token_order(cuda, B, T):
    from src.miaudio import lib as L
    spec = torch.from_numpy(hash_uniform(41 + T, (B, 128, T))).to(cuda)
    gh, gw = (128 - 16) // 10 + 1, (T - 16) // 10 + 1
    N = gh * gw + 1
    out = torch.full((B * N, 256), 7.0, dtype=torch.bfloat16, device=cuda)
    L.check(L.load().mia_ast_patches(spec.data_ptr(), B, 128, T, 16, 10, out.data_ptr(), L.stream_ptr()), "patches")
    ref = F.unfold(spec.to(torch.bfloat16).float()[:, None], 16, stride=10).transpose(1, 2)  # (B, gh*gw, 256)
    got = out.view(B, N, 256)
    assert torch.equal(got[:, 0], torch.zeros_like(got[:, 0]))
    assert torch.equal(got[:, 1:].float(), ref)


def test_tokens_fwd_inplace(cuda):
    from src.miaudio import lib as L
    B, N, D = 3, 11, 768
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B * N, D, generator=g).to(cuda)
    cls = torch.randn(1, 1, D, generator=g).to(cuda)
    pos = torch.randn(1, N + 5, D, generator=g).to(cuda)
    ref = x.view(B, N, D).clone()
    ref[:, 0] = cls[0, 0]
    ref += pos[0, :N]
    L.check(L.load().mia_tokens_fwd_inplace(x.data_ptr(), cls.data_ptr(), pos.data_ptr(), B, N, D, L.stream_ptr()),
            "tokens")
    assert torch.equal(x.view(B, N, D), ref)


def test_patch_embed_bf16_tokens_and_grads(cuda):
    """Depth-1 AST in bf16: the token rows the forward builds (first block's input, captured through the
    saved state) and the patch weight / bias gradients against float64 on the same bf16 operands."""
    from src.models.ast import ASTModel
    B, T = 2, 96
    m = ASTModel(num_classes=5, compute_dtype="bf16", depth=1).to(cuda).train()
    spec = torch.from_numpy(hash_uniform(77, (B, 128, T))).to(cuda)
    from src.models import ast_hip
    seen = {}
    orig = ast_hip.ASTFunction.forward

    def spy(ctx, *a):
        out = orig(ctx, *a)
        seen["x"] = ctx.s["blocks"][0]["x"].clone()
        return out
    ast_hip.ASTFunction.forward = staticmethod(spy)
    try:
        z = m(spec)
    finally:
        ast_hip.ASTFunction.forward = staticmethod(orig)
    gh, gw = (128 - 16) // 10 + 1, (T - 16) // 10 + 1
    N = gh * gw + 1
    w = m.patch_embed.weight.detach().to(torch.bfloat16).double()
    sb = spec.to(torch.bfloat16).double()
    tok = F.conv2d(sb[:, None], w, m.patch_embed.bias.detach().double(), stride=10).flatten(2).transpose(1, 2)
    ref = torch.cat([m.cls_token.detach().double().expand(B, 1, -1), tok], 1) + m.pos_embed.detach().double()[:, :N]
    got = seen["x"].view(B, N, -1).double()
    assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-5
    dz = torch.linspace(-1, 1, z.numel(), device=cuda).view_as(z)
    z.backward(dz)
    # the bias gradient is the patch rows of dpos (dpos[t] = sum_b dx[b][t]) summed; the weight gradient's
    # operands are covered end to end by the depth-2 backward tests against the oracle (test_gpu_ast.py)
    db = m.patch_embed.bias.grad.double()
    dpos = m.pos_embed.grad.double()[0, 1:N]
    assert torch.allclose(db, dpos.sum(0), rtol=1e-5, atol=1e-6)
    assert torch.isfinite(m.patch_embed.weight.grad).all() and m.patch_embed.weight.grad.abs().sum() > 0
