"""GPU: attention / LayerNorm kernels vs float64 torch, and ASTModel (HIP path) vs the reference's
golden outputs (reference ASTModel code run with the offline timm restatement + hash DeiT weights).
f32 compute: probabilities within 1e-3 rel, argmax exact.  bf16 compute: argmax exact, 5e-2."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ast as oast
from oracle.synth import hash_uniform
from src.miaudio import lib as L

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _attn_ref(qkv, B, N, H):
    q, k, v = qkv.double().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    q.requires_grad_(True), k.requires_grad_(True), v.requires_grad_(True)
    o = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ v
    return q, k, v, o


@pytest.mark.parametrize("dt", [L.BF16, L.F32])
@pytest.mark.parametrize("B,N,H", [(2, 100, 2), (1, 257, 3), (2, 1645, 1), (3, 37, 2), (4, 300, 2), (8, 1645, 1),
                                   (1, 64, 2), (1, 128, 1), (1, 192, 1), (1, 520, 1)])
def test_attention_fwd_bwd(cuda, dt, B, N, H):
    g = torch.Generator().manual_seed(N + H)
    tdt = torch.bfloat16 if dt == L.BF16 else torch.float32
    qkv = (torch.randn(B, N, 3 * H * 64, generator=g) * 1.5).to(tdt)
    dout = torch.randn(B, N, H * 64, generator=g).to(tdt)
    q, k, v, o = _attn_ref(qkv, B, N, H)
    o.backward(dout.double().view(B, N, H, 64).permute(0, 2, 1, 3))
    tq = qkv.to(cuda)
    out = torch.empty(B, N, H * 64, dtype=tdt, device=cuda)
    lse = torch.empty(B, H, N, device=cuda)
    lib = L.load()
    L.check(lib.mia_attn_fwd(tq.data_ptr(), out.data_ptr(), lse.data_ptr(), dt, B, N, H, 0.125, L.stream_ptr()), "fwd")
    dq = torch.empty_like(tq)
    work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(dt, B, N, H)), dtype=torch.uint8, device=cuda)
    L.check(lib.mia_attn_bwd(tq.data_ptr(), out.data_ptr(), dout.to(cuda).data_ptr(), lse.data_ptr(), dq.data_ptr(),
                             work.data_ptr(), dt, B, N, H, 0.125, L.stream_ptr()), "bwd")
    torch.cuda.synchronize()
    tol = 2e-2 if dt == L.BF16 else 1e-5
    assert rel(out.view(B, N, H, 64).permute(0, 2, 1, 3), o) < tol
    lse_ref = torch.logsumexp(q.detach() @ k.detach().transpose(-1, -2) / 8.0, -1)  # (B, H, N)
    assert float((lse.cpu().double() - lse_ref).abs().max()) < (2e-2 if dt == L.BF16 else 1e-5)
    dqkv = dq.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    assert rel(dqkv[0], q.grad) < 3 * tol
    assert rel(dqkv[1], k.grad) < 3 * tol
    assert rel(dqkv[2], v.grad) < 3 * tol


@pytest.mark.parametrize("profile", ["grow", "decay", "spike"])
def test_attention_running_max_paths(cuda, profile):
    """The bf16 forward keeps its running max across tiles until a tile's exp-sum passes 2^16, then
    moves it (rescaling O, l and the already computed next tile).  Key norms that grow along the
    sequence force that move in the middle of the loop many times; decaying norms leave the first
    tile's max standing (later p tiny, never rescaled); a single huge key forces it exactly once."""
    B, N, H = 2, 1645, 2
    g = torch.Generator().manual_seed(7)
    qkv = torch.randn(B, N, 3, H, 64, generator=g) * 1.5
    pos = torch.arange(N, dtype=torch.float64) / N
    if profile == "grow":
        qkv[:, :, 1] *= (1 + 6 * pos).view(1, N, 1, 1).float()
    elif profile == "decay":
        qkv[:, :, 1] *= (7 - 6 * pos).view(1, N, 1, 1).float()
    else:
        qkv[:, 1000, 1] = qkv[:, 700, 0] * 6  # key 1000 aligned with query 700, scores ~ +300
    qkv = qkv.reshape(B, N, 3 * H * 64).to(torch.bfloat16)
    dout = torch.randn(B, N, H * 64, generator=g).to(torch.bfloat16)
    q, k, v, o = _attn_ref(qkv, B, N, H)
    o.backward(dout.double().view(B, N, H, 64).permute(0, 2, 1, 3))
    tq = qkv.to(cuda)
    out = torch.empty(B, N, H * 64, dtype=torch.bfloat16, device=cuda)
    lse = torch.empty(B, H, N, device=cuda)
    lib = L.load()
    L.check(lib.mia_attn_fwd(tq.data_ptr(), out.data_ptr(), lse.data_ptr(), L.BF16, B, N, H, 0.125, L.stream_ptr()),
            "fwd")
    dq = torch.empty_like(tq)
    work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=cuda)
    L.check(lib.mia_attn_bwd(tq.data_ptr(), out.data_ptr(), dout.to(cuda).data_ptr(), lse.data_ptr(), dq.data_ptr(),
                             work.data_ptr(), L.BF16, B, N, H, 0.125, L.stream_ptr()), "bwd")
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all() and torch.isfinite(dq.float()).all()
    # The kernel feeds Q * scale * log2(e) to the MFMA in bf16: one more rounding of q of the same size
    # as the bf16 rounding autocast already applies to the qkv Linear output.  Its effect grows with
    # the score magnitude (these profiles reach ~75 log2 units), so the output is held to 2e-2
    # against softmax of that rounded Q, and to 5e-2 against the exact float64 reference.
    c = 0.125 * math.log2(math.e)
    qr = (q.detach().float() * c).to(torch.bfloat16).double() / c
    o_qr = (torch.softmax(qr @ k.detach().transpose(-1, -2) / 8.0, -1) @ v.detach()).permute(0, 2, 1, 3)
    o_ref = o.detach().permute(0, 2, 1, 3)
    got = out.view(B, N, H, 64).double().cpu()
    assert float((got - o_qr).abs().max() / o_qr.abs().max()) < 2e-2
    assert float((got - o_ref).abs().max() / o_ref.abs().max()) < 5e-2
    lse_ref = torch.logsumexp(q.detach() @ k.detach().transpose(-1, -2) / 8.0, -1)
    assert float(((lse.cpu().double() - lse_ref).abs() / lse_ref.abs().clamp_min(1.0)).max()) < 5e-3
    # the backward recomputes P from that forward's lse, so its reference is the rounded-Q one too
    qr_ = qr.clone().requires_grad_(True)
    k_, v_ = k.detach().clone().requires_grad_(True), v.detach().clone().requires_grad_(True)
    o_r = torch.softmax(qr_ @ k_.transpose(-1, -2) / 8.0, -1) @ v_
    o_r.backward(dout.double().view(B, N, H, 64).permute(0, 2, 1, 3))
    dqkv = dq.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    for i, (ref_r, ref) in enumerate(zip((qr_.grad, k_.grad, v_.grad), (q.grad, k.grad, v.grad))):
        assert rel(dqkv[i], ref_r) < 6e-2, ("dq", "dk", "dv")[i]
        assert rel(dqkv[i], ref) < 1.2e-1, ("dq", "dk", "dv")[i]


@pytest.mark.parametrize("D", [768, 384, 1000])
def test_layernorm(cuda, D):
    from src.models.ast_hip import _ln, _ln_bwd
    g = torch.Generator().manual_seed(D)
    x = torch.randn(300, D, generator=g) * 2 + 1
    w = torch.rand(D, generator=g) + 0.5
    b = torch.randn(D, generator=g)
    xr = x.double().requires_grad_(True)
    wr, br = w.double().requires_grad_(True), b.double().requires_grad_(True)
    y = F.layer_norm(xr, (D,), wr, br, 1e-6)
    dy = torch.randn(300, D, generator=g)
    y.backward(dy.double())
    tx, tw, tb = x.to(cuda), w.to(cuda), b.to(cuda)
    yo, m, r, _ = _ln(tx, tw, tb, torch.float32, 300, D)
    dx = torch.ones(300, D, device=cuda)
    dg, db, cs = _ln_bwd(dy.to(cuda), tx, tw, m, r, dx, 300, D, True)
    dx2 = torch.ones(300, D, device=cuda)
    dg2, db2, _ = _ln_bwd(dy.to(cuda), tx, tw, m, r, dx2, 300, D, True)
    torch.cuda.synchronize()
    # reproducible bit for bit (both the vectorised D = 768 kernel and the generic one)
    assert torch.equal(dg, dg2) and torch.equal(db, db2) and torch.equal(dx, dx2)
    assert cs is None
    assert rel(yo, y) < 1e-5
    assert rel(dx - 1.0, xr.grad) < 1e-4
    assert rel(dg, wr.grad) < 1e-4 and rel(db, br.grad) < 1e-4


@pytest.mark.parametrize("rows", [300, 4096 + 17])
def test_layernorm_bwd_colsum(cuda, rows):
    """The LayerNorm backward that also returns the column sums of its bf16 copy dx2 (the proj / fc2
    bias gradients in the AST backward): dx, dx2, dgamma, dbeta bit-identical to the plain backward,
    the column sums equal to float64 sums of the stored dx2."""
    from src.models.ast_hip import _ln, _ln_bwd
    D = 768
    g = torch.Generator(device=cuda).manual_seed(rows)
    x = torch.randn(rows, D, generator=g, device=cuda) * 2 + 1
    w = torch.rand(D, generator=g, device=cuda) + 0.5
    b = torch.randn(D, generator=g, device=cuda)
    dy = torch.randn(rows, D, generator=g, device=cuda).to(torch.bfloat16)
    acc0 = torch.randn(rows, D, generator=g, device=cuda)
    _, m, r, _ = _ln(x, w, b, torch.bfloat16, rows, D)
    dxa, dxb = acc0.clone(), acc0.clone()
    d2a = torch.empty(rows, D, dtype=torch.bfloat16, device=cuda)
    d2b = torch.empty_like(d2a)
    lib = L.load()
    dga, dba = torch.empty(D, device=cuda), torch.empty(D, device=cuda)
    ws = torch.empty(int(lib.mia_layernorm_partial_bytes(rows, D)), dtype=torch.uint8, device=cuda)
    L.check(lib.mia_layernorm_bwd(dy.data_ptr(), L.BF16, x.data_ptr(), L.F32, w.data_ptr(), m.data_ptr(), r.data_ptr(),
                                  dxa.data_ptr(), L.F32, 1, d2a.data_ptr(), L.BF16, dga.data_ptr(), dba.data_ptr(),
                                  ws.data_ptr(), rows, D, L.stream_ptr()), "ln_bwd")
    dgb, dbb, cs = _ln_bwd(dy, x, w, m, r, dxb, rows, D, True, dx2=d2b)
    torch.cuda.synchronize()
    assert torch.equal(dxa, dxb) and torch.equal(d2a, d2b)
    assert torch.equal(dga, dgb) and torch.equal(dba, dbb)
    assert rel(cs, d2b.double().sum(0)) < 1e-5


def _ast(cuda, compute):
    import os
    os.environ["MIA_QUIET"] = "1"
    from src.models.ast import ASTModel
    m = ASTModel(num_classes=50, compute_dtype=compute)
    m.load_vit_state(oast.deit_hash_state(300))
    hw, hb = oast.head_hash(900, 50)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    return m.to(cuda)


def test_ast_param_count_and_names(cuda, golden):
    m = _ast(cuda, "f32")
    assert sum(p.numel() for p in m.parameters()) == int(golden["ast_nparams"])
    assert "transformer.11.mlp.fc2.weight" in m.state_dict()
    pe = m.pos_embed.detach().double().cpu()
    np.testing.assert_allclose([float(pe.sum()), float((pe ** 2).sum())], golden["ast_pos_embed_cs"], rtol=1e-5)


def test_ast_forward_f32_vs_golden(cuda, golden):
    m = _ast(cuda, "f32").eval()
    x = torch.from_numpy(hash_uniform(31, (2, 128, 1379))).to(cuda)
    with torch.no_grad():
        p = m(x).cpu().numpy()
    ref = golden["ast_probs"]
    assert np.abs(p - ref).max() / np.abs(ref).max() < 1e-3
    assert np.array_equal(p.argmax(1), ref.argmax(1))


def test_ast_forward_bf16(cuda, golden):
    m = _ast(cuda, "bf16").eval()
    x = torch.from_numpy(hash_uniform(31, (2, 128, 1379))).to(cuda)
    with torch.no_grad():
        p = m(x).cpu().numpy()
    ref = golden["ast_probs"]
    assert np.abs(p - ref).max() / np.abs(ref).max() < 5e-2
    assert np.array_equal(p.argmax(1), ref.argmax(1))


def test_ast_backward_f32_vs_oracle(cuda):
    """Two transformer blocks (depth override) so the CPU autograd reference stays fast."""
    import os
    os.environ["MIA_QUIET"] = "1"
    from src.models.ast import ASTModel
    torch.set_num_threads(16)
    m = ASTModel(num_classes=10, compute_dtype="f32", depth=2)
    st = oast.deit_hash_state(300, depth=2)
    m.load_vit_state(st)
    hw, hb = oast.head_hash(901, 10)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    m = m.to(cuda)
    x = hash_uniform(32, (2, 128, 1379))
    y = torch.zeros(2, 10)
    y[0, 3], y[1, 5], y[1, 2] = 1.0, 0.6, 0.4
    p = m(torch.from_numpy(x).to(cuda))
    loss = -torch.sum(y.to(cuda) * torch.log(torch.softmax(p, 1) + 1e-8), 1).mean()
    loss.backward()
    ref = oast.model_params(st, hw, hb, depth=2)
    for v in ref.values():
        v.requires_grad_(True)
    pr = oast.forward(ref, torch.from_numpy(x), depth=2)
    lr = -torch.sum(y * torch.log(torch.softmax(pr, 1) + 1e-8), 1).mean()
    lr.backward()
    assert abs(float(loss) - float(lr)) < 1e-4
    names = {"patch_embed.weight": "patch_embed.weight", "cls_token": "cls_token", "pos_embed": "pos_embed",
             "transformer.0.attn.qkv.weight": "transformer.0.attn.qkv.weight",
             "transformer.1.mlp.fc1.weight": "transformer.1.mlp.fc1.weight",
             "transformer.1.norm2.weight": "transformer.1.norm2.weight", "head.weight": "head.weight"}
    sd = dict(m.named_parameters())
    for mine, theirs in names.items():
        got, want = sd[mine].grad.cpu().double(), ref[theirs].grad.double()
        l2 = float((got - want).norm() / want.norm().clamp_min(1e-30))
        assert l2 < 1e-3, (mine, l2)


@pytest.mark.parametrize("B,N,H,mx", [(2, 1645, 12, False), (1, 77, 2, True), (3, 130, 3, False)])
def test_attn_saved_q_equals_plain(cuda, B, N, H, mx):
    """The training form of the bf16 attention (forward writes Q' into the backward workspace, the
    backward's prep skips it) gives outputs, lse, MX copies and dqkv identical to the plain entries."""
    from src.miaudio import lib as L
    g = torch.Generator(device=cuda).manual_seed(N + H)
    qkv = (torch.randn(B * N, 3 * H * 64, generator=g, device=cuda) * 0.7).to(torch.bfloat16)
    dout = torch.randn(B * N, H * 64, generator=g, device=cuda).to(torch.bfloat16)
    scale = 64 ** -0.5
    lib, s = L.load(), L.stream_ptr()
    nws = int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H))
    res = []
    for saved in (False, True):
        out = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device=cuda)
        lse = torch.empty(B, H, N, device=cuda)
        q8 = torch.empty(B * N, H * 64, dtype=torch.uint8, device=cuda) if mx else None
        s8 = torch.empty(B * N, H * 2, dtype=torch.uint8, device=cuda) if mx else None
        work = torch.full((nws,), 255, dtype=torch.uint8, device=cuda)
        dqkv = torch.empty_like(qkv)
        if saved:
            L.check(lib.mia_attn_fwd_save_q(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(),
                                            q8.data_ptr() if mx else None, s8.data_ptr() if mx else None,
                                            work.data_ptr(), B, N, H, scale, s), "fwd_save_q")
            L.check(lib.mia_attn_bwd_saved_q(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                             dqkv.data_ptr(), work.data_ptr(), B, N, H, scale, s), "bwd_saved_q")
        else:
            if mx:
                L.check(lib.mia_attn_fwd_mx(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), q8.data_ptr(),
                                            s8.data_ptr(), B, N, H, scale, s), "fwd_mx")
            else:
                L.check(lib.mia_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), L.BF16, B, N, H, scale, s),
                        "fwd")
            L.check(lib.mia_attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dqkv.data_ptr(),
                                     work.data_ptr(), L.BF16, B, N, H, scale, s), "bwd")
        torch.cuda.synchronize()
        res.append([out, lse, dqkv] + ([q8, s8] if mx else []))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _err_word(lib, work, B, N, H):
    off = int(lib.mia_attn_bwd_error_offset(B, N, H))
    return int(work[off:off + 4].view(torch.int32).item())


@pytest.mark.parametrize("B,N,H", [(2, 1645, 3), (1, 520, 2), (3, 1000, 2), (1, 2050, 1), (2, 777, 2), (4, 64, 3),
                                   (1, 385, 2)])
def test_attention_bwd_fused_vs_two_pass(cuda, B, N, H):
    """The fused backward (S, dP, dS once per tile; dQ summed over the key blocks by the ordered hand-off)
    against the two-kernel form and float64: both within the bf16 bounds of test_attention_fwd_bwd, the
    fused one bit-identical from call to call (fixed summation order), its error word 0 (every bounded
    hand-off wait matched), nothing written outside dqkv."""
    g = torch.Generator().manual_seed(N * 7 + H)
    qkv = (torch.randn(B, N, 3 * H * 64, generator=g) * 1.5).to(torch.bfloat16)
    dout = torch.randn(B, N, H * 64, generator=g).to(torch.bfloat16)
    q, k, v, o = _attn_ref(qkv, B, N, H)
    o.backward(dout.double().view(B, N, H, 64).permute(0, 2, 1, 3))
    lib, s = L.load(), L.stream_ptr()
    tq, td = qkv.to(cuda), dout.to(cuda)
    out = torch.empty(B, N, H * 64, dtype=torch.bfloat16, device=cuda)
    lse = torch.empty(B, H, N, device=cuda)
    work = torch.full((int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)),), 255, dtype=torch.uint8, device=cuda)
    L.check(lib.mia_attn_fwd_save_q(tq.data_ptr(), out.data_ptr(), lse.data_ptr(), None, None, work.data_ptr(), B, N,
                                    H, 0.125, s), "fwd_save_q")
    res = {}
    for name in ("fused", "fused2", "two"):
        full = torch.full((B * N * 3 * H * 64 + 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        dq = full[:B * N * 3 * H * 64]
        if name == "two":
            L.check(lib.mia_attn_bwd_two_pass(tq.data_ptr(), out.data_ptr(), td.data_ptr(), lse.data_ptr(),
                                              dq.data_ptr(), work.data_ptr(), B, N, H, 0.125, 1, s), "two")
        else:
            L.check(lib.mia_attn_bwd_fused(tq.data_ptr(), out.data_ptr(), td.data_ptr(), lse.data_ptr(),
                                           dq.data_ptr(), work.data_ptr(), B, N, H, 0.125, 1, s), "fused")
            torch.cuda.synchronize()
            assert _err_word(lib, work, B, N, H) == 0
        torch.cuda.synchronize()
        assert torch.isnan(full[-64:].float()).all()
        res[name] = dq.view(B, N, 3, H, 64).clone()
    assert torch.equal(res["fused"], res["fused2"])
    for name in ("fused", "two"):
        d = res[name].permute(2, 0, 3, 1, 4)
        for i, ref in enumerate((q.grad, k.grad, v.grad)):
            assert rel(d[i], ref) < 6e-2, (name, "qkv"[i], rel(d[i], ref))
    # the two forms differ only in summation order (and the f32 path of dS into dQ)
    print(f"fused vs two-pass max rel {rel(res['fused'].float(), res['two'].float()):.3g}")


@pytest.mark.parametrize("B,N,H", [(2, 1645, 3), (1, 300, 2), (3, 1000, 2), (1, 2050, 1), (2, 777, 2), (4, 64, 3),
                                   (1, 128, 2), (1, 129, 1), (1, 385, 2), (2, 37, 1)])
def test_attention_bwd_onepass_vs_two_pass(cuda, B, N, H):
    """The one-pass training backward (mia_attn_bwd_onepass: S, dP, dS once per tile; dQ summed over the 256-key
    blocks by the ordered hand-off of running sums) against float64 and the two-kernel form: within the bf16
    bounds of test_attention_fwd_bwd, bit-identical from call to call (fixed summation order), the sticky
    error word still 0 (every bounded hand-off wait matched), nothing written outside dqkv.  The shapes cover
    two to nine key blocks at rotation lag 3 (with 64-query tiles and 256-key blocks lag 3 always leaves two
    steps between contributions), a single key block (N <= 256, lag 1), ragged tails of both tile sizes."""
    g = torch.Generator().manual_seed(N * 5 + H)
    qkv = (torch.randn(B, N, 3 * H * 64, generator=g) * 1.5).to(torch.bfloat16)
    dout = torch.randn(B, N, H * 64, generator=g).to(torch.bfloat16)
    q, k, v, o = _attn_ref(qkv, B, N, H)
    o.backward(dout.double().view(B, N, H, 64).permute(0, 2, 1, 3))
    lib, s = L.load(), L.stream_ptr()
    tq, td = qkv.to(cuda), dout.to(cuda)
    out = torch.empty(B, N, H * 64, dtype=torch.bfloat16, device=cuda)
    lse = torch.empty(B, H, N, device=cuda)
    saved = torch.full((int(lib.mia_attn_saved_q_bytes(B, N, H)),), 255, dtype=torch.uint8, device=cuda)
    L.check(lib.mia_attn_fwd_save_q(tq.data_ptr(), out.data_ptr(), lse.data_ptr(), None, None, saved.data_ptr(), B, N,
                                    H, 0.125, s), "fwd_save_q")
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    res = {}
    for name in ("one", "one2", "two"):
        full = torch.full((B * N * 3 * H * 64 + 64,), float("nan"), dtype=torch.bfloat16, device=cuda)
        dq = full[:B * N * 3 * H * 64]
        if name == "two":
            L.check(lib.mia_attn_bwd_saved_q(tq.data_ptr(), out.data_ptr(), td.data_ptr(), lse.data_ptr(),
                                             dq.data_ptr(), saved.data_ptr(), B, N, H, 0.125, s), "two")
        else:
            chain = torch.full((int(lib.mia_attn_bwd_chain_bytes(B, N, H)),), 255, dtype=torch.uint8, device=cuda)
            L.check(lib.mia_attn_bwd_onepass(tq.data_ptr(), out.data_ptr(), td.data_ptr(), lse.data_ptr(),
                                             dq.data_ptr(), saved.data_ptr(), chain.data_ptr(), err.data_ptr(), B, N,
                                             H, 0.125, 1, s), "onepass")
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        assert torch.isnan(full[-64:].float()).all()
        res[name] = dq.view(B, N, 3, H, 64).clone()
    assert torch.equal(res["one"], res["one2"])
    for name in ("one", "two"):
        d = res[name].permute(2, 0, 3, 1, 4)
        for i, ref in enumerate((q.grad, k.grad, v.grad)):
            assert rel(d[i], ref) < 6e-2, (name, "qkv"[i], rel(d[i], ref))
    e = rel(res["one"].float(), res["two"].float())
    print(f"one-pass vs two-pass max rel {e:.3g}")
    assert e < 5e-3, e
