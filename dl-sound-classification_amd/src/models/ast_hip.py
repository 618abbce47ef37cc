"""AST forward/backward on the MI355X kernels (one autograd node for the whole transformer).

Reference op sequence: src/models/ast.py:50-63 + timm 1.0.16 Block (pre-LN, qkv Linear with bias,
SDPA, proj, LN, fc1, exact-erf GELU, fc2), LN eps 1e-6, sigmoid head on the CLS token.
HBM layout per block (T = B*1645 tokens, D = 768): residual stream x (T, 768) f32; LN outputs,
qkv (T, 3, 12, 64), attention output (T, 12, 64) and fc1 pre-activation (T, 3072) in the compute
dtype.  fc1's epilogue writes both gelu(u) (fc2's operand) and the derivative gelu'(u)
(MIA_ACT_GELU_SAVE_D; u itself has no other reader); the fc1 backward multiplies it in the epilogue of
the fc2 dgrad GEMM (MIA_DACT_MUL); residual adds are GEMM epilogues (MIA_ACT_ADD_AUX / accumulate).  In bf16 mode the
linear weights are cast to bf16 once per step and every GEMM operand is bf16, so the projections run
on the LDS-DMA dense kernel (mia_gemm path 5).
"""
from __future__ import annotations

import os

import torch

from ..miaudio import kernels as K
from ..miaudio import lib as L

EPS = 1e-6


def _ln(x, g, b, out_dtype, rows, D, mx: bool = False):
    """LayerNorm forward -> (y, mean, rstd[, MX-fp8 copy of y when mx: mia_layernorm_fwd_mx])."""
    y = torch.empty(rows, D, dtype=out_dtype, device=x.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    if mx:
        yq = K.mx_empty(rows, D, x.device)
        L.check(L.load().mia_layernorm_fwd_mx(x.data_ptr(), L.dtype_code(x), g.data_ptr(), b.data_ptr(), y.data_ptr(),
                                              yq.q.data_ptr(), yq.scales.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                              rows, D, EPS, L.stream_ptr()), "mia_layernorm_fwd_mx")
        return y, mean, rstd, yq
    L.check(L.load().mia_layernorm_fwd(x.data_ptr(), L.dtype_code(x), g.data_ptr(), b.data_ptr(), y.data_ptr(),
                                       L.dtype_code(y), mean.data_ptr(), rstd.data_ptr(), rows, D, EPS, L.stream_ptr()),
            "mia_layernorm_fwd")
    return y, mean, rstd, None


def _ln_bwd(dy, x, g, mean, rstd, dx, rows, D, accumulate: bool, dx2=None, dx2_mx=None):
    """LayerNorm backward into dx (optionally accumulating); dx2 receives a second copy of the result
    (the bf16 operand of the next linear backward).  Returns (dgamma, dbeta, colsum(dx2) or None): with
    dx2 the column sums of its stored values -- the next linear's bias gradient -- come from the same
    pass (mia_layernorm_bwd_colsum).  dx2_mx (fp8-mixed): an MXTensor receiving the MX-fp8 copy of the
    stored bf16 dx2 (mia_layernorm_bwd_colsum_mx), the next MX backward-data GEMM's A operand."""
    dg = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty(D, dtype=torch.float32, device=x.device)
    lib = L.load()
    ws = K.workspace(lib.mia_layernorm_partial_bytes(rows, D), x.device, "ln")
    if dx2_mx is not None:
        cs = torch.empty(D, dtype=torch.float32, device=x.device)
        L.check(lib.mia_layernorm_bwd_colsum_mx(dy.data_ptr(), L.dtype_code(dy), x.data_ptr(), L.dtype_code(x),
                                                g.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                                L.dtype_code(dx), int(accumulate), dx2.data_ptr(), dg.data_ptr(),
                                                db.data_ptr(), cs.data_ptr(), dx2_mx.q.data_ptr(),
                                                dx2_mx.scales.data_ptr(), ws.data_ptr(), rows, D, L.stream_ptr()),
                "mia_layernorm_bwd_colsum_mx")
        return dg, db, cs
    if dx2 is not None and D == 768:
        cs = torch.empty(D, dtype=torch.float32, device=x.device)
        L.check(lib.mia_layernorm_bwd_colsum(dy.data_ptr(), L.dtype_code(dy), x.data_ptr(), L.dtype_code(x),
                                             g.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                             L.dtype_code(dx), int(accumulate), dx2.data_ptr(), L.dtype_code(dx2),
                                             dg.data_ptr(), db.data_ptr(), cs.data_ptr(), ws.data_ptr(), rows, D,
                                             L.stream_ptr()), "mia_layernorm_bwd_colsum")
        return dg, db, cs
    L.check(lib.mia_layernorm_bwd(dy.data_ptr(), L.dtype_code(dy), x.data_ptr(), L.dtype_code(x), g.data_ptr(),
                                  mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), L.dtype_code(dx), int(accumulate),
                                  L.ptr(dx2), L.dtype_code(dx2) if dx2 is not None else 0, dg.data_ptr(),
                                  db.data_ptr(), ws.data_ptr(), rows, D, L.stream_ptr()),
            "mia_layernorm_bwd")
    return dg, db, None


def _linear(x, W, bias, out, M, cd, act=L.ACT_NONE, aux=None, pre=L.PRE_NONE, tag=None):
    """out[M, N] = act(x[M, K] @ W[N, K]^T + bias)"""
    Nf, Kf = W.shape
    K.gemm(K.dense(x, L.KC, M, Kf, pre=pre), K.dense(W, L.KC, Nf, Kf),
           K.epilogue(out, Nf, act=act, bias=bias, aux=aux, ldaux=Nf), M, Nf, Kf, cd, tag=tag)


ATTN_SAVE_Q = True  # bf16 training: the attention forward writes Q' for the backward (mia_attn_fwd_save_q)
# bf16 training backward: the two-kernel form (mia_attn_bwd_saved_q: dK/dV pass + dQ pass, S / dP recomputed
# in the second) or the one-pass kernel (mia_attn_bwd_onepass, no recompute).  Measured at the benched grid
# (B 256, N 1645, H 12; tools/bench_attn_bwd.py, gpurun_out r5i): two-pass 7.3 ms, one-pass 8.1-8.2 ms per
# layer, so the two-pass form is the default; tools and tests flip this for A/B runs
ATTN_ONEPASS = False
# fp8-mixed: the backward-data GEMMs that run on MX-fp8 operands (dy quantised per call, W^T from the f32 master);
# the weight gradients stay bf16.  MIA_MX_DGRAD="" keeps every backward GEMM in bf16 (A/B switch).
MX_DGRAD = frozenset(t for t in os.environ.get("MIA_MX_DGRAD", "fc2,fc1,proj").split(",") if t)


def _linear_bwd(dy, x, W, M, cd, dx_out=None, dact=None, dact_aux=None, x_pre=L.PRE_NONE, tag="", db=None,
                dx_colsum=None, wt_mx=None, dy_mx=None, dx_mx=None):
    """dW = dy^T x (f32), db = colsum(dy) (unless the producer of dy already summed it), dx = dy @ W
    (optionally with an activation backward; dx_colsum receives dx's column sums, the next linear's
    bias gradient).  wt_mx (fp8-mixed): the MX copy of W^T -- the backward-data GEMM then runs on MX-fp8
    operands: dy_mx, the MX copy of dy its producer wrote (quantised here when None); dx_mx receives the MX
    copy of the stored dx (the next MX backward-data GEMM's A operand).  The weight gradient stays bf16."""
    Nf, Kf = W.shape
    if cd == L.BF16 and dy.dtype == torch.float32:
        dy = K.cast(dy, torch.bfloat16)  # bf16 GEMM operands (f32 accumulation inside)
    dW = torch.empty(Nf, Kf, dtype=torch.float32, device=dy.device)
    a_cs = None
    if db is None:  # the weight-gradient GEMM sums dy's columns from the A tiles it reads
        db = a_cs = torch.empty(Nf, dtype=torch.float32, device=dy.device)
    K.gemm(K.dense(dy, L.RC, M, Nf), K.dense(x, L.RC, M, Kf, pre=x_pre), K.epilogue(dW, Kf, a_colsum=a_cs),
           Nf, Kf, M, cd, tag=tag + ".wgrad")
    if dx_out is not None and wt_mx is not None:
        K.gemm_mxfp8(dy_mx if dy_mx is not None else K.mx_quantize(dy), wt_mx,
                     K.epilogue(dx_out, Kf, act=dact if dact is not None else L.ACT_NONE, aux=dact_aux, ldaux=Kf,
                                colsum=dx_colsum, mx=dx_mx), tag=tag + ".dgrad")
    elif dx_out is not None:
        K.gemm(K.dense(dy, L.KC, M, Nf), K.dense(W, L.RC, Nf, Kf),
               K.epilogue(dx_out, Kf, act=dact if dact is not None else L.ACT_NONE, aux=dact_aux, ldaux=Kf,
                          colsum=dx_colsum),
               M, Kf, Nf, cd, tag=tag + ".dgrad")
    return dW, db


class ASTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, spec, compute: int, grad: bool, *params):
        if not spec.is_cuda:
            raise RuntimeError("ASTModel runs on the MI355X HIP kernels only (input is on CPU)")
        mx = compute == L.MXFP8  # fp8-mixed: block linears' forward GEMMs on MX-fp8 operands
        cd = L.BF16 if mx else compute
        tdt = L.torch_dtype(cd)
        dev = spec.device
        B, Fm, Tf = spec.shape
        spec = spec.contiguous().float()
        D, Hh = model.emb_dim, model.num_heads
        ps, st = model.patch_size, model.patch_stride
        gh, gw = (Fm - ps) // st + 1, (Tf - ps) // st + 1
        Np = gh * gw
        N = Np + 1
        if N > model.pos_embed.shape[1]:
            raise ValueError(f"{N} tokens exceed the positional table ({model.pos_embed.shape[1]})")
        Tt = B * N
        pw, pb, cls, pos = params[0], params[1], params[2], params[3]
        # patch embedding: Conv2d(1, D, 16, stride 10).  bf16: the patch matrix in token order (zero cls
        # rows, mia_ast_patches) through the dense 256x256 GEMM straight into the token rows of x, then the
        # cls / positional rows in place; f32 (or a patch size that is not a multiple of 8, which the patch
        # matrix kernel cannot take): an implicit GEMM over the spectrogram
        x = torch.empty(Tt, D, dtype=torch.float32, device=dev)
        pmat = None
        if cd == L.BF16 and ps % 8 == 0:
            pmat = torch.empty(Tt, ps * ps, dtype=torch.bfloat16, device=dev)
            L.check(L.load().mia_ast_patches(spec.data_ptr(), B, Fm, Tf, ps, st, pmat.data_ptr(), L.stream_ptr()),
                    "mia_ast_patches")
            K.gemm(K.dense(pmat, L.KC, Tt, ps * ps), K.dense(K.bf16_shadow(pw).reshape(D, -1), L.KC, D, ps * ps),
                   K.epilogue(x, D, bias=pb), Tt, D, ps * ps, cd, tag="patch.fwd")
            L.check(L.load().mia_tokens_fwd_inplace(x.data_ptr(), cls.data_ptr(), pos.data_ptr(), B, N, D,
                                                    L.stream_ptr()), "mia_tokens_fwd_inplace")
        else:
            patches = torch.empty(B * Np, D, dtype=torch.float32, device=dev)
            K.gemm(K.conv(spec, L.KC, B, Fm, Tf, 1, gh, gw, ps, ps, sh=st, sw=st, row_kind=True),
                   K.dense(pw.reshape(D, -1), L.KC, D, ps * ps), K.epilogue(patches, D, bias=pb), B * Np, D, ps * ps,
                   cd, tag="patch.fwd")
            L.check(L.load().mia_tokens_fwd(patches.data_ptr(), cls.data_ptr(), pos.data_ptr(), x.data_ptr(), B, Np,
                                            D, L.stream_ptr()), "mia_tokens_fwd")
        saved_blocks = []
        nb = len(model.transformer)
        scale = (D // Hh) ** -0.5
        wcast = []
        for i in range(nb):
            g1, b1, wqkv, bqkv, wproj, bproj, g2, b2, w1, bb1, w2, bb2 = params[4 + 12 * i: 16 + 12 * i]
            wmx = [K.mx_quantize(w) for w in (wqkv, wproj, w1, w2)] if mx else None  # from the f32 masters
            if cd == L.BF16:
                wqkv, wproj, w1, w2 = (K.bf16_shadow(w) for w in (wqkv, wproj, w1, w2))
            wcast.append((wqkv, wproj, w1, w2))

            def lin(xin, xq, wi, W, bias, out, tag, **kw):
                """x W^T + bias (+ epilogue); fp8-mixed: on the MX copy xq the producer wrote beside the
                bf16 activation (which the backward keeps using)."""
                if mx:
                    K.gemm_mxfp8(xq, wmx[wi], K.epilogue(out, W.shape[0], bias=bias, ldaux=W.shape[0], **kw), tag=tag)
                else:
                    kw.pop("mx", None)
                    _linear(xin, W, bias, out, Tt, cd, tag=tag, **kw)

            h, m1, r1, hq = _ln(x, g1, b1, tdt, Tt, D, mx=mx)
            qkv = torch.empty(Tt, 3 * D, dtype=tdt, device=dev)
            lin(h, hq, 0, wqkv, bqkv, qkv, "qkv.fwd")
            a = torch.empty(Tt, D, dtype=tdt, device=dev)
            aq = K.mx_empty(Tt, D, dev) if mx else None
            lse = torch.empty(B, Hh, N, dtype=torch.float32, device=dev)
            # bf16 training: the forward also writes Q' (the scaled query operand) into the backward's
            # attention workspace, so the backward's prep pass neither re-reads q nor rewrites Q'
            aw = None
            if cd == L.BF16 and ATTN_SAVE_Q and grad:
                # Q' + the row-constant fragments only (what the two-kernel backward reads); the one-pass
                # backward's running dQ sums are the backward's own transient workspace
                aw = torch.empty(int(L.load().mia_attn_saved_q_bytes(B, N, Hh)), dtype=torch.uint8, device=dev)
            with K.probe("attn.fwd", 4.0 * B * Hh * N * N * (D // Hh), (qkv.numel() + a.numel()) * qkv.element_size()):
                if aw is not None:
                    L.check(L.load().mia_attn_fwd_save_q(qkv.data_ptr(), a.data_ptr(), lse.data_ptr(),
                                                         aq.q.data_ptr() if mx else None,
                                                         aq.scales.data_ptr() if mx else None, aw.data_ptr(), B, N,
                                                         Hh, scale, L.stream_ptr()), "mia_attn_fwd_save_q")
                elif mx:
                    L.check(L.load().mia_attn_fwd_mx(qkv.data_ptr(), a.data_ptr(), lse.data_ptr(), aq.q.data_ptr(),
                                                     aq.scales.data_ptr(), B, N, Hh, scale, L.stream_ptr()),
                            "mia_attn_fwd_mx")
                else:
                    L.check(L.load().mia_attn_fwd(qkv.data_ptr(), a.data_ptr(), lse.data_ptr(), cd, B, N, Hh, scale,
                                                  L.stream_ptr()), "mia_attn_fwd")
            xm = torch.empty(Tt, D, dtype=torch.float32, device=dev)
            lin(a, aq, 1, wproj, bproj, xm, "proj.fwd", act=L.ACT_ADD_AUX, aux=x)
            h2, m2, r2, h2q = _ln(xm, g2, b2, tdt, Tt, D, mx=mx)
            gd = torch.empty(Tt, w1.shape[0], dtype=tdt, device=dev)  # gelu'(u), u = fc1's pre-activation
            gu = torch.empty(Tt, w1.shape[0], dtype=tdt, device=dev)  # gelu(u)
            guq = K.mx_empty(Tt, w1.shape[0], dev) if mx else None
            lin(h2, h2q, 2, w1, bb1, gu, "fc1.fwd", act=L.ACT_GELU_SAVE_D, aux=gd, mx=guq)
            xo = torch.empty(Tt, D, dtype=torch.float32, device=dev)
            lin(gu, guq, 3, w2, bb2, xo, "fc2.fwd", act=L.ACT_ADD_AUX, aux=xm)
            del hq, aq, h2q, guq
            saved_blocks.append(dict(x=x, m1=m1, r1=r1, h=h, qkv=qkv, a=a, lse=lse, xm=xm, m2=m2, r2=r2, h2=h2, gd=gd,
                                     gu=gu, attn_work=aw))
            x = xo
        # final norm only matters for the CLS rows (ast.py:62-63 takes x[:, 0])
        gn, bn_, wh, bh = params[4 + 12 * nb: 8 + 12 * nb]
        xc = x.view(B, N, D)[:, 0].contiguous()
        hc, mc, rc, _ = _ln(xc, gn, bn_, torch.float32, B, D)
        z = torch.empty(B, wh.shape[0], dtype=torch.float32, device=dev)
        _linear(hc, wh, bh, z, B, cd, tag="head.fwd")
        probs = torch.sigmoid(z)
        ctx.s = dict(B=B, N=N, Np=Np, D=D, H=Hh, cd=cd, mx=mx, spec=spec if pmat is None else None, pmat=pmat, gh=gh, gw=gw, blocks=saved_blocks, xc=xc, wcast=wcast,
                     mc=mc, rc=rc, hc=hc, probs=probs, scale=scale)
        ctx.model = model
        ctx.params = params
        return probs

    @staticmethod
    def backward(ctx, dprobs):
        s, p, model = ctx.s, ctx.params, ctx.model
        B, N, Np, D, Hh, cd = s["B"], s["N"], s["Np"], s["D"], s["H"], s["cd"]
        tdt = L.torch_dtype(cd)
        dev = dprobs.device
        Tt = B * N
        nb = len(model.transformer)
        grads = [None] * len(p)
        ready = getattr(model, "_grad_ready", None)

        def emit(lo, hi):
            if ready is None:
                return
            ready([(p[i], grads[i]) for i in range(lo, hi)])
            for i in range(lo, hi):
                grads[i] = None

        pr = s["probs"]
        dz = (dprobs.float() * pr * (1.0 - pr)).contiguous()  # sigmoid backward (B x classes)
        gn, bn_, wh, bh = p[4 + 12 * nb: 8 + 12 * nb]
        dhc = torch.empty(B, D, dtype=torch.float32, device=dev)
        dWh, dbh = _linear_bwd(dz, s["hc"], wh, B, cd, dx_out=dhc, tag="head")
        dxc = torch.empty(B, D, dtype=torch.float32, device=dev)
        dgn, dbn, _ = _ln_bwd(dhc, s["xc"], gn, s["mc"], s["rc"], dxc, B, D, False)
        grads[4 + 12 * nb: 8 + 12 * nb] = [dgn, dbn, dWh, dbh]
        emit(4 + 12 * nb, 8 + 12 * nb)
        dx = torch.zeros(Tt, D, dtype=torch.float32, device=dev)
        dx.view(B, N, D)[:, 0] = dxc
        # bf16 mode: a bf16 copy of the residual gradient feeds the next linear backward's GEMMs
        if cd == L.BF16:  # only the cls rows are non-zero: a fill, not a cast pass over the whole f32 tensor
            dxb = torch.zeros(Tt, D, dtype=torch.bfloat16, device=dev)
            dxb.view(B, N, D)[:, 0] = dxc.to(torch.bfloat16)
        else:
            dxb = dx
        dxb2 = torch.empty_like(dxb) if cd == L.BF16 else None
        db_next = None  # column sums of dxb from the LayerNorm backward that wrote it (bf16 mode)
        # fp8-mixed: MX copies of dxb written by the LayerNorm backwards (the first one quantised here)
        use_mx = s["mx"] and ("fc2" in MX_DGRAD or "proj" in MX_DGRAD)
        dxb_mx = None
        if use_mx and "fc2" in MX_DGRAD:
            # = mx_quantize(dxb) byte for byte: all-zero blocks are zero bytes with scale byte 0, and only the
            # cls rows of dxb are non-zero
            dxb_mx = K.mx_empty(Tt, D, dev)
            dxb_mx.q.zero_()
            dxb_mx.scales.zero_()
            cq = K.mx_quantize(dxb.view(B, N, D)[:, 0])
            dxb_mx.q.view(B, N, D)[:, 0] = cq.q
            dxb_mx.scales.view(B, N, D // 32)[:, 0] = cq.scales
        dxb2_mx = K.mx_empty(Tt, D, dev) if use_mx else None
        for i in reversed(range(nb)):
            sb = s["blocks"][i]
            g1, b1, wqkv, bqkv, wproj, bproj, g2, b2, w1, bb1, w2, bb2 = p[4 + 12 * i: 16 + 12 * i]
            wt = {}
            if s["mx"]:  # MX copies of W^T for the fp8 backward-data GEMMs, from the f32 masters
                wt = {t: K.mx_quantize_t(w) for t, w in (("qkv", wqkv), ("proj", wproj), ("fc1", w1), ("fc2", w2))
                      if t in MX_DGRAD}
            wqkv, wproj, w1, w2 = s["wcast"][i]
            # fc2 (input gelu(u)) and fc1 with gelu' fused into the dgrad epilogue
            du = torch.empty(Tt, w1.shape[0], dtype=tdt, device=dev)
            du_mx = K.mx_empty(Tt, w1.shape[0], dev) if "fc2" in wt and "fc1" in wt else None
            db1_ = torch.empty(w1.shape[0], dtype=torch.float32, device=dev)  # fc1 bias grad = colsum(du)
            dW2, db2_ = _linear_bwd(dxb, sb["gu"], w2, Tt, cd, dx_out=du, dact=L.DACT_MUL, dact_aux=sb["gd"],
                                    tag="fc2", db=db_next, dx_colsum=db1_, wt_mx=wt.get("fc2"), dy_mx=dxb_mx,
                                    dx_mx=du_mx)
            dh2 = torch.empty(Tt, D, dtype=tdt, device=dev)
            dW1, db1_ = _linear_bwd(du, sb["h2"], w1, Tt, cd, dx_out=dh2, tag="fc1", db=db1_, wt_mx=wt.get("fc1"),
                                    dy_mx=du_mx)
            del du_mx
            dg2, dbt2, db_proj = _ln_bwd(dh2, sb["xm"], g2, sb["m2"], sb["r2"], dx, Tt, D, True, dx2=dxb2,
                                         dx2_mx=dxb2_mx)  # d(xm)
            if dxb2 is not None:
                dxb, dxb2 = dxb2, dxb
                dxb_mx, dxb2_mx = dxb2_mx, dxb_mx
            else:
                dxb = dx
            da = torch.empty(Tt, D, dtype=tdt, device=dev)
            dWp, dbp = _linear_bwd(dxb, sb["a"], wproj, Tt, cd, dx_out=da, tag="proj", db=db_proj, wt_mx=wt.get("proj"),
                                   dy_mx=dxb_mx)
            dqkv = torch.empty(Tt, 3 * D, dtype=tdt, device=dev)
            work = sb["attn_work"]
            with K.probe("attn.bwd", 8.0 * B * Hh * N * N * (D // Hh),  # 2x fwd, recompute not credited
                         (2 * dqkv.numel() + 2 * da.numel()) * dqkv.element_size()):
                if work is not None and ATTN_ONEPASS:  # Q' already written by the forward
                    chain = torch.empty(int(L.load().mia_attn_bwd_chain_bytes(B, N, Hh)), dtype=torch.uint8, device=dev)
                    L.check(L.load().mia_attn_bwd_onepass(sb["qkv"].data_ptr(), sb["a"].data_ptr(), da.data_ptr(),
                                                          sb["lse"].data_ptr(), dqkv.data_ptr(), work.data_ptr(),
                                                          chain.data_ptr(), K.attn_err_word(dev).data_ptr(), B, N, Hh,
                                                          s["scale"], 1, L.stream_ptr()), "mia_attn_bwd_onepass")
                    del chain
                elif work is not None:
                    L.check(L.load().mia_attn_bwd_saved_q(sb["qkv"].data_ptr(), sb["a"].data_ptr(), da.data_ptr(),
                                                          sb["lse"].data_ptr(), dqkv.data_ptr(), work.data_ptr(), B, N,
                                                          Hh, s["scale"], L.stream_ptr()), "mia_attn_bwd_saved_q")
                else:
                    work = torch.empty(int(L.load().mia_attn_bwd_workspace_bytes(cd, B, N, Hh)), dtype=torch.uint8,
                                       device=dev)
                    L.check(L.load().mia_attn_bwd(sb["qkv"].data_ptr(), sb["a"].data_ptr(), da.data_ptr(),
                                                  sb["lse"].data_ptr(), dqkv.data_ptr(), work.data_ptr(), cd, B, N, Hh,
                                                  s["scale"], L.stream_ptr()), "mia_attn_bwd")
            dh = torch.empty(Tt, D, dtype=tdt, device=dev)
            dWq, dbq = _linear_bwd(dqkv, sb["h"], wqkv, Tt, cd, dx_out=dh, tag="qkv", wt_mx=wt.get("qkv"))
            if use_mx and dxb2_mx is None:
                dxb2_mx = K.mx_empty(Tt, D, dev)
            dg1, dbt1, db_next = _ln_bwd(dh, sb["x"], g1, sb["m1"], sb["r1"], dx, Tt, D, True, dx2=dxb2,
                                         dx2_mx=dxb2_mx)  # d(block in)
            if dxb2 is not None:
                dxb, dxb2 = dxb2, dxb
                dxb_mx, dxb2_mx = dxb2_mx, dxb_mx
            else:
                dxb = dx
            grads[4 + 12 * i: 16 + 12 * i] = [dg1, dbt1, dWq, dbq, dWp, dbp, dg2, dbt2, dW1, db1_, dW2, db2_]
            emit(4 + 12 * i, 16 + 12 * i)
            s["blocks"][i] = None
        # tokens: dcls, dpos (first N rows of the table), dpatches
        pos = p[3]
        dpos = torch.zeros_like(pos)
        dcls = torch.empty(1, 1, D, dtype=torch.float32, device=dev)
        pw = p[0]
        ps, st = model.patch_size, model.patch_stride
        dWpe = torch.empty(D, ps * ps, dtype=torch.float32, device=dev)
        if s["pmat"] is not None:
            # bf16: dW = dx^T P over all token rows (the zero cls rows of P add nothing), on the bf16 copy of
            # dx the last LayerNorm backward wrote; the bias gradient = the patch rows of dpos summed
            L.check(L.load().mia_tokens_bwd(dx.data_ptr(), None, dcls.data_ptr(), dpos.data_ptr(), B, Np, D,
                                            L.stream_ptr()), "mia_tokens_bwd")
            K.gemm(K.dense(dxb, L.RC, Tt, D), K.dense(s["pmat"], L.RC, Tt, ps * ps), K.epilogue(dWpe, ps * ps), D,
                   ps * ps, Tt, cd, tag="patch.wgrad")
            grads[1] = K.colsum(dpos.view(-1, D)[1:N], Np, D)
        else:
            dpatch = torch.empty(B * Np, D, dtype=torch.float32, device=dev)
            L.check(L.load().mia_tokens_bwd(dx.data_ptr(), dpatch.data_ptr(), dcls.data_ptr(), dpos.data_ptr(), B,
                                            Np, D, L.stream_ptr()), "mia_tokens_bwd")
            spec = s["spec"]
            Fm, Tf = spec.shape[1], spec.shape[2]
            K.gemm(K.dense(dpatch, L.RC, B * Np, D),
                   K.conv(spec, L.RC, B, Fm, Tf, 1, s["gh"], s["gw"], ps, ps, sh=st, sw=st, row_kind=True),
                   K.epilogue(dWpe, ps * ps), D, ps * ps, B * Np, cd, tag="patch.wgrad")
            grads[1] = K.colsum(dpatch, B * Np, D)
        grads[0] = dWpe.view_as(pw)
        grads[2] = dcls
        grads[3] = dpos
        emit(0, 4)
        ctx.s = None
        return (None, None, None, None, *grads)
