"""EnvNet-v2 forward/backward on the MI355X kernels (one autograd node for the whole network).

Data layout in HBM (B = batch):
  x            (B, T) f32 waveform                       — read by conv1 as an NWC view with C=2
  y1 / y2      (B*W1, 32) / (B*W2, 64) raw conv outputs  — channels-last, compute dtype
  X0           (B, 64, 860)  pooled frontend, written transposed (= envnet_v2.py:82 transpose(1,2))
  ya_k / yb_k  (B, H, W, C) raw trunk conv outputs       — NHWC
  p_k          pooled trunk maps (NHWC; the last one NCHW-flat = nn.Flatten order)
  h1, h2       (B, 4096) post-ReLU/dropout FC activations
BatchNorm apply + ReLU is never materialised: it is fused into the next conv's operand loader
(MIA_PRE_AFFINE_RELU) or into the pool kernel.  Backward recomputes it from the raw outputs.
Reference op sequence: src/models/envnet_v2.py:14-85.
"""
from __future__ import annotations

import itertools
import os

import torch

from ..miaudio import kernels as K
from ..miaudio import lib as L

_SEED = itertools.count(0x5EED)
# A/B switch: conv4's backward-data without the fused ReLU+BN backward sums (a separate reduce pass)
C8_BNSEP = os.environ.get("MIA_C8_BNSEP", "0") == "1"
# A/B switch: conv3's ReLU+BN backward as its own pass instead of inside the conv3 weight-gradient kernel
C3_BNSEP = os.environ.get("MIA_C3_BNSEP", "0") == "1"
FC1_CHUNK_ROWS = 256  # rows of FC1's weight gradient per data-parallel all-reduce (256 x 84480 f32 = 86.5 MB)


def _use_conv8(cd: int, cin: int, cout: int, kh: int, kw: int) -> bool:
    """conv4 (32 -> 32, 8x8) forward / backward-data on the row-rolling kernel (csrc/conv8.hip) in
    bf16; the f32 parity path runs the generic row-window implicit GEMM."""
    return cd == L.BF16 and cin == 32 and cout == 32 and kh == 8 and kw == 8

# (conv module path, bn module path, cin, cout, kh, kw)
TRUNK = [
    (("trunk", 0, 0), ("trunk", 0, 1), 1, 32, 8, 8),
    (("trunk", 0, 3), ("trunk", 0, 4), 32, 32, 8, 8),
    (("trunk", 1, 0), ("trunk", 1, 1), 32, 64, 1, 4),
    (("trunk", 1, 3), ("trunk", 1, 4), 64, 64, 1, 4),
    (("trunk", 2, 0), ("trunk", 2, 1), 64, 128, 1, 2),
    (("trunk", 2, 3), ("trunk", 2, 4), 128, 128, 1, 2),
    (("trunk", 3, 0), ("trunk", 3, 1), 128, 256, 1, 2),
    (("trunk", 3, 3), ("trunk", 3, 4), 256, 256, 1, 2),
]
TRUNK_POOL = [(5, 3), (1, 2), (1, 2), (1, 2)]


def geometry(T: int):
    W1 = (T - 64) // 2 + 1
    W2 = (W1 - 16) // 2 + 1
    Wp = W2 // 64
    g = {"T": T, "W1": W1, "W2": W2, "Wp": Wp, "trunk": []}
    H, W = 64, Wp
    for blk in range(4):
        ka = TRUNK[2 * blk]
        ha, wa = H - ka[4] + 1, W - ka[5] + 1
        kb = TRUNK[2 * blk + 1]
        hb, wb = ha - kb[4] + 1, wa - kb[5] + 1
        ph, pw = TRUNK_POOL[blk]
        g["trunk"].append(((H, W), (ha, wa), (hb, wb), (hb // ph, wb // pw)))
        H, W = hb // ph, wb // pw
    g["flat"] = 256 * H * W
    return g


def _frontend_work(B: int, g: dict, tdt: torch.dtype, backward: bool):
    """Algorithmic (FLOP, HBM bytes) of the frontend 1-D conv path (conv1 -> BN -> ReLU -> conv2 -> BN
    -> ReLU -> maxpool), SURVEY.md §8(d): compulsory tensor traffic with X = the f32 waveform,
    S1 / S2 = the conv1 / conv2 outputs, P = the pooled map (compute dtype).
    fwd = X + 2 S1 + 2 S2 + P;  bwd = P + 4 S2 + 4 S1 + X."""
    es = torch.finfo(tdt).bits // 8
    X = g["T"] * 4
    S1 = g["W1"] * 32 * es
    S2 = g["W2"] * 64 * es
    P = 64 * g["Wp"] * es
    flop = 2.0 * (g["W1"] * 32 * 64 + g["W2"] * 64 * 512)  # conv1 + conv2 MACs x 2
    if backward:
        return B * 2 * flop, B * (P + 4 * S2 + 4 * S1 + X)
    return B * flop, B * (X + 2 * S1 + 2 * S2 + P)


def _param_list(m):
    """Flat parameter order handed to the autograd Function (also the grad order)."""
    ps = [m.frontend[0].weight, m.frontend[0].bias, m.frontend[1].weight, m.frontend[1].bias,
          m.frontend[3].weight, m.frontend[3].bias, m.frontend[4].weight, m.frontend[4].bias]
    for blk in range(4):
        seq = m.trunk[blk]
        ps += [seq[0].weight, seq[0].bias, seq[1].weight, seq[1].bias,
               seq[3].weight, seq[3].bias, seq[4].weight, seq[4].bias]
    for idx in (1, 4, 7):
        ps += [m.classifier[idx].weight, m.classifier[idx].bias]
    return ps


def _bns(m):
    out = [m.frontend[1], m.frontend[4]]
    for blk in range(4):
        out += [m.trunk[blk][1], m.trunk[blk][4]]
    return out


class EnvNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, compute: int, *params):
        if not x.is_cuda:
            raise RuntimeError("EnvNetV2 runs on the MI355X HIP kernels only (input is on CPU)")
        B = x.shape[0]
        x = x.reshape(B, -1).contiguous().float()
        T = x.shape[1]
        if T % 2:
            raise ValueError(f"EnvNetV2 expects an even clip length (got {T})")
        g = geometry(T)
        if g["flat"] != model.classifier[1].in_features:
            raise ValueError(f"clip length {T} gives {g['flat']} trunk features, FC1 expects "
                             f"{model.classifier[1].in_features} (envnet_v2.py:51)")
        training = model.training
        cd = compute
        tdt = L.torch_dtype(cd)
        dev = x.device
        bns = _bns(model)
        p = params
        W1, W2, Wp = g["W1"], g["W2"], g["Wp"]
        saved = {"g": g, "B": B, "cd": cd}

        def bn(i, y, P, C):
            mod = bns[i]
            return K.bn_fwd_stats(y, P, C, mod.weight, mod.bias, mod.running_mean, mod.running_var,
                                  mod.momentum if mod.momentum is not None else 0.1, mod.eps, training)

        # every conv weight's forward operand (OHWI, compute dtype) in one launch; kept for the backward's
        # (1, 2)-conv GEMMs, which take the same operand
        wpk = dict(zip([0, 4] + [8 + 8 * b + o for b in range(4) for o in (0, 4)],
                       K.pack_weights([(p[i], cd, 0) for i in [0, 4] + [8 + 8 * b + o for b in range(4) for o in (0, 4)]])))
        saved["wpk"] = wpk
        # ---- frontend conv1: CONVROW over the (B, T/2, 2) view of the waveform
        fe = K.probe("frontend.fwd", *_frontend_work(B, g, tdt, backward=False))
        fe.__enter__()
        w1 = wpk[0]
        y1 = torch.empty(B * W1, 32, dtype=tdt, device=dev)
        if cd == L.BF16:
            # wave-persistent conv1 with the BN1 batch statistics accumulated in its epilogue
            st = K.fe_conv1_fwd(x, w1, p[1], y1, B, T, stats=training, tag="conv1.fwd")
            if training:
                m0 = bns[0]
                bn1 = K.bn_finalize_shifted(st[0], st[1], B * W1, 32, p[1], m0.weight, m0.bias, m0.running_mean,
                                            m0.running_var, m0.momentum if m0.momentum is not None else 0.1, m0.eps)
            else:
                bn1 = bn(0, y1, B * W1, 32)
        else:
            A = K.conv(x, L.KC, B, 1, T // 2, 2, 1, W1, 1, 32, row_kind=True)
            Bo = K.dense(w1, L.KC, 32, 64)
            K.gemm(A, Bo, K.epilogue(y1, 32, bias=p[1]), B * W1, 32, 64, cd, tag="conv1.fwd")
            bn1 = bn(0, y1, B * W1, 32)
        # ---- conv2 (stride 2) with BN1+ReLU fused into the operand load
        w2 = wpk[4]
        y2 = torch.empty(B * W2, 64, dtype=tdt, device=dev)
        if cd == L.BF16:
            K.fe_conv2_fwd(y1, bn1.scale, bn1.shift, w2, p[5], y2, B, W1, W2, tag="conv2.fwd")
        else:
            A = K.conv(y1, L.KC, B, 1, W1, 32, 1, W2, 1, 16, sw=2, pre=L.PRE_AFFINE_RELU, scale=bn1.scale,
                       shift=bn1.shift)
            K.gemm(A, K.dense(w2, L.KC, 64, 512), K.epilogue(y2, 64, bias=p[5]), B * W2, 64, 512, cd,
                   tag="conv2.fwd")
        # ---- maxpool (1,64) of relu(bn2(y2)), written as the transposed trunk image (B, 64, Wp)
        X0 = torch.empty(B, 64, Wp, dtype=tdt, device=dev)
        am0 = torch.empty(B, Wp, 64, dtype=torch.uint8, device=dev)
        if cd == L.BF16 and training:
            # one pass over y2: window winners on the raw values (monotone BN+ReLU) + BN2 statistics,
            # then the pooled relu(bn2(winner)) once the statistics are final
            win0 = torch.empty(B, Wp, 64, dtype=tdt, device=dev)
            part2, nb2 = K.pool_raw_stats(y2, B, 1, W2, 64, 1, 64, p[6], p[5], win0, am0)
            m1 = bns[1]
            bn2 = K.bn_finalize_shifted(part2, nb2, B * W2, 64, p[5], m1.weight, m1.bias, m1.running_mean,
                                        m1.running_var, m1.momentum if m1.momentum is not None else 0.1, m1.eps)
            K.pool_apply(win0, B, 1, Wp, 64, bn2, X0, 1)
        else:
            bn2 = bn(1, y2, B * W2, 64)
            K.pool_fwd(y2, B, 1, W2, 64, 1, 64, bn2, X0, 1, am0)
        fe.__exit__(None, None, None)
        saved.update(x=x, y1=y1, y2=y2, bn1=bn1, bn2=bn2, X0=X0, am0=am0,
                     win0=win0 if cd == L.BF16 and training else None)

        # ---- trunk
        inp = X0
        trunk_saved = []
        for blk in range(4):
            (H, W), (ha, wa), (hb, wb), (hp, wp) = g["trunk"][blk]
            _, _, cin, cout, kh, kw = TRUNK[2 * blk]
            pa = 8 + 8 * blk
            wa_ = wpk[pa]
            ya = torch.empty(B * ha * wa, cout, dtype=tdt, device=dev)
            dense_w2 = cd == L.BF16 and kh == 1 and kw == 2 and cin > 1  # blocks 3-4: (1, 2) convs
            conv3_st = None
            if dense_w2:
                # (1, 2) conv as one dense GEMM over every input pixel (the input map carries a pad pixel)
                K.conv_w2_fwd(inp.reshape(B * H * W, cin), B * H, W, cin, wa_, p[pa + 1], ya, tag=f"t{blk}a.fwd")
            elif cd == L.BF16 and cin == 1 and kh == 8 and kw == 8 and cout == 32 and W % 4 == 0:
                # conv3: wave-persistent, BN statistics accumulated in its epilogue
                conv3_st = K.fe_conv3_fwd(inp, wa_, p[pa + 1], ya, B, H, W, stats=training, tag=f"t{blk}a.fwd")
            else:
                if cin == 1:
                    A = K.conv(inp, L.KC, B, H, W, 1, ha, wa, kh, kw, row_kind=True)
                else:
                    A = K.conv(inp, L.KC, B, H, W, cin, ha, wa, kh, kw)
                K.gemm(A, K.dense(wa_, L.KC, cout, kh * kw * cin), K.epilogue(ya, cout, bias=p[pa + 1]),
                       B * ha * wa, cout, kh * kw * cin, cd, tag=f"t{blk}a.fwd")
            if conv3_st is not None:
                mb = bns[2 + 2 * blk]
                bna = K.bn_finalize_shifted(conv3_st[0], conv3_st[1], B * ha * wa, cout, p[pa + 1], mb.weight, mb.bias,
                                            mb.running_mean, mb.running_var,
                                            mb.momentum if mb.momentum is not None else 0.1, mb.eps)
            else:
                bna = bn(2 + 2 * blk, ya, B * ha * wa, cout)
            _, _, cin2, cout2, kh2, kw2 = TRUNK[2 * blk + 1]
            wb_ = wpk[pa + 4]
            yb = torch.empty(B * hb * wb, cout2, dtype=tdt, device=dev)
            act = None
            conv8_st = None
            conv8 = _use_conv8(cd, cin2, cout2, kh2, kw2)
            if conv8:
                # conv4 (32 -> 32, 8x8): row-rolling MFMA kernel, BN+ReLU on staging, BN stats in its epilogue
                conv8_st = K.trunk_conv8(ya, wb_, yb, B, ha, wa, scale=bna.scale, shift=bna.shift, bias=p[pa + 5],
                                         stats=training, tag=f"t{blk}b.fwd")
            elif dense_w2:
                # relu(bn_a(ya)) materialised once (bf16, + pad pixel): the forward GEMM's A operand and
                # the backward weight-gradient operand
                act = torch.empty(B * ha * wa + 1, cin2, dtype=tdt, device=dev)[: B * ha * wa]
                K.bn_relu_apply(ya, B * ha * wa, cin2, bna, act)
                K.conv_w2_fwd(act, B * ha, wa, cin2, wb_, p[pa + 5], yb, tag=f"t{blk}b.fwd")
            else:
                A = K.conv(ya, L.KC, B, ha, wa, cin2, hb, wb, kh2, kw2, pre=L.PRE_AFFINE_RELU, scale=bna.scale,
                           shift=bna.shift)
                K.gemm(A, K.dense(wb_, L.KC, cout2, kh2 * kw2 * cin2), K.epilogue(yb, cout2, bias=p[pa + 5]),
                       B * hb * wb, cout2, kh2 * kw2 * cin2, cd, tag=f"t{blk}b.fwd")
            if conv8_st is not None:
                mb = bns[3 + 2 * blk]
                bnb = K.bn_finalize_shifted(conv8_st[0], conv8_st[1], B * hb * wb, cout2, p[pa + 5], mb.weight, mb.bias,
                                            mb.running_mean, mb.running_var,
                                            mb.momentum if mb.momentum is not None else 0.1, mb.eps)
            else:
                bnb = bn(3 + 2 * blk, yb, B * hb * wb, cout2)
            ph, pw = TRUNK_POOL[blk]
            last = blk == 3
            # (non-last pools carry one pad pixel: the next block's dense (1, 2)-conv view reads it)
            pooled = torch.empty(B, cout2, hp, wp, dtype=tdt, device=dev) if last else \
                torch.empty(B * hp * wp + 1, cout2, dtype=tdt, device=dev)[: B * hp * wp].view(B, hp, wp, cout2)
            am = torch.empty(B, hp, wp, cout2, dtype=torch.uint8, device=dev)
            win = torch.empty(B, hp, wp, cout2, dtype=tdt, device=dev) if training else None
            K.pool_fwd(yb, B, hb, wb, cout2, ph, pw, bnb, pooled, 2 if last else 0, am, win=win)
            trunk_saved.append(dict(inp=inp, ya=ya, yb=yb, bna=bna, bnb=bnb, am=am, act=act, win=win))
            inp = pooled
        flat = inp.reshape(B, -1)
        saved["trunk"] = trunk_saved
        saved["flat"] = flat

        # ---- classifier (bf16 mode: FC1/FC2 weights cast to bf16 once per step -> LDS-DMA dense GEMM;
        # f32 mode: weights streamed as f32)
        drop_p = model.classifier[3].p if training else 0.0
        h = flat
        hs = []
        wfc = []
        for li, idx in enumerate((1, 4, 7)):
            Wt, bias = p[40 + 2 * li], p[41 + 2 * li]
            fout, fin = Wt.shape
            last = li == 2
            K.wait_param(Wt)  # data-parallel fc1_exchange="shard": the rows the other ranks updated
            if cd == L.BF16 and not last:
                Wt = K.bf16_shadow(Wt)
            wfc.append(Wt)
            out = torch.empty(B, fout, dtype=torch.float32 if last else tdt, device=dev)
            K.gemm(K.dense(h, L.KC, B, fin), K.dense(Wt, L.KC, fout, fin),
                   K.epilogue(out, fout, act=L.ACT_NONE if last else L.ACT_RELU, bias=bias), B, fout, fin, cd,
                   tag=f"fc{li + 1}.fwd")
            if not last and drop_p > 0:
                K.dropout_(out, drop_p, next(_SEED) * 0x9E3779B1)
            hs.append(out)
            h = out
        saved["h1"], saved["h2"] = hs[0], hs[1]
        saved["wfc"] = wfc
        saved["drop_p"] = drop_p
        if getattr(model, "_debug_capture", False):
            model._debug = saved
        ctx.saved = saved
        ctx.model = model
        ctx.params = params
        return hs[2]

    @staticmethod
    def backward(ctx, glogits):
        s = ctx.saved
        p = ctx.params
        g = s["g"]
        B, cd = s["B"], s["cd"]
        tdt = L.torch_dtype(cd)
        dev = glogits.device
        bns = _bns(ctx.model)
        grads = [None] * len(p)
        glogits = glogits.contiguous().float()
        keep_scale = 1.0 / (1.0 - s["drop_p"]) if s["drop_p"] > 0 else 1.0
        ready = getattr(ctx.model, "_grad_ready", None)
        chunk_ready = getattr(ctx.model, "_grad_chunk_ready", None)
        gather = getattr(ctx.model, "_grad_gather", None)

        def emit(lo, hi):
            # hand finished gradients to the data-parallel reducer now (overlaps the rest of the
            # backward); autograd then gets None for them so it does not accumulate twice
            if ready is None:
                return
            ready([(p[i], grads[i]) for i in range(lo, hi)])
            for i in range(lo, hi):
                grads[i] = None

        # ---- classifier backward
        acts = [s["flat"], s["h1"], s["h2"]]
        dcur = glogits
        for li in (2, 1, 0):
            Wt = s["wfc"][li]
            fout, fin = Wt.shape
            hin = acts[li]
            dW = torch.empty(fout, fin, dtype=torch.float32, device=dev) if li > 0 else None
            if (li == 0 and gather is not None and cd == L.BF16 and fout % 128 == 0 and fin % 128 == 0
                    and B % 64 == 0 and gather(p[40], dcur, hin)):
                # data-parallel, gather form (ddp.py): the operands went to the reducer, which defers the
                # averaged gradient over every rank's rows to FusedAdam; nothing to write here
                pass
            elif li == 0 and chunk_ready is not None and fout % FC1_CHUNK_ROWS == 0 and fout > FC1_CHUNK_ROWS:
                dW = torch.empty(fout, fin, dtype=torch.float32, device=dev)
                # data-parallel: FC1's 1.38 GB weight gradient as row chunks of 86.5 MB, each all-reduced
                # as soon as its GEMM is enqueued (the reducer averages it in place; the per-tile sums of
                # squares would describe the un-averaged gradient, so none are written)
                for lo in range(0, fout, FC1_CHUNK_ROWS):
                    part = dW[lo:lo + FC1_CHUNK_ROWS]
                    K.gemm(K.dense(dcur[:, lo:], L.RC, B, FC1_CHUNK_ROWS, ld=fout), K.dense(hin, L.RC, B, fin),
                           K.epilogue(part, fin), FC1_CHUNK_ROWS, fin, B, cd, tag="fc1.wgrad")
                    chunk_ready(p[40], dW, part, lo + FC1_CHUNK_ROWS == fout)
            elif (li == 0 and ready is None and chunk_ready is None and cd == L.BF16 and p[40].grad is None
                  and K.defers_to_fused_adam(p[40]) and fout % 128 == 0 and fin % 128 == 0
                  and B % 64 == 0):
                # single GPU under FusedAdam: FC1's 1.38 GB weight gradient is never written -- its sums
                # of squares now, the product recomputed inside the fused Adam GEMM at the step
                K.defer_weight_grad(p[40], K.dense(dcur, L.RC, B, fout), K.dense(hin, L.RC, B, fin), fout, fin, B,
                                    keep=(dcur, hin), tag="fc1.wgrad")
            else:
                if dW is None:
                    dW = torch.empty(fout, fin, dtype=torch.float32, device=dev)
                # FC1/FC2: the GEMM epilogue also writes per-tile sums of squares of dW, so the clip-norm
                # pass of FusedAdam does not re-read the 1.4 GB (K.sqsum_slots)
                sq = K.sqsum_slots(dW, fout, fin) if li < 2 else None
                K.gemm(K.dense(dcur, L.RC, B, fout), K.dense(hin, L.RC, B, fin), K.epilogue(dW, fin, sqsum=sq), fout,
                       fin, B, cd, tag=f"fc{li + 1}.wgrad")
                if sq is not None:
                    K.tag_sqsum(p[40 + 2 * li], dW, sq)
            grads[40 + 2 * li] = dW
            grads[41 + 2 * li] = K.colsum(dcur, B, fout)
            if li > 0:
                dprev = torch.empty(B, fin, dtype=tdt, device=dev)
                K.gemm(K.dense(dcur, L.KC, B, fout), K.dense(Wt, L.RC, fout, fin),
                       K.epilogue(dprev, fin, act=L.DACT_NZ, aux=hin, ldaux=fin, act_scale=keep_scale),
                       B, fin, fout, cd, tag=f"fc{li + 1}.dgrad")
            else:
                dprev = torch.empty(B, fin, dtype=tdt, device=dev)
                K.gemm(K.dense(dcur, L.KC, B, fout), K.dense(Wt, L.RC, fout, fin), K.epilogue(dprev, fin),
                       B, fin, fout, cd, tag=f"fc{li + 1}.dgrad")
            dcur = dprev
            emit(40 + 2 * li, 42 + 2 * li)

        # ---- trunk backward
        # the flipped / parity / row-split operands the backward-data passes below may take, in one launch
        # (the forward's OHWI packs are reused as they are)
        wpk = s["wpk"]
        bjobs = [(8 + 8 * b + o, 1) for b in range(4) for o in (0, 4)] + [(4, 2)]
        bjobs += [(8 + 8 * b, 3) for b in range(4) if TRUNK[2 * b][2] == 1]
        wbk = dict(zip(bjobs, K.pack_weights([(p[i], cd, m) for i, m in bjobs])))
        dpool = dcur  # (B, 84480) in NCHW-flat order of the last pool
        for blk in (3, 2, 1, 0):
            ts = s["trunk"][blk]
            (H, W), (ha, wa), (hb, wb), (hp, wp) = g["trunk"][blk]
            _, _, cin, cout, kh, kw = TRUNK[2 * blk]
            _, _, cin2, cout2, kh2, kw2 = TRUNK[2 * blk + 1]
            pa = 8 + 8 * blk
            ph, pw = TRUNK_POOL[blk]
            Pb = B * hb * wb
            lay = 2 if blk == 3 else 0
            # reductions gathered at the argmax positions, then one dense pass x -> dy
            gm, dgb, dbb = K.pool_bwd_gather(dpool, lay, ts["am"], ts["yb"], B, hb, wb, cout2, ph, pw, ts["bnb"],
                                             win=ts["win"])
            grads[pa + 6], grads[pa + 7] = dgb, dbb
            dyb = torch.empty(Pb, cout2, dtype=tdt, device=dev)
            dbias_b = torch.empty(cout2, dtype=torch.float32, device=dev)
            K.pool_bn_relu_bwd_apply(gm, ts["am"], ts["yb"], B, hb, wb, cout2, ph, pw, bns[3 + 2 * blk].weight,
                                     ts["bnb"], dgb, dbb, dyb, dbias_b)
            grads[pa + 5] = dbias_b
            # wgrad b: dW[co][(ky,kx,ci)] = sum_pix dyb[pix][co] * relu(bn_a(ya))[pix + tap][ci]
            Kb = kh2 * kw2 * cin2
            dWb = torch.empty(cout2, Kb, dtype=torch.float32, device=dev)
            Pa = B * ha * wa
            da = torch.empty(Pa, cout, dtype=tdt, device=dev)
            red = None  # (dgamma, dbeta) of bn_a when the backward-data kernel formed them
            if ts["act"] is not None:
                # (1, 2) conv: shifted dY once, then wgrad and dgrad as two dense GEMMs
                K.trunk_bwd_w2(dyb, ts["act"], B * ha, wa, cout2, cin2, wpk[pa + 4], dWb, da, wflip=wbk[(pa + 4, 1)],
                               tag=f"t{blk}b")
            else:
                K.gemm(K.dense(dyb, L.RC, Pb, cout2),
                       K.conv(ts["ya"], L.RC, B, ha, wa, cin2, hb, wb, kh2, kw2, pre=L.PRE_AFFINE_RELU,
                              scale=ts["bna"].scale, shift=ts["bna"].shift),
                       K.epilogue(dWb, Kb), cout2, Kb, Pb, cd, tag=f"t{blk}b.wgrad")
                # dgrad b -> grad of relu(bn_a(ya)), then ReLU/BN backward
                wbf = wbk[(pa + 4, 1)]
                Kdb = kh2 * kw2 * cout2
                if _use_conv8(cd, cin2, cout2, kh2, kw2) and not C8_BNSEP:
                    # conv4: the ReLU+BN backward sums of bn_a come out of the backward-data epilogue
                    red = K.trunk_conv8_dgrad_bn(dyb, wbf, da, B, hb, wb, ts["ya"], ts["bna"], tag=f"t{blk}b.dgrad")
                elif _use_conv8(cd, cin2, cout2, kh2, kw2):
                    K.trunk_conv8(dyb, wbf, da, B, hb, wb, ph=kh2 - 1, pw=kw2 - 1, tag=f"t{blk}b.dgrad")
                else:
                    K.gemm(K.conv(dyb, L.KC, B, hb, wb, cout2, ha, wa, kh2, kw2, ph=kh2 - 1, pw=kw2 - 1),
                           K.dense(wbf, L.KC, cin2, Kdb), K.epilogue(da, cin2), Pa, cin2, Kdb, cd,
                           tag=f"t{blk}b.dgrad")
            gwb = torch.empty_like(p[pa + 4])
            K.unpack_ohwi_grad(dWb, p[pa + 4].shape, gwb)
            grads[pa + 4] = gwb
            dga, dba = red if red is not None else K.bn_relu_bwd_reduce(da, None, ts["ya"], Pa, cout, ts["bna"])
            grads[pa + 2], grads[pa + 3] = dga, dba
            dbias_a = torch.empty(cout, dtype=torch.float32, device=dev)
            grads[pa + 1] = dbias_a
            dya = da
            Ka = kh * kw * cin
            dWa = torch.empty(cout, Ka, dtype=torch.float32, device=dev)
            dense_w2 = ts["act"] is not None
            c3w = cin == 1 and cd == L.BF16 and kh == 8 and kw == 8 and cout == 32 and W % 4 == 0
            if c3w and not C3_BNSEP:
                # conv3: the ReLU+BN backward applied while the weight-gradient kernel stages dY (in place)
                K.conv3_wgrad_bn(ts["inp"], da, ts["ya"], da, dWa, dbias_a, B, H, W, bns[2 + 2 * blk].weight,
                                 ts["bna"], dga, dba, tag=f"t{blk}a.wgrad")
            else:
                K.bn_relu_bwd_apply(da, ts["ya"], da, Pa, cout, bns[2 + 2 * blk].weight, ts["bna"], dga, dba,
                                    dbias_a)
            # wgrad a
            if c3w and not C3_BNSEP:
                pass  # formed above
            elif dense_w2:
                dinp = torch.empty(B * H * W, cin, dtype=tdt, device=dev)
                K.trunk_bwd_w2(dya, ts["inp"].reshape(B * H * W, cin), B * H, W, cout, cin, wpk[pa],
                               dWa, dinp, tag=f"t{blk}a", wflip=wbk[(pa, 1)])
            elif c3w:
                # conv3 weight gradient: wave-persistent, dY read once (csrc/conv3w.hip)
                K.conv3_wgrad(ts["inp"], dya, dWa, B, H, W, tag=f"t{blk}a.wgrad")
            else:
                if cin == 1:
                    Bop = K.conv(ts["inp"], L.RC, B, H, W, 1, ha, wa, kh, kw, row_kind=True)
                else:
                    Bop = K.conv(ts["inp"], L.RC, B, H, W, cin, ha, wa, kh, kw)
                K.gemm(K.dense(dya, L.RC, Pa, cout), Bop, K.epilogue(dWa, Ka), cout, Ka, Pa, cd,
                       tag=f"t{blk}a.wgrad")
            gwa = torch.empty_like(p[pa])
            K.unpack_ohwi_grad(dWa, p[pa].shape, gwa)
            grads[pa] = gwa
            # dgrad a -> gradient of the block input (pooled map of the previous stage)
            if dense_w2:
                pass  # computed with the weight gradient above
            elif cin == 1 and cd == L.BF16 and kh == 8 and kw == 8 and cout == 32:
                # 1-channel 8x8 conv: one sweep over dY rows, kernel row ky on the MFMA N side
                dinp = torch.empty(B, H, W, dtype=tdt, device=dev)
                K.conv1ch_dgrad(dya, p[pa], B, ha, wa, dinp, tag=f"t{blk}a.dgrad")
            elif cin == 1:
                # 1-channel 8x8 conv: P[b][r][iw][ky] = sum_{j,co} dya[b][r][iw+j-7][co] W[co][0][ky][7-j]
                wr = wbk[(pa, 3)]
                Pm = torch.empty(B * ha * W, kh, dtype=torch.float32, device=dev)
                K.gemm(K.conv(dya, L.KC, B, ha, wa, cout, ha, W, 1, kw, pw=kw - 1),
                       K.dense(wr, L.KC, kh, kw * cout), K.epilogue(Pm, kh), B * ha * W, kh, kw * cout, cd,
                       tag=f"t{blk}a.dgrad")
                dinp = torch.empty(B, H, W, dtype=tdt, device=dev)
                K.col2im_rows(Pm, B, ha, W, kh, dinp)
            else:
                waf = wbk[(pa, 1)]
                dinp = torch.empty(B * H * W, cin, dtype=tdt, device=dev)
                Kda = kh * kw * cout
                K.gemm(K.conv(dya, L.KC, B, ha, wa, cout, H, W, kh, kw, ph=kh - 1, pw=kw - 1),
                       K.dense(waf, L.KC, cin, Kda), K.epilogue(dinp, cin), B * H * W, cin, Kda, cd,
                       tag=f"t{blk}a.dgrad")
            dpool = dinp
            emit(pa, pa + 8)

        # ---- frontend backward
        fe = K.probe("frontend.bwd", *_frontend_work(B, g, tdt, backward=True))
        fe.__enter__()
        W1, W2, Wp = g["W1"], g["W2"], g["Wp"]
        P2, P1 = B * W2, B * W1
        gm, dg2, db2 = K.pool_bwd_gather(dpool, 1, s["am0"], s["y2"], B, 1, W2, 64, 1, 64, s["bn2"], win=s["win0"])
        grads[6], grads[7] = dg2, db2
        dy2 = torch.empty(P2, 64, dtype=tdt, device=dev)
        dbias2 = torch.empty(64, dtype=torch.float32, device=dev)
        K.pool_bn_relu_bwd_apply(gm, s["am0"], s["y2"], B, 1, W2, 64, 1, 64, bns[1].weight, s["bn2"], dg2, db2, dy2,
                                 dbias2)
        grads[5] = dbias2
        dW2 = torch.empty(64, 512, dtype=torch.float32, device=dev)
        if cd == L.BF16:
            K.fe_conv2_wgrad(dy2, s["y1"], s["bn1"].scale, s["bn1"].shift, dW2, B, W1, W2, tag="conv2.wgrad")
        else:
            K.gemm(K.dense(dy2, L.RC, P2, 64),
                   K.conv(s["y1"], L.RC, B, 1, W1, 32, 1, W2, 1, 16, sw=2, pre=L.PRE_AFFINE_RELU,
                          scale=s["bn1"].scale, shift=s["bn1"].shift),
                   K.epilogue(dW2, 512), 64, 512, P2, cd, tag="conv2.wgrad")
        gw2 = torch.empty_like(p[4])
        K.unpack_ohwi_grad(dW2, p[4].shape, gw2)
        grads[4] = gw2
        # stride-2 dgrad as two stride-1 parity convolutions
        wpar = wbk[(4, 2)]
        da1 = torch.empty(P1, 32, dtype=tdt, device=dev)
        if cd == L.BF16:
            K.fe_conv2_dgrad(dy2, wpar, da1, B, W1, W2, tag="conv2.dgrad")
        else:
            wpar = wpar.view(2, 32 * 8 * 64)
            for par in (0, 1):
                Tp = (W1 - par + 1) // 2
                K.gemm(K.conv(dy2, L.KC, B, 1, W2, 64, 1, Tp, 1, 8, pw=7),
                       K.dense(wpar[par], L.KC, 32, 512),
                       K.epilogue(da1, 32, rowmap=(Tp, W1, 2, par)), B * Tp, 32, 512, cd, tag="conv2.dgrad")
        dbias1 = torch.empty(32, dtype=torch.float32, device=dev)
        dW1 = torch.empty(32, 64, dtype=torch.float32, device=dev)
        T = g["T"]
        if cd == L.BF16:
            # BN1+ReLU backward and conv1 weight gradient in one pass (linear form): dS1 is never
            # formed, the BN reductions come out of the same read of da1 / y1
            dg1, db1 = K.fe_conv1_wgrad_bn(s["x"], da1, s["y1"], B, T, bns[0].weight, s["bn1"], dW1, dbias1,
                                           tag="conv1.wgrad")
            grads[2], grads[3] = dg1, db1
        else:
            dg1, db1 = K.bn_relu_bwd_reduce(da1, None, s["y1"], P1, 32, s["bn1"])
            grads[2], grads[3] = dg1, db1
            K.bn_relu_bwd_apply(da1, s["y1"], da1, P1, 32, bns[0].weight, s["bn1"], dg1, db1, dbias1)
            K.gemm(K.dense(da1, L.RC, P1, 32), K.conv(s["x"], L.RC, B, 1, T // 2, 2, 1, W1, 1, 32, row_kind=True),
                   K.epilogue(dW1, 64), 32, 64, P1, cd, tag="conv1.wgrad")
        grads[1] = dbias1
        grads[0] = dW1.view_as(p[0])
        fe.__exit__(None, None, None)
        emit(0, 8)
        ctx.saved = None
        return (None, None, None, *grads)


def envnet_forward(model, x, compute: int):
    return EnvNetFunction.apply(model, x, compute, *_param_list(model))
