"""Tensor-level wrappers over the C ABI (one function per kernel family).

Every call enqueues on ``torch.cuda.current_stream()``; torch allocates all memory (outputs and
workspaces).  Shapes are validated here, geometry is validated again in the library.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import os

import torch

from . import lib as L

_WS: dict = {}


def workspace(nbytes: int, device, slot: str = "main") -> torch.Tensor:
    """Stream-ordered scratch buffer reused across calls (grown on demand)."""
    key = (str(device), slot)
    buf = _WS.get(key)
    nbytes = max(int(nbytes), 256)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(int(nbytes * 1.25) + 256, dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def _s():
    return L.stream_ptr()


_ATTN_ERR: dict = {}


def attn_err_word(device) -> torch.Tensor:
    """The sticky error word of the one-pass attention backward on ``device`` (mia_attn_bwd_onepass: a bounded
    hand-off wait that gave up sets it; the library never clears it)."""
    key = str(device)
    w = _ATTN_ERR.get(key)
    if w is None:
        w = _ATTN_ERR[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return w


def check_attention_errors() -> None:
    """Raise if any one-pass attention backward since start-up gave up a hand-off wait (its dQ was invalid).
    Host sync: call at epoch ends / the end of a benchmark, not per step."""
    for key, w in _ATTN_ERR.items():
        if int(w.item()) != 0:
            raise RuntimeError(f"attention backward on {key}: a dQ hand-off wait timed out (mia_attn_bwd_onepass); "
                               "the gradients of that step are invalid")
    check_logmel_errors()


_LOGMEL_ERR: dict = {}


def logmel_err_word(device) -> torch.Tensor:
    """The 8 sticky u32 words of the log-mel FFT self-check on ``device`` (mia_logmel_fwd ``err``: [0] frames that
    failed Parseval / the vanishing checksum on all 3 tries, [1..3] the first (clip + 1, frame, wave), [4] frames
    that passed on a retry, [5..7] the first of those).  The library never clears them."""
    key = str(device)
    w = _LOGMEL_ERR.get(key)
    if w is None:
        w = _LOGMEL_ERR[key] = torch.zeros(8, dtype=torch.int32, device=device)
    return w


def logmel_error_counts() -> dict:
    """{device: (failed, retried, first_failed (clip, frame, wave) | None, first_retried | None)}.  Host sync."""
    res = {}
    for key, w in _LOGMEL_ERR.items():
        v = [int(x) for x in w.cpu().tolist()]
        res[key] = (v[0], v[4], (v[1] - 1, v[2], v[3]) if v[1] else None, (v[5] - 1, v[6], v[7]) if v[5] else None)
    return res


def check_logmel_errors() -> None:
    """Raise if a log-mel frame failed its in-kernel FFT self-check on every try since start-up (its features are
    invalid); frames that passed on a retry are reported by ``logmel_error_counts`` only.  Host sync."""
    for key, (bad, _, first, _) in logmel_error_counts().items():
        if bad:
            raise RuntimeError(f"log-mel on {key}: {bad} frame(s) failed the FFT self-check on every try (first: "
                               f"clip {first[0]}, frame {first[1]}, wave {first[2]}); their features are invalid")


# ------------------------------------------------------------------------------------ GEMM
def dense(t: torch.Tensor, layout: int, rows: int, cols: int, ld: int | None = None,
          pre: int = L.PRE_NONE, scale=None, shift=None, dtype: int | None = None) -> L.MiaOperand:
    o = L.MiaOperand()
    o.ptr = t.data_ptr()
    o.kind = L.OP_DENSE
    o.dtype = L.dtype_code(t) if dtype is None else dtype
    o.layout = layout
    o.pre = pre
    o.rows, o.cols, o.ld = rows, cols, cols if ld is None else ld
    o.pre_scale = L.ptr(scale)
    o.pre_shift = L.ptr(shift)
    o._keep = (t, scale, shift)  # the descriptor owns its tensors until the launch is enqueued
    return o


def conv(t: torch.Tensor, layout: int, n, h, w, c, oh, ow, kh, kw, sh=1, sw=1, ph=0, pw=0,
         pre: int = L.PRE_NONE, scale=None, shift=None, row_kind: bool = False) -> L.MiaOperand:
    o = L.MiaOperand()
    o.ptr = t.data_ptr()
    o.kind = L.OP_CONVROW if row_kind else L.OP_CONV
    o.dtype = L.dtype_code(t)
    o.layout = layout
    o.pre = pre
    o.n, o.h, o.w, o.c = n, h, w, c
    o.oh, o.ow, o.kh, o.kw = oh, ow, kh, kw
    o.sh, o.sw, o.ph, o.pw = sh, sw, ph, pw
    o.pre_scale = L.ptr(scale)
    o.pre_shift = L.ptr(shift)
    o._keep = (t, scale, shift)
    return o


def epilogue(out: torch.Tensor, ldc: int, act: int = L.ACT_NONE, bias=None, aux=None, ldaux: int = 0,
             accumulate: bool = False, alpha: float = 1.0, act_scale: float = 1.0,
             rowmap=None, sqsum=None, colsum=None, mx=None, a_colsum=None) -> L.MiaEpilogue:
    """Output descriptor of a GEMM.  ``sqsum``: optional f64 tensor of ``mia_gemm_sqsum_slots(M, N)``
    entries that receives the per-tile sums of squares of a plain f32 output (see ``sqsum_slots``).
    ``colsum``: optional f32 (N,) tensor receiving the column sums of the stored output (the bias
    gradient of the linear whose dy this output is).  ``mx``: optional MXTensor (mx_empty) receiving an
    MX-fp8 copy of a bf16 output (256x256 kernels only).  ``a_colsum``: optional f32 (M,) tensor receiving
    the column sums over k of a k-by-m (RC) A operand -- the bias gradient of a weight-gradient GEMM's dy."""
    e = L.MiaEpilogue()
    e.ptr = out.data_ptr()
    e.dtype = L.dtype_code(out)
    e.act = act
    e.accumulate = int(accumulate)
    e.ldc = ldc
    if rowmap is not None:
        e.rm_inner, e.rm_outer, e.rm_istride, e.rm_offset = rowmap
    e.bias = L.ptr(bias)
    if aux is not None:
        e.aux = aux.data_ptr()
        e.aux_dtype = L.dtype_code(aux)
        e.ldaux = ldaux
    e.alpha = alpha
    e.act_scale = act_scale
    e.sqsum = L.ptr(sqsum)
    e.colsum = L.ptr(colsum)
    if mx is not None:  # MXTensor receiving the MX-fp8 copy of the bf16 output
        e.mx_q, e.mx_scales = mx.q.data_ptr(), mx.scales.data_ptr()
    e.a_colsum = L.ptr(a_colsum)
    e._keep = (out, bias, aux, sqsum, colsum, mx, a_colsum)
    return e


def sqsum_slots(out: torch.Tensor, M: int, N: int) -> torch.Tensor:
    """A sum-of-squares slot buffer (f64, one per 128 x 128 tile) for the plain f32 GEMM output ``out``
    (M x N); pass it as ``epilogue(..., sqsum=)``, then ``tag_sqsum(param, out, buf)``."""
    buf = torch.empty(int(L.load().mia_gemm_sqsum_slots(M, N)), dtype=torch.float64, device=out.device)
    return buf


def gemm_sqsum_only(A: L.MiaOperand, B: L.MiaOperand, M: int, N: int, K: int, sq: torch.Tensor,
                    tag: str | None = None):
    """Per-tile sums of squares of the f32 product A^T B (mia_gemm_sqsum_only): nothing else stored."""
    rec = PROBE is not None and tag in PROBE
    if rec:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    L.check(L.load().mia_gemm_sqsum_only(A, B, M, N, K, sq.data_ptr(), _s()), "mia_gemm_sqsum_only")
    if rec:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        PROBE[tag].append((e0, e1, 2 * M * N * K, _operand_bytes(A, M, K) + _operand_bytes(B, N, K)))


def defer_weight_grad(param: torch.Tensor, A: L.MiaOperand, B: L.MiaOperand, M: int, N: int, K: int,
                      keep, tag: str | None = None) -> None:
    """Defer the f32 weight gradient ``A^T B`` (M x N, the parameter's shape) of ``param`` to the optimizer:
    only its per-tile sums of squares are computed now (the clip norm's share); FusedAdam.step recomputes
    the product inside the fused Adam GEMM (mia_gemm_adam), so the gradient is never written or re-read.
    ``keep``: the operand tensors (kept alive until the step)."""
    if getattr(param, "_mia_deferred", None) is not None:
        raise RuntimeError("a deferred weight gradient is still pending: call the optimizer's step() "
                           "(FusedAdam) between backward passes, or build the model's optimizer as torch.optim")
    sq = torch.empty(int(L.load().mia_gemm_sqsum_slots(M, N)), dtype=torch.float64, device=param.device)
    gemm_sqsum_only(A, B, M, N, K, sq, tag=tag)
    param._mia_deferred = dict(A=A, B=B, M=M, N=N, K=K, sq=sq, keep=keep)


def defers_to_fused_adam(p: torch.Tensor) -> bool:
    """True while the FusedAdam that last took ``p`` is alive (src/training/optim.py keeps a weak reference
    on the parameter): only then may a model defer ``p``'s weight gradient to the optimizer step."""
    ref = getattr(p, "_mia_fused_adam", None)
    return callable(ref) and ref() is not None


def materialise_deferred_grad(param: torch.Tensor) -> None:
    """Write a pending deferred weight gradient (defer_weight_grad) into ``param.grad`` with the same GEMM
    main loop, for an optimizer that does not fuse it."""
    d = getattr(param, "_mia_deferred", None)
    if d is None:
        return
    if "row0" in d:
        raise RuntimeError("a row-sharded deferred gradient (GradAllReducer fc1_exchange='shard') is applied "
                           "by FusedAdam only; use fc1_exchange='gather' with another optimizer")
    dW = torch.empty(d["M"], d["N"], dtype=torch.float32, device=param.device)
    gemm(d["A"], d["B"], epilogue(dW, d["N"]), d["M"], d["N"], d["K"], L.BF16)
    param._mia_deferred = None
    param.grad = dW.view_as(param) if param.grad is None else param.grad.add_(dW.view_as(param))


def tag_sqsum(param: torch.Tensor, grad: torch.Tensor, buf: torch.Tensor) -> None:
    """Record on ``param`` that ``buf`` holds the per-tile sums of squares of the gradient ``grad``, so
    FusedAdam's clip-norm pass reads the slots instead of the tensor.  The tag lives on the parameter
    (autograd hands ``grad``'s storage on as ``param.grad`` under a new Python object) and holds
    ``grad``'s storage -- not ``grad``: a second tensor reference would make autograd copy the gradient
    instead of adopting it -- so that memory cannot be reused by another tensor while tagged; with the
    version it records, any later write to the gradient (an all-reduce, an accumulation) invalidates it."""
    param._mia_sqsum = (buf, grad.untyped_storage(), grad.data_ptr(), grad.numel(), grad._version)


def valid_sqsum(param: torch.Tensor, grad: torch.Tensor):
    """The slot buffer tagged on ``param`` if it still describes ``grad``'s current contents, else None."""
    tag = getattr(param, "_mia_sqsum", None)
    if tag is None:
        return None
    buf, st, ptr, numel, ver = tag
    if (grad.untyped_storage().data_ptr() != st.data_ptr() or grad.data_ptr() != ptr or grad.numel() != numel
            or grad._version != ver):
        return None
    return buf


def _tiles(M, N):
    if M <= 32:
        bm, bn = 32, 128
    elif N <= 32:
        bm, bn = 256, 32
    elif N <= 64:
        bm, bn = 128, 64
    elif M <= 64:
        bm, bn = 64, 128
    else:
        bm, bn = 128, 128
    return math.ceil(M / bm) * math.ceil(N / bn)


def auto_split(M: int, N: int, K: int, target_blocks: int = 1024, min_k: int = 1024) -> int:
    tiles = _tiles(M, N)
    if tiles >= target_blocks:
        return 1
    split = math.ceil(target_blocks / tiles)
    split = min(split, max(1, K // min_k))
    return max(1, min(split, 256))


# Live kernel probe (bench.py): tag -> list of (start_event, end_event, flops, bytes).
PROBE: dict | None = None


class probe:
    """Times the enclosed launches with HIP events on the current stream when ``tag`` is being probed
    (bench.py's live per-kernel roofline); ``flop`` / ``nbytes`` are the algorithmic work of the launch."""

    def __init__(self, tag: str, flop: float, nbytes: float):
        self.tag, self.flop, self.nbytes = tag, flop, nbytes
        self.on = PROBE is not None and tag in PROBE

    def __enter__(self):
        if self.on:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if self.on and exc[0] is None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            PROBE[self.tag].append((self.e0, e1, self.flop, self.nbytes))
        return False


def _operand_bytes(o: L.MiaOperand, M_or_N: int, K: int) -> int:
    es = 4 if o.dtype == L.F32 else 2
    if o.kind == L.OP_DENSE:
        return o.rows * o.cols * es
    return o.n * o.h * o.w * o.c * es  # each input element is read once from HBM (tile reuse on chip)


def gemm(A: L.MiaOperand, B: L.MiaOperand, E: L.MiaEpilogue, M: int, N: int, K: int, compute: int,
         split_k: int | None = None, device=None, tag: str | None = None):
    lib = L.load()
    if split_k is None:
        path = lib.mia_gemm_path(A, B, M, N, K, compute, 2) if compute == L.BF16 else 0
        if path == 2:  # row-window wgrad: (KH / ky-per-block) x split blocks, >= ~32 chunks of 128 px each
            chunks = B.n * B.oh * -(-B.ow // 128)
            split_k = max(2, min(512, chunks // 32))
        elif path == 3:  # single-channel tap wgrad: split blocks over chunks of 256 px
            chunks = B.n * B.oh * -(-B.ow // 256)
            split_k = max(2, min(1024, chunks // 16))
        else:
            split_k = auto_split(M, N, K)
    ws = None
    nws = lib.mia_gemm_workspace_bytes_ex(A, B, E, M, N, K, compute, split_k)
    if nws > 0:
        ws = workspace(nws, device or torch.cuda.current_device(), "gemm")
    rec = PROBE is not None and tag in PROBE
    if rec:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    L.check(lib.mia_gemm(A, B, E, M, N, K, compute, split_k, L.ptr(ws), _s()), "mia_gemm")
    if rec:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        out_b = M * N * (4 if E.dtype == L.F32 else 2)
        PROBE[tag].append((e0, e1, 2 * M * N * K, _operand_bytes(A, M, K) + _operand_bytes(B, N, K) + out_b))


# ------------------------------------------------------------------------------------ BN / pool
@dataclass
class BNState:
    mean: torch.Tensor
    invstd: torch.Tensor
    scale: torch.Tensor
    shift: torch.Tensor


def bn_fwd_stats(x: torch.Tensor, P: int, C: int, gamma, beta, running_mean, running_var, momentum: float,
                 eps: float, training: bool) -> BNState:
    dev = x.device
    st = torch.empty(4, C, dtype=torch.float32, device=dev)
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(P, C), dev, "bn")
    L.check(lib.mia_bn_fwd_stats(x.data_ptr(), L.dtype_code(x), P, C, L.ptr(gamma), L.ptr(beta),
                                 L.ptr(running_mean), L.ptr(running_var), momentum, eps, int(training),
                                 st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr(),
                                 ws.data_ptr(), _s()), "mia_bn_fwd_stats")
    return BNState(st[0], st[1], st[2], st[3])


def bn_relu_bwd_reduce(dact, dz, x, P, C, bn: BNState):
    """ReLU+BN backward reductions (dgamma, dbeta); dz=None: the masked gradient is not written
    (bn_relu_bwd_apply recomputes the mask)."""
    dev = x.device
    g = torch.empty(2, C, dtype=torch.float32, device=dev)
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(P, C), dev, "bn")
    L.check(lib.mia_bn_relu_bwd_reduce(dact.data_ptr(), L.ptr(dz), x.data_ptr(), L.dtype_code(x), P, C,
                                       bn.scale.data_ptr(), bn.shift.data_ptr(), bn.mean.data_ptr(),
                                       bn.invstd.data_ptr(), g[0].data_ptr(), g[1].data_ptr(), ws.data_ptr(),
                                       _s()), "mia_bn_relu_bwd_reduce")
    return g[0], g[1]  # dgamma, dbeta


def bn_bwd_apply(dz, x, dx, P, C, gamma, bn: BNState, dgamma, dbeta, dbias=None):
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(P, C), x.device, "bn")
    L.check(lib.mia_bn_bwd_apply(dz.data_ptr(), x.data_ptr(), dx.data_ptr(), L.dtype_code(x), P, C,
                                 L.ptr(gamma), bn.mean.data_ptr(), bn.invstd.data_ptr(), dgamma.data_ptr(),
                                 dbeta.data_ptr(), L.ptr(dbias), ws.data_ptr(), _s()), "mia_bn_bwd_apply")


def bn_relu_bwd_apply(dact, x, dx, P, C, gamma, bn: BNState, dgamma, dbeta, dbias=None):
    """dx = BN backward of relu(bn(x)) with the ReLU mask recomputed from x (one pass)."""
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(P, C), x.device, "bn")
    L.check(lib.mia_bn_relu_bwd_apply(dact.data_ptr(), x.data_ptr(), dx.data_ptr(), L.dtype_code(x), P, C,
                                      L.ptr(gamma), bn.scale.data_ptr(), bn.shift.data_ptr(), bn.mean.data_ptr(),
                                      bn.invstd.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), L.ptr(dbias),
                                      ws.data_ptr(), _s()), "mia_bn_relu_bwd_apply")


def pool_bwd_gather(dout, out_layout, argmax, x, n, h, w, c, kh, kw, bn: BNState, win=None):
    """Sparse half of the pooled backward: (gm, dgamma, dbeta); gm = ReLU-masked gradient at each
    pooled cell's argmax, f32 (n, h//kh, w//kw, c).  ``win``: the raw winner values the forward
    saved (pool_raw_stats), read instead of gathering x at the argmax positions."""
    if win is not None and (win.dtype != x.dtype or win.numel() != n * (h // kh) * (w // kw) * c):
        raise ValueError("pool_bwd_gather: win must hold one x-typed value per pooled cell and channel")
    dev = x.device
    g = torch.empty(2, c, dtype=torch.float32, device=dev)
    gm = torch.empty(n * (h // kh) * (w // kw), c, dtype=torch.float32, device=dev)
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(n * h * w, c), dev, "bn")
    L.check(lib.mia_pool_bwd_gather(dout.data_ptr(), out_layout, argmax.data_ptr(), x.data_ptr(), L.ptr(win),
                                    L.dtype_code(x), n, h, w, c, kh, kw, bn.scale.data_ptr(), bn.shift.data_ptr(), bn.mean.data_ptr(),
                                    bn.invstd.data_ptr(), gm.data_ptr(), g[0].data_ptr(), g[1].data_ptr(),
                                    ws.data_ptr(), _s()), "mia_pool_bwd_gather")
    return gm, g[0], g[1]


def pool_bn_relu_bwd_apply(gm, argmax, x, n, h, w, c, kh, kw, gamma, bn: BNState, dgamma, dbeta, dx, dbias=None):
    """Dense half: BN backward of the pooled layer, g taken from gm at the argmax (one pass x -> dx)."""
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(n * h * w, c), x.device, "bn")
    L.check(lib.mia_pool_bn_relu_bwd_apply(gm.data_ptr(), argmax.data_ptr(), x.data_ptr(), L.dtype_code(x), n, h, w,
                                           c, kh, kw, L.ptr(gamma), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                                           dgamma.data_ptr(), dbeta.data_ptr(), dx.data_ptr(), L.ptr(dbias),
                                           ws.data_ptr(), _s()), "mia_pool_bn_relu_bwd_apply")


def pool_fwd(x, n, h, w, c, kh, kw, bn: BNState, out, out_layout, argmax, win=None):
    """maxpool(relu(bn(x))) with the argmax per cell; ``win`` (optional, x's dtype, one value per cell and
    channel) receives the winner's raw x for pool_bwd_gather."""
    if win is not None and (win.dtype != x.dtype or win.numel() != n * (h // kh) * (w // kw) * c):
        raise ValueError("pool_fwd: win must hold one x-typed value per pooled cell and channel")
    L.check(L.load().mia_pool_fwd(x.data_ptr(), L.dtype_code(x), n, h, w, c, kh, kw, bn.scale.data_ptr(),
                                  bn.shift.data_ptr(), out.data_ptr(), out_layout, argmax.data_ptr(), L.ptr(win),
                                  _s()),
            "mia_pool_fwd")


def pool_raw_stats(x, n, h, w, c, kh, kw, gamma, kshift, win, argmax):
    """maxpool(relu(bn(x))) winners before the BN statistics exist (bf16, training): writes the raw
    winner values `win` (n, h/kh, w/kw, c) bf16 and `argmax`, returns (partial, nblk) of the BN shifted
    sums about kshift for bn_finalize_shifted; pool_apply then writes the pooled output."""
    assert x.dtype == torch.bfloat16 and win.dtype == torch.bfloat16 and x.is_contiguous()
    nblk = 2048
    part = torch.empty(nblk, c, 2, dtype=torch.float32, device=x.device)
    L.check(L.load().mia_pool_raw_stats(x.data_ptr(), n, h, w, c, kh, kw, gamma.data_ptr(), kshift.data_ptr(),
                                        win.data_ptr(), argmax.data_ptr(), part.data_ptr(), nblk, _s()),
            "mia_pool_raw_stats")
    return part, nblk


def pool_apply(win, n, oh, ow, c, bn: BNState, out, out_layout):
    L.check(L.load().mia_pool_apply(win.data_ptr(), n, oh, ow, c, bn.scale.data_ptr(), bn.shift.data_ptr(),
                                    out.data_ptr(), L.dtype_code(out), out_layout, _s()), "mia_pool_apply")


def pool_bwd_bn_relu_reduce(dout, out_layout, argmax, x, n, h, w, c, kh, kw, bn: BNState, dz):
    g = torch.empty(2, c, dtype=torch.float32, device=x.device)
    lib = L.load()
    ws = workspace(lib.mia_bn_partial_bytes(n * h * w, c), x.device, "bn")
    L.check(lib.mia_pool_bwd_bn_relu_reduce(dout.data_ptr(), out_layout, argmax.data_ptr(), x.data_ptr(),
                                            L.dtype_code(x), n, h, w, c, kh, kw, bn.scale.data_ptr(),
                                            bn.shift.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                                            dz.data_ptr(), g[0].data_ptr(), g[1].data_ptr(), ws.data_ptr(), _s()),
            "mia_pool_bwd_bn_relu_reduce")
    return g[0], g[1]


def colsum(x, P, C, ld=None):
    out = torch.empty(C, dtype=torch.float32, device=x.device)
    ws = workspace(1024 * C * 4, x.device, "colsum")  # MIA_COLSUM_MAXBLK * C floats
    L.check(L.load().mia_colsum(x.data_ptr(), L.dtype_code(x), P, C, C if ld is None else ld, out.data_ptr(),
                                ws.data_ptr(), _s()), "mia_colsum")
    return out


def col2im_rows(p, n, ph, w, kh, out):
    L.check(L.load().mia_col2im_rows(p.data_ptr(), n, ph, w, kh, out.data_ptr(), L.dtype_code(out), _s()),
            "mia_col2im_rows")


def conv1ch_dgrad(dy: torch.Tensor, w: torch.Tensor, n: int, oh: int, ow: int, out: torch.Tensor,
                  tag: str | None = None):
    """dX of the 1-input-channel 8x8 conv (bf16): dy (n*oh*ow, 32) NHWC, w f32 (32, 1, 8, 8) -> out (n, oh+7, ow+7)."""
    assert dy.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and w.dtype == torch.float32
    assert dy.numel() == n * oh * ow * 32 and out.numel() == n * (oh + 7) * (ow + 7) and w.numel() == 32 * 64
    assert dy.is_contiguous() and out.is_contiguous() and w.is_contiguous()
    flop = 2.0 * n * oh * ow * 32 * 64
    with probe(tag or "", flop, dy.numel() * 2 + out.numel() * 2):
        L.check(L.load().mia_conv1ch_dgrad(dy.data_ptr(), w.data_ptr(), out.data_ptr(), n, oh, ow, _s()),
                "mia_conv1ch_dgrad")


def fe_conv1_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, y1: torch.Tensor, n: int, t: int,
                 stats: bool, tag: str | None = None):
    """EnvNet conv1 forward (bf16 out): x f32 (n, t), w bf16 (32, 64), bias f32 (32) -> y1 (n*w1, 32).
    stats=True also returns (partial, nblk): the BN1 shifted sums about bias, for bn_finalize_shifted."""
    w1 = (t - 64) // 2 + 1
    assert x.dtype == torch.float32 and w.dtype == torch.bfloat16 and y1.dtype == torch.bfloat16
    assert x.numel() == n * t and w.numel() == 32 * 64 and y1.numel() == n * w1 * 32 and bias.numel() == 32
    nw = 4096
    part = torch.empty(nw, 32, 2, dtype=torch.float32, device=x.device) if stats else None
    with probe(tag or "", 2.0 * n * w1 * 32 * 64, x.numel() * 4 + y1.numel() * 2):
        L.check(L.load().mia_fe_conv1_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr(), y1.data_ptr(), L.ptr(part),
                                          nw, n, t, _s()), "mia_fe_conv1_fwd")
    return (part, nw) if stats else None


def fe_conv3_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, y: torch.Tensor, n: int, h: int, wd: int,
                 stats: bool, tag: str | None = None):
    """EnvNet trunk conv3 (1 -> 32, 8x8) forward, bf16: x (n, h, wd), w (32, 64) -> y (n*(h-7)*(wd-7), 32).
    stats=True also returns (partial, nblk) of the BN shifted sums about bias."""
    oh, ow = h - 7, wd - 7
    assert x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and y.dtype == torch.bfloat16
    assert x.numel() == n * h * wd and w.numel() == 32 * 64 and y.numel() == n * oh * ow * 32
    nw = 4096
    part = torch.empty(nw, 32, 2, dtype=torch.float32, device=x.device) if stats else None
    with probe(tag or "", 2.0 * n * oh * ow * 32 * 64, x.numel() * 2 + y.numel() * 2):
        L.check(L.load().mia_fe_conv3_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr(), y.data_ptr(), L.ptr(part),
                                          nw, n, h, wd, _s()), "mia_fe_conv3_fwd")
    return (part, nw) if stats else None


def trunk_conv8(x: torch.Tensor, w: torch.Tensor, y: torch.Tensor, n: int, h: int, wd: int, ph: int = 0,
                pw: int = 0, scale=None, shift=None, bias=None, stats: bool = False, tag: str | None = None):
    """EnvNet trunk conv4 (32 -> 32, 8x8), bf16, row-rolling kernel: x (n*h*wd, 32) NHWC, w packed OHWI
    (32, 2048) -> y (n*oh*ow, 32), oh = h+2ph-7, ow = wd+2pw-7.  scale/shift: BN+ReLU applied to x.
    stats=True (needs bias) also returns (partial, nblk) of the BN shifted sums about bias."""
    oh, ow = h + 2 * ph - 7, wd + 2 * pw - 7
    assert x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and y.dtype == torch.bfloat16
    assert x.numel() == n * h * wd * 32 and w.numel() == 32 * 2048 and y.numel() == n * oh * ow * 32
    assert x.is_contiguous() and w.is_contiguous() and y.is_contiguous()
    assert (scale is None) == (shift is None) and (not stats or bias is not None)
    nblk = 256
    part = torch.empty(4 * nblk, 32, 2, dtype=torch.float32, device=x.device) if stats else None
    with probe(tag or "", 2.0 * n * oh * ow * 32 * 2048, x.numel() * 2 + y.numel() * 2):
        L.check(L.load().mia_trunk_conv8(x.data_ptr(), L.ptr(scale), L.ptr(shift), w.data_ptr(), L.ptr(bias),
                                         y.data_ptr(), L.ptr(part), nblk, n, h, wd, ph, pw, _s()), "mia_trunk_conv8")
    return (part, 4 * nblk) if stats else None


def trunk_conv8_dgrad_bn(dy: torch.Tensor, w: torch.Tensor, dx: torch.Tensor, n: int, h: int, wd: int,
                         bx: torch.Tensor, bn: BNState, tag: str | None = None):
    """conv4 backward-data (dy (n*h*wd, 32) -> dx (n*(h+7)*(wd+7), 32), w the layout-1 flipped pack) with the
    ReLU+BN backward sums of bn (input bx, dx's shape) formed in its epilogue: returns (dgamma, dbeta) as
    bn_relu_bwd_reduce(dx, None, bx, ...) does."""
    oh, ow = h + 7, wd + 7
    assert dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and dx.dtype == torch.bfloat16
    assert bx.dtype == torch.bfloat16 and bx.numel() == dx.numel() and bx.is_contiguous()
    assert dy.numel() == n * h * wd * 32 and w.numel() == 32 * 2048 and dx.numel() == n * oh * ow * 32
    assert dy.is_contiguous() and w.is_contiguous() and dx.is_contiguous()
    nblk = 256
    part = workspace(4 * nblk * 64 * 4, dy.device, "c8red")
    g = torch.empty(2, 32, dtype=torch.float32, device=dy.device)
    with probe(tag or "", 2.0 * n * oh * ow * 32 * 2048, dy.numel() * 2 + dx.numel() * 2 + bx.numel() * 2):
        L.check(L.load().mia_trunk_conv8_dgrad_bn(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), nblk, n, h, wd,
                                                  bx.data_ptr(), bn.scale.data_ptr(), bn.shift.data_ptr(),
                                                  bn.mean.data_ptr(), bn.invstd.data_ptr(), g[0].data_ptr(),
                                                  g[1].data_ptr(), part.data_ptr(), _s()), "mia_trunk_conv8_dgrad_bn")
    return g[0], g[1]  # dgamma, dbeta


def conv3_wgrad(x: torch.Tensor, dy: torch.Tensor, dw: torch.Tensor, n: int, h: int, wd: int,
                tag: str | None = None):
    """Weight gradient of EnvNet trunk conv3 (1 -> 32, 8x8), bf16: x (n, h, wd), dy (n*(h-7)*(wd-7), 32)
    -> dw f32 (32, 64) (taps ky*8 + kx)."""
    oh, ow = h - 7, wd - 7
    assert x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16 and dw.dtype == torch.float32
    assert x.numel() == n * h * wd and dy.numel() == n * oh * ow * 32 and dw.numel() == 32 * 64
    assert x.is_contiguous() and dy.is_contiguous() and dw.is_contiguous()
    nw = 4096
    part = workspace(nw * 2048 * 4 + 64 * 2048 * 8, x.device, "conv3w")
    with probe(tag or "", 2.0 * n * oh * ow * 32 * 64, x.numel() * 2 + dy.numel() * 2):
        L.check(L.load().mia_conv3_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), part.data_ptr(), nw, n, h, wd,
                                         _s()), "mia_conv3_wgrad")


def conv3_wgrad_bn(x: torch.Tensor, da: torch.Tensor, ya: torch.Tensor, dy: torch.Tensor, dw: torch.Tensor,
                   dbias: torch.Tensor, n: int, h: int, wd: int, gamma, bn: BNState, dgamma, dbeta,
                   tag: str | None = None):
    """conv3_wgrad with dY formed from the ReLU+BN backward of conv3's BN while staging: dy = the
    bn_relu_bwd_apply of da (gradient of relu(bn(ya))) -- written out (may be da itself) -- and dbias its
    column sum, in the same pass as the weight gradient dw."""
    oh, ow = h - 7, wd - 7
    for t in (da, ya, dy):
        assert t.dtype == torch.bfloat16 and t.numel() == n * oh * ow * 32 and t.is_contiguous()
    assert x.dtype == torch.bfloat16 and x.numel() == n * h * wd and x.is_contiguous()
    assert dw.dtype == torch.float32 and dw.numel() == 32 * 64 and dbias.dtype == torch.float32 and dbias.numel() == 32
    nw = 4096
    lib = L.load()
    part = workspace(int(lib.mia_conv3_wgrad_workspace_bytes(nw)), x.device, "conv3w")
    with probe(tag or "", 2.0 * n * oh * ow * 32 * 64, x.numel() * 2 + da.numel() * 6):
        L.check(lib.mia_conv3_wgrad_bn(x.data_ptr(), da.data_ptr(), ya.data_ptr(), dy.data_ptr(), dw.data_ptr(),
                                       dbias.data_ptr(), part.data_ptr(), nw, n, h, wd, L.ptr(gamma),
                                       bn.scale.data_ptr(), bn.shift.data_ptr(), bn.mean.data_ptr(),
                                       bn.invstd.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), _s()),
                "mia_conv3_wgrad_bn")


def bn_finalize_shifted(partial: torch.Tensor, nblk: int, P: int, C: int, kshift: torch.Tensor, gamma, beta,
                        running_mean, running_var, momentum: float, eps: float) -> BNState:
    """Training-mode BN statistics from shifted partial sums (mia_bn_finalize_shifted)."""
    st = torch.empty(4, C, dtype=torch.float32, device=partial.device)
    L.check(L.load().mia_bn_finalize_shifted(partial.data_ptr(), nblk, P, C, kshift.data_ptr(), L.ptr(gamma),
                                             L.ptr(beta), L.ptr(running_mean), L.ptr(running_var), momentum, eps, 1,
                                             st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr(),
                                             _s()), "mia_bn_finalize_shifted")
    return BNState(st[0], st[1], st[2], st[3])


def fe_conv2_fwd(y1: torch.Tensor, scale, shift, w: torch.Tensor, bias, y2: torch.Tensor, n: int, w1: int,
                 w2: int, tag: str | None = None):
    """EnvNet conv2 forward (bf16): y1 (n*w1, 32), optional BN1 scale/shift (+ReLU) applied to the
    input, w packed OHWI (64, 16*32), bias f32 (64) or None -> y2 (n*w2, 64)."""
    assert y1.dtype == torch.bfloat16 and y2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
    assert y1.numel() == n * w1 * 32 and y2.numel() == n * w2 * 64 and w.numel() == 64 * 512
    assert y1.is_contiguous() and y2.is_contiguous() and w.is_contiguous()
    flop = 2.0 * n * w2 * 64 * 512
    with probe(tag or "", flop, y1.numel() * 2 + y2.numel() * 2):
        L.check(L.load().mia_fe_conv2_fwd(y1.data_ptr(), L.ptr(scale), L.ptr(shift), w.data_ptr(), L.ptr(bias),
                                          y2.data_ptr(), n, w1, w2, _s()), "mia_fe_conv2_fwd")


def fe_conv2_dgrad(dy2: torch.Tensor, wpar: torch.Tensor, da1: torch.Tensor, n: int, w1: int, w2: int,
                   tag: str | None = None):
    """Backward-data of EnvNet conv2 (bf16): dy2 (n*w2, 64), wpar = pack_weight(W, bf16, 2)
    (2*32, 8*64) -> da1 (n*w1, 32)."""
    assert dy2.dtype == torch.bfloat16 and da1.dtype == torch.bfloat16 and wpar.dtype == torch.bfloat16
    assert dy2.numel() == n * w2 * 64 and da1.numel() == n * w1 * 32 and wpar.numel() == 64 * 512
    assert dy2.is_contiguous() and da1.is_contiguous() and wpar.is_contiguous()
    flop = 2.0 * n * w1 * 32 * 512
    with probe(tag or "", flop, dy2.numel() * 2 + da1.numel() * 2):
        L.check(L.load().mia_fe_conv2_dgrad(dy2.data_ptr(), wpar.data_ptr(), da1.data_ptr(), n, w1, w2, _s()),
                "mia_fe_conv2_dgrad")


def fe_conv2_wgrad(dy2: torch.Tensor, y1: torch.Tensor, scale, shift, dw: torch.Tensor, n: int, w1: int, w2: int,
                   tag: str | None = None):
    """Weight gradient of EnvNet conv2 (bf16 operands): dy2 (n*w2, 64), y1 (n*w1, 32) with BN1
    scale/shift (+ReLU) applied while staging -> dw f32 (64, 16*32) in OHWI order."""
    assert dy2.dtype == torch.bfloat16 and y1.dtype == torch.bfloat16 and dw.dtype == torch.float32
    assert dy2.numel() == n * w2 * 64 and y1.numel() == n * w1 * 32 and dw.numel() == 64 * 512
    nlaunch = -(-(n * w1 * 64) // (2 ** 31 - 1)) + 1
    nbytes = 512 * nlaunch * 64 * 512 * 4
    ws = workspace(nbytes, dy2.device, "fw")
    flop = 2.0 * n * w2 * 64 * 512
    with probe(tag or "", flop, (dy2.numel() + y1.numel()) * 2):
        L.check(L.load().mia_fe_conv2_wgrad(dy2.data_ptr(), y1.data_ptr(), L.ptr(scale), L.ptr(shift), dw.data_ptr(),
                                            n, w1, w2, ws.data_ptr(), ws.numel(), _s()), "mia_fe_conv2_wgrad")


def fe_conv1_wgrad_bn(x: torch.Tensor, dact: torch.Tensor, y1: torch.Tensor, n: int, t: int, gamma, bn: BNState,
                      dw: torch.Tensor, dbias: torch.Tensor, tag: str | None = None):
    """BN1+ReLU backward and EnvNet conv1 weight/bias gradient in one pass (bf16 operands):
    x f32 (n, t) waveform, dact = dL/d relu(bn1(y1)) and y1 bf16 (n*w1, 32) -> dw f32 (32, 64),
    dbias f32 (32); returns (dgamma, dbeta) of BN1."""
    w1 = (t - 64) // 2 + 1
    assert dact.dtype == torch.bfloat16 and y1.dtype == torch.bfloat16 and x.dtype == torch.float32
    assert dact.numel() == n * w1 * 32 and y1.numel() == n * w1 * 32 and x.numel() == n * t
    assert dw.numel() == 32 * 64 and dw.dtype == torch.float32 and dbias.numel() == 32
    split = 512
    ws = workspace((split * (2 * 2048 + 96) + 2 * 2048 + n * 80 + 2 * 160 + 4) * 4, x.device, "tapw")
    g = torch.empty(2, 32, dtype=torch.float32, device=x.device)
    flop = 4.0 * n * w1 * 32 * 64
    with probe(tag or "", flop, (dact.numel() + y1.numel()) * 2 + x.numel() * 4):
        L.check(L.load().mia_fe_conv1_wgrad_bn(
            x.data_ptr(), dact.data_ptr(), y1.data_ptr(), n, t, bn.scale.data_ptr(), bn.shift.data_ptr(),
            L.ptr(gamma), bn.mean.data_ptr(), bn.invstd.data_ptr(), g[0].data_ptr(), g[1].data_ptr(),
            dw.data_ptr(), dbias.data_ptr(), ws.data_ptr(), split, _s()), "mia_fe_conv1_wgrad_bn")
    return g[0], g[1]


def bn_relu_apply(x: torch.Tensor, P: int, C: int, bn: BNState, out: torch.Tensor):
    """out = bf16(relu(x * bn.scale + bn.shift)) for bf16 (P, C) activations."""
    assert x.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and x.numel() == P * C == out.numel()
    L.check(L.load().mia_bn_relu_apply(x.data_ptr(), P, C, bn.scale.data_ptr(), bn.shift.data_ptr(), out.data_ptr(),
                                       _s()), "mia_bn_relu_apply")


def conv_w2_fwd(x: torch.Tensor, rows: int, w: int, cin: int, wpk: torch.Tensor, bias, out: torch.Tensor,
                tag: str | None = None):
    """(1, 2) conv forward, stride 1 (EnvNet trunk blocks 3-4), as one dense GEMM over every input
    pixel (rows of the im2col view overlap: ld = cin, length 2*cin) whose epilogue drops each row's last
    column (drop-mode row map, MIA_RM_DROP; MIA_W2_DROPCOPY=1: a full-grid output + mia_drop_last_col).
    x bf16 (rows*w, cin) whose storage holds ONE extra pixel (read by the dropped last output);
    wpk bf16 (cout, 2*cin) OHWI; out bf16 (rows*(w-1), cout)."""
    cout = wpk.numel() // (2 * cin)
    assert x.dtype == torch.bfloat16 and wpk.dtype == torch.bfloat16 and out.dtype == torch.bfloat16
    assert x.numel() == rows * w * cin and out.numel() == rows * (w - 1) * cout
    assert x.untyped_storage().nbytes() - x.storage_offset() * 2 >= (rows * w + 1) * cin * 2, "x needs a pad pixel"
    P = rows * w
    if not W2_DROPCOPY:
        # the epilogue's drop-mode row map stores the w - 1 valid columns of every row straight into out
        gemm(dense(x, L.KC, P, 2 * cin, ld=cin), dense(wpk, L.KC, cout, 2 * cin),
             epilogue(out, cout, bias=bias, rowmap=(w, w - 1, 1, L.RM_DROP)), P, cout, 2 * cin, L.BF16, tag=tag)
        return
    ypad = workspace(P * cout * 2, x.device, "w2fwd")[: P * cout * 2].view(torch.bfloat16)
    gemm(dense(x, L.KC, P, 2 * cin, ld=cin), dense(wpk, L.KC, cout, 2 * cin), epilogue(ypad, cout, bias=bias),
         P, cout, 2 * cin, L.BF16, tag=tag)
    L.check(L.load().mia_drop_last_col(ypad.data_ptr(), rows, w, cout, out.data_ptr(), _s()), "mia_drop_last_col")


W2_SHIFT = os.environ.get("MIA_W2_SHIFT", "0") == "1"  # A/B switch: the interleaved shifted-copy form
W2_DROPCOPY = os.environ.get("MIA_W2_DROPCOPY", "0") == "1"  # A/B switch: full-grid forward output + column drop


def trunk_bwd_w2(dy: torch.Tensor, a: torch.Tensor, rows: int, w: int, cout: int, cin: int, wpk: torch.Tensor,
                 dw: torch.Tensor, dx: torch.Tensor, tag: str = "", wflip: torch.Tensor | None = None):
    """Backward of a (1, 2) conv, stride 1 (EnvNet trunk blocks 3-4).  One pass lays dy on the input grid
    (G = [zero pixel] + dy with a zero last column per row, mia_pad_w2; it also zeroes a's pad pixel), then two
    dense GEMMs through overlapping views of G and a (rows of 2 pixels at a 1-pixel stride):
    dw (cout, 2*cin) OHWI f32 = G[1:]^T [a[q], a[q+1]], and dx (rows*w, cin) bf16 = [G[q], G[q+1]] Wflip with
    Wflip = the mode-1 pack (cin, 2*cout), [ci][kx'][co] = W[co][ci][0][1-kx'] -- half the bytes of the
    interleaved shifted copy Ashift[q][co*2+kx] = dy[q-kx][co] of the previous form (MIA_W2_SHIFT=1, which
    uses wpk (cout, 2*cin) read as the (2*cout, cin) K-major matrix).  a must carry one pad pixel."""
    assert dy.dtype == torch.bfloat16 and a.dtype == torch.bfloat16 and dw.dtype == torch.float32
    assert dy.numel() == rows * (w - 1) * cout and a.numel() == rows * w * cin and dw.numel() == cout * 2 * cin
    assert dx.numel() == rows * w * cin and dx.dtype == torch.bfloat16 and wpk.numel() == cout * 2 * cin
    P = rows * w
    if not W2_SHIFT and wflip is not None:
        assert a.untyped_storage().nbytes() - a.storage_offset() * 2 >= (P + 1) * cin * 2, "a needs a pad pixel"
        G = workspace((P + 1) * cout * 2, dy.device, "w2shift")[: (P + 1) * cout * 2].view(torch.bfloat16)
        L.check(L.load().mia_pad_w2(dy.data_ptr(), rows, w, cout, G.data_ptr(), a.data_ptr() + P * cin * 2, cin, _s()),
                "mia_pad_w2")
        G1 = G[cout:]
        gemm(dense(G1, L.RC, P, cout), dense(a, L.RC, P, 2 * cin, ld=cin), epilogue(dw, 2 * cin), cout, 2 * cin, P,
             L.BF16, tag=f"{tag}.wgrad" if tag else None)
        gemm(dense(G, L.KC, P, 2 * cout, ld=cout), dense(wflip, L.KC, cin, 2 * cout), epilogue(dx, cin), P, cin,
             2 * cout, L.BF16, tag=f"{tag}.dgrad" if tag else None)
        return
    ash = workspace(P * 2 * cout * 2, dy.device, "w2shift")[: P * 2 * cout * 2].view(torch.bfloat16)
    L.check(L.load().mia_shift_pad_w2(dy.data_ptr(), rows, w, cout, ash.data_ptr(), _s()), "mia_shift_pad_w2")
    gemm(dense(ash, L.RC, P, 2 * cout), dense(a, L.RC, P, cin), epilogue(dw, cin), 2 * cout, cin, P, L.BF16,
         tag=f"{tag}.wgrad" if tag else None)
    gemm(dense(ash, L.KC, P, 2 * cout), dense(wpk, L.RC, 2 * cout, cin), epilogue(dx, cin), P, cin, 2 * cout,
         L.BF16, tag=f"{tag}.dgrad" if tag else None)


def pack_weight(src: torch.Tensor, dtype: int, mode: int) -> torch.Tensor:
    cout, cin, kh, kw = src.shape
    out = torch.empty(src.numel(), dtype=L.torch_dtype(dtype), device=src.device)
    L.check(L.load().mia_pack_weight(src.data_ptr(), out.data_ptr(), dtype, cout, cin, kh, kw, mode, _s()),
            "mia_pack_weight")
    return out


def pack_weights(jobs):
    """mia_pack_weight for several weights in one launch per 16 (mia_pack_weights): jobs = [(src f32 (cout, cin,
    kh, kw), dtype, mode)], returns the packed tensors in order."""
    outs = []
    for s0 in range(0, len(jobs), L.PACK_BATCH):
        chunk = jobs[s0:s0 + L.PACK_BATCH]
        arr = (L.MiaPackJob * len(chunk))()
        for k, (src, dtype, mode) in enumerate(chunk):
            cout, cin, kh, kw = src.shape
            out = torch.empty(src.numel(), dtype=L.torch_dtype(dtype), device=src.device)
            arr[k] = L.MiaPackJob(src.data_ptr(), out.data_ptr(), dtype, cout, cin, kh, kw, mode)
            outs.append(out)
        L.check(L.load().mia_pack_weights(arr, len(chunk), _s()), "mia_pack_weights")
    return outs


def unpack_ohwi_grad(src_ohwi: torch.Tensor, shape, out: torch.Tensor):
    cout, cin, kh, kw = shape
    L.check(L.load().mia_pack_weight(src_ohwi.data_ptr(), out.data_ptr(), L.F32, cout, cin, kh, kw, 4, _s()),
            "mia_pack_weight(grad)")


def dropout_(x: torch.Tensor, p: float, seed: int):
    L.check(L.load().mia_dropout(x.data_ptr(), L.dtype_code(x), x.numel(), p, seed & ((1 << 64) - 1), _s()),
            "mia_dropout")


def soft_ce(logits: torch.Tensor, y: torch.Tensor, input_sigmoid: bool):
    B, C = logits.shape
    loss = torch.empty(1, dtype=torch.float32, device=logits.device)
    correct = torch.empty(1, dtype=torch.int32, device=logits.device)
    dlogits = torch.empty_like(logits)
    L.check(L.load().mia_soft_ce(logits.data_ptr(), y.data_ptr(), B, C, int(input_sigmoid), loss.data_ptr(),
                                 dlogits.data_ptr(), correct.data_ptr(), _s()), "mia_soft_ce")
    return loss[0], dlogits, correct[0]


def wait_param(p: torch.Tensor) -> None:
    """Order the current stream after a pending update of ``p``'s operand rows by another stream (the
    comm-stream all-gather of GradAllReducer fc1_exchange="shard"); no-op otherwise."""
    ev = getattr(p, "_mia_ready", None)
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)
        p._mia_ready = None


def bf16_shadow(p: torch.Tensor) -> torch.Tensor:
    """bf16 GEMM-operand copy of an f32 parameter, kept on the parameter and refreshed by FusedAdam in
    its update pass (no per-step cast).  Recast when anything else changed the parameter in place
    (``_version`` moved: load_state_dict, DDP broadcast, a non-fused optimizer)."""
    wait_param(p)
    sh = getattr(p, "_mia_bf16", None)
    if sh is not None and getattr(p, "_mia_bf16_ver", None) == p._version and sh.shape == p.shape:
        return sh
    if sh is None or sh.shape != p.shape or sh.device != p.device:
        sh = torch.empty(p.shape, dtype=torch.bfloat16, device=p.device)
    L.check(L.load().mia_cast(p.data_ptr(), L.F32, sh.data_ptr(), L.BF16, p.numel(), _s()), "mia_cast")
    p._mia_bf16 = sh
    p._mia_bf16_ver = p._version
    return sh


def cast(src: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    out = torch.empty(src.shape, dtype=dtype, device=src.device)
    L.check(L.load().mia_cast(src.data_ptr(), L.dtype_code(src), out.data_ptr(), L.dtype_code(out), src.numel(),
                              _s()), "mia_cast")
    return out


# ------------------------------------------------------------------------------------ MX-fp8
class MXTensor:
    """An MX-fp8 operand: e4m3 bytes ``q`` [rows][cols] (torch.uint8) and E8M0 scales [rows][cols / 32]."""

    def __init__(self, q: torch.Tensor, scales: torch.Tensor):
        self.q, self.scales = q, scales

    @property
    def shape(self):
        return self.q.shape


def mx_empty(rows: int, cols: int, device) -> MXTensor:
    return MXTensor(torch.empty(rows, cols, dtype=torch.uint8, device=device),
                    torch.empty(rows, cols // 32, dtype=torch.uint8, device=device))


def mx_quantize(x: torch.Tensor) -> MXTensor:
    """OCP MX-fp8 quantisation of a row-major [rows][cols] bf16/f32 tensor (mia_mx_quantize)."""
    if not x.is_cuda:
        raise RuntimeError("mx_quantize runs on the MI355X HIP kernels only (input is on CPU)")
    x = x.contiguous()
    rows, cols = x.shape
    q = torch.empty(rows, cols, dtype=torch.uint8, device=x.device)
    sc = torch.empty(rows, cols // 32, dtype=torch.uint8, device=x.device)
    L.check(L.load().mia_mx_quantize(x.data_ptr(), L.dtype_code(x), rows, cols, cols, q.data_ptr(), cols,
                                     sc.data_ptr(), _s()), "mia_mx_quantize")
    return MXTensor(q, sc)


def mx_quantize_t(x: torch.Tensor) -> MXTensor:
    """OCP MX-fp8 quantisation of the transpose of a row-major [rows][cols] bf16/f32 tensor: q [cols][rows]
    with one scale per 32 consecutive rows (mia_mx_quantize_t; the backward-data operand W^T of W[out][in])."""
    if not x.is_cuda:
        raise RuntimeError("mx_quantize_t runs on the MI355X HIP kernels only (input is on CPU)")
    x = x.contiguous()
    rows, cols = x.shape
    q = torch.empty(cols, rows, dtype=torch.uint8, device=x.device)
    sc = torch.empty(cols, rows // 32, dtype=torch.uint8, device=x.device)
    L.check(L.load().mia_mx_quantize_t(x.data_ptr(), L.dtype_code(x), rows, cols, cols, q.data_ptr(), rows,
                                       sc.data_ptr(), _s()), "mia_mx_quantize_t")
    return MXTensor(q, sc)


def gemm_mxfp8(a: MXTensor, b: MXTensor, E: L.MiaEpilogue, tag: str | None = None):
    """C = epilogue(A B^T) on MX-fp8 operands A [M][K], B [N][K] (mia_gemm_mxfp8_ex; an epilogue with column
    sums -- the x-gelu' backward-data one -- gets its partials' workspace here)."""
    M, K = a.q.shape
    N = b.q.shape[0]
    lib = L.load()
    ws = None
    if E.colsum:
        ws = workspace(lib.mia_gemm_mxfp8_workspace_bytes(M, N, 1), a.q.device, "mxgemm")
    rec = PROBE is not None and tag in PROBE
    if rec:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    L.check(lib.mia_gemm_mxfp8_ex(a.q.data_ptr(), a.scales.data_ptr(), a.q.stride(0), b.q.data_ptr(),
                                  b.scales.data_ptr(), b.q.stride(0), E, M, N, K, L.ptr(ws), _s()),
            "mia_gemm_mxfp8")
    if rec:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        nb = (M + N) * K * (1 + 1 / 32) + M * N * (4 if E.dtype == L.F32 else 2)
        PROBE[tag].append((e0, e1, 2 * M * N * K, nb))
