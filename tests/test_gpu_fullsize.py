"""GPU: parity at the BENCHED sizes (verdict r3, What's missing 2).

The oracle-sized tests elsewhere run B <= 64.  Several paths are only taken at full size: the deferred FC1
weight gradient at B = 256, the persistent kernels' item splits over 256 clips, the 256x256 GEMM at
M = 421 120 token rows, the attention grid at B*H = 3 072, the shape-dependent split-K choices.  Here:

* one EnvNetV2 bf16 train step at B = 256 (FusedAdam alive, so FC1's gradient is deferred into the Adam
  GEMM) against the oracle step on the same GPU under bf16 autocast and in f32, with the self-calibrated
  bounds of tests/test_gpu_e2e_bf16.py (reference: src/models/envnet_v2.py:76-85);
* one ASTModel depth-12 bf16 train step at B = 32 the same way (reference: src/models/ast.py:50-63);
* the attention kernels at B = 256, H = 12, N = 1645 (the benched grid) against float64 on sampled
  (clip, head) pairs, forward and backward (timm Attention, ast.py:38,60-61);
* batch independence at full size: eval-mode EnvNet, AST bf16 and AST fp8-mixed outputs of clips 0-3 at
  B = 256 against a B = 4 run of the same clips (eval BatchNorm uses running statistics and nothing else
  crosses clips, so only kernel choices that depend on the batch -- tile / split shapes of the FC GEMMs --
  may change a summation order; tolerances below).
"""
import math
import os
import time

import pytest
import torch

from oracle import ast as oast
from oracle import envnet as oenv
from oracle.synth import hash_uniform, synth_waveform
from tests._util import envnet_with_hash_params, hash_params
from tests.test_gpu_e2e_bf16 import _check, _oracle_step, _rel

pytestmark = pytest.mark.gpu
_T0 = time.time()


def _t(msg):
    print(f"[fullsize {time.time() - _T0:7.1f}s] {msg}", flush=True)


def _labels(cuda, B, seed):
    g = torch.Generator().manual_seed(seed)
    y = torch.zeros(B, 50)
    y[torch.arange(B), torch.randint(0, 50, (B,), generator=g)] = 1.0
    return y.to(cuda)


def test_envnet_bf16_step_b256_deferred_fc1_vs_autocast_oracle(cuda):
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    B = 256
    x = torch.from_numpy(synth_waveform(41, B, 220_500)[:, None, :]).to(cuda)
    y = _labels(cuda, B, 41)
    m = envnet_with_hash_params(cuda, compute_dtype="bf16").train()
    names = [n for n, _ in m.named_parameters()]
    opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)  # built first: FC1 is deferred
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    z = m(x)
    loss, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=False)
    z.backward(dz)
    assert dict(m.named_parameters())["classifier.1.weight"].grad is None  # the deferred path at B = 256
    opt.step()
    assert opt.last_deferred == 1
    total = float(opt.last_total_norm)
    deltas = {n: p.detach() - before[n] for n, p in m.named_parameters()}
    zz, loss = z.detach().float(), float(loss)
    _t("envnet b256: HIP step done")
    del z, dz, m, opt, before
    torch.cuda.empty_cache()

    def ref(autocast):
        p = {k: torch.from_numpy(v.copy()).to(cuda) for k, v in hash_params(100).items()}
        for n in names:
            p[n].requires_grad_(True)
        r = _oracle_step(p, names, lambda q: oenv.forward(q, x, training=True, dropout_p=0.0), y, autocast)
        torch.cuda.empty_cache()
        _t(f"envnet b256: oracle step done (autocast={autocast})")
        return r

    r16, r32 = ref(True), ref(False)
    _check("envnet-b256", zz, loss, total, deltas, {}, r16, r32,
           tol={"logits": 0.17, "logits_f32": 0.12, "loss": 0.03, "gradnorm": 0.03, "sign": 0.95})


def _ast(cuda, cd, depth, st, hw, hb):
    from src.models.ast import ASTModel
    m = ASTModel(num_classes=50, compute_dtype=cd, depth=depth)
    m.load_vit_state(st)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    return m.to(cuda)


def test_ast_depth12_bf16_step_b32_vs_autocast_oracle(cuda):
    os.environ["MIA_QUIET"] = "1"
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    B = 32
    st = oast.deit_hash_state(300)
    hw, hb = oast.head_hash(901, 50)
    m = _ast(cuda, "bf16", 12, st, hw, hb).train()
    x = torch.from_numpy(hash_uniform(33, (B, 128, 1379))).to(cuda)
    y = _labels(cuda, B, 33)
    pmap = dict(m.named_parameters())
    before = {n: p.detach().clone() for n, p in pmap.items()}
    probs = m(x)
    loss, dp, _ = K.soft_ce(probs.detach().float().contiguous(), y, input_sigmoid=False)
    probs.backward(dp)
    opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    opt.step()
    total = float(opt.last_total_norm)
    deltas = {n: p.detach() - before[n] for n, p in pmap.items()}
    pp, loss = probs.detach().float(), float(loss)
    _t("ast d12 b32: HIP step done")
    del probs, dp, m, opt, before, pmap
    torch.cuda.empty_cache()
    ref_names = list(oast.model_params(st, hw, hb))
    assert set(ref_names) == set(deltas), set(ref_names) ^ set(deltas)

    def ref(autocast):
        p = {k: v.to(cuda).requires_grad_(True) for k, v in oast.model_params(st, hw, hb).items()}
        r = _oracle_step(p, ref_names, lambda q: oast.forward(q, x), y, autocast)
        torch.cuda.empty_cache()
        _t(f"ast d12 b32: oracle step done (autocast={autocast})")
        return r

    r16, r32 = ref(True), ref(False)
    # depth 12 instead of 2: the fixed bounds are the depth-2 test's widened 3x; the self-calibrated bounds
    # (HIP no further from f32 than 1.25x autocast's distance) are the same
    _check("ast-d12-b32", pp, loss, total, deltas, {}, r16, r32,
           tol={"logits": 0.045, "loss": 0.006, "gradnorm": 0.018, "sign": 0.97})


def test_ast_depth2_bf16_step_b256_vs_autocast_oracle(cuda):
    """The AST bf16 training step at the benched batch (B = 256: the full attention grid, the GEMM shapes of the
    bench) with two transformer blocks, against the oracle's autocast-bf16 and f32 steps (torch on the same
    GPU): logits, loss, clip norm and the Adam update directions, with the depth-2 bounds widened 2x for the
    larger batch and the self-calibrated bounds of _check."""
    os.environ["MIA_QUIET"] = "1"
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    B = 256
    st = oast.deit_hash_state(300, depth=2)
    hw, hb = oast.head_hash(901, 50)
    m = _ast(cuda, "bf16", 2, st, hw, hb).train()
    x = torch.from_numpy(hash_uniform(35, (B, 128, 1379))).to(cuda)
    y = _labels(cuda, B, 35)
    pmap = dict(m.named_parameters())
    before = {n: p.detach().clone() for n, p in pmap.items()}
    probs = m(x)
    loss, dp, _ = K.soft_ce(probs.detach().float().contiguous(), y, input_sigmoid=False)
    probs.backward(dp)
    opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    opt.step()
    total = float(opt.last_total_norm)
    deltas = {n: p.detach() - before[n] for n, p in pmap.items()}
    pp, loss = probs.detach().float(), float(loss)
    _t("ast d2 b256: HIP step done")
    del probs, dp, m, opt, before, pmap
    torch.cuda.empty_cache()
    ref_names = list(oast.model_params(st, hw, hb, depth=2))

    def ref(autocast):
        p = {k: v.to(cuda).requires_grad_(True) for k, v in oast.model_params(st, hw, hb, depth=2).items()}
        r = _oracle_step(p, ref_names, lambda q: oast.forward(q, x, depth=2), y, autocast)
        torch.cuda.empty_cache()
        _t(f"ast d2 b256: oracle step done (autocast={autocast})")
        return r

    r16, r32 = ref(True), ref(False)
    _check("ast-d2-b256", pp, loss, total, deltas, {}, r16, r32,
           tol={"logits": 0.03, "loss": 0.004, "gradnorm": 0.012, "sign": 0.98})


def test_attention_benched_grid_b256_h12(cuda):
    """mia_attn_fwd_save_q / mia_attn_bwd_saved_q (the training form) and the one-pass / fused backwards over
    the whole benched grid (B*H = 3 072 (clip, head) pairs of 1 645 tokens); every pair against float64, with
    the bounds of test_gpu_ast.test_attention_fwd_bwd (bf16)."""
    from src.miaudio import lib as L
    B, N, H = 256, 1645, 12
    g = torch.Generator(device=cuda).manual_seed(5)
    qkv = (torch.randn(B * N, 3 * H * 64, generator=g, device=cuda) * 1.5).to(torch.bfloat16)
    dout = torch.randn(B * N, H * 64, generator=g, device=cuda).to(torch.bfloat16)
    lib, s = L.load(), L.stream_ptr()
    out = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device=cuda)
    lse = torch.empty(B, H, N, device=cuda)
    work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=cuda)
    dq = torch.full_like(qkv, float("nan"))
    L.check(lib.mia_attn_fwd_save_q(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), None, None, work.data_ptr(), B,
                                    N, H, 0.125, s), "fwd_save_q")
    L.check(lib.mia_attn_bwd_saved_q(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dq.data_ptr(),
                                     work.data_ptr(), B, N, H, 0.125, s), "bwd_saved_q")
    torch.cuda.synchronize()
    assert torch.isfinite(dq.float()).all() and torch.isfinite(out.float()).all()
    # the fused one-pass form over the same grid (7 key blocks per (b, h) handing dQ on): error word 0 and
    # the two-kernel result up to summation order
    dq2 = torch.full_like(qkv, float("nan"))
    L.check(lib.mia_attn_bwd_fused(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dq2.data_ptr(),
                                   work.data_ptr(), B, N, H, 0.125, 1, s), "bwd_fused")
    torch.cuda.synchronize()
    off = int(lib.mia_attn_bwd_error_offset(B, N, H))
    assert int(work[off:off + 4].view(torch.int32).item()) == 0
    e = float((dq2.float() - dq.float()).abs().max() / dq.float().abs().max())
    assert e < 5e-3, e
    # the one-pass backward (7 key blocks of 256 per (b, h) handing dQ on at lag 3): the sticky error word
    # still 0, bit-identical from call to call, the two-kernel result up to summation order
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    chain = torch.empty(int(lib.mia_attn_bwd_chain_bytes(B, N, H)), dtype=torch.uint8, device=cuda)
    ones = []
    for _ in range(2):
        d1 = torch.full_like(qkv, float("nan"))
        L.check(lib.mia_attn_bwd_onepass(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                         d1.data_ptr(), work.data_ptr(), chain.data_ptr(), err.data_ptr(), B, N, H,
                                         0.125, 1, s), "bwd_onepass")
        ones.append(d1)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(ones[0], ones[1])
    e = float((ones[0].float() - dq.float()).abs().max() / dq.float().abs().max())
    assert e < 5e-3, e
    one = ones[0]
    del chain, ones
    # EVERY (clip, head) pair of the grid against float64 (computed on the GPU, one clip's 12 heads at a
    # time): forward output and lse, and the three gradients of both the two-kernel and the one-pass form,
    # each within the bounds of test_gpu_ast.test_attention_fwd_bwd (max |error| / max |reference| per pair)
    qkv4 = qkv.view(B, N, 3, H, 64)
    worst = {"out": 0.0, "lse": 0.0, "two": 0.0, "one": 0.0}
    for b in range(B):
        q, k, v = (qkv4[b, :, i].permute(1, 0, 2).double().requires_grad_(True) for i in range(3))
        s_ = (q @ k.transpose(1, 2)) / 8.0
        o = torch.softmax(s_, -1) @ v
        o.backward(dout.view(B, N, H, 64)[b].permute(1, 0, 2).double())
        with torch.no_grad():
            got = out.view(B, N, H, 64)[b].permute(1, 0, 2).double()
            worst["out"] = max(worst["out"], float(((got - o).abs().amax((1, 2)) / o.abs().amax((1, 2))).max()))
            # lse relative to the clip's score range: Q' = bf16(q scale log2 e) rounds every score by up to
            # 2^-9 of its size (here |S| reaches ~12; test_attention_fwd_bwd's 2e-2 absolute is for |S| ~ 4)
            lref = torch.logsumexp(s_, -1)
            worst["lse"] = max(worst["lse"], float((lse[b].double() - lref).abs().max() / s_.abs().max()))
            for name, d in (("two", dq), ("one", one)):
                d4 = d.view(B, N, 3, H, 64)[b]
                for i, ref in enumerate((q.grad, k.grad, v.grad)):
                    e = (d4[:, i].permute(1, 0, 2).double() - ref).abs().amax((1, 2)) / ref.abs().amax((1, 2))
                    worst[name] = max(worst[name], float(e.max()))
        del q, k, v, s_, o
    print("benched grid, all 3 072 (clip, head) pairs vs float64, worst per-pair max-relative (lse: absolute "
          "error / max |S| of the clip):", worst)
    assert worst["out"] < 2e-2 and worst["lse"] < 4e-3, worst
    assert worst["two"] < 6e-2 and worst["one"] < 6e-2, worst


def test_envnet_eval_batch_independence_b256(cuda):
    B = 256
    m = envnet_with_hash_params(cuda, compute_dtype="bf16").eval()
    x = torch.from_numpy(synth_waveform(43, B, 220_500)[:, None, :]).to(cuda)
    with torch.no_grad():
        z256 = m(x)[:4].float()
        z4 = m(x[:4].contiguous()).float()
    e = _rel(z256, z4)
    print(f"envnet eval B=256 vs B=4: rel-L2 {e:.3g}, max |d| {float((z256 - z4).abs().max()):.3g}")
    # clips never mix in eval; the FC GEMMs' kernel / split choice depends on B (M = rows), so their sums may
    # be ordered differently: one bf16 rounding of the logits at most
    assert e < 8e-3, e
    assert torch.equal(z256.argmax(1), z4.argmax(1))


@pytest.mark.parametrize("cd", ["bf16", "fp8"])
def test_ast_eval_batch_independence_b256(cuda, cd):
    os.environ["MIA_QUIET"] = "1"
    B = 256
    st = oast.deit_hash_state(300)
    hw, hb = oast.head_hash(901, 50)
    m = _ast(cuda, cd, 12, st, hw, hb).eval()
    x = torch.from_numpy(hash_uniform(34, (B, 128, 1379))).to(cuda)
    with torch.no_grad():
        p256 = m(x)[:4].float()
        torch.cuda.empty_cache()
        p4 = m(x[:4].contiguous()).float()
    e = _rel(p256, p4)
    print(f"ast[{cd}] eval B=256 vs B=4: rel-L2 {e:.3g}, max |d| {float((p256 - p4).abs().max()):.3g}")
    # every token row is computed independently of the batch (LayerNorm per row, attention per (clip, head),
    # MX blocks along K within a row): the 256-row GEMM tiles only change which rows share a tile
    assert e < 2e-3, e
    assert torch.equal(p256.argmax(1), p4.argmax(1))
    del m
    torch.cuda.empty_cache()
    assert math.isfinite(e)
