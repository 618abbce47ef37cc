"""GPU: fused clip + Adam (mia_clip_adam) against torch.nn.utils.clip_grad_norm_ + torch.optim.Adam
(reference engine.py:299-310, base_training.yaml:51,56-59), and the bf16 operand copies it refreshes."""
import pytest
import torch

from src.miaudio import kernels as K
from src.training.optim import FusedAdam

pytestmark = pytest.mark.gpu


def test_adam_refreshes_bf16_shadow(cuda):
    g = torch.Generator().manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(n, generator=g).to(cuda)) for n in (1003, 4096, 7)]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    sh0 = K.bf16_shadow(ps[1])  # live copy on one tensor only
    assert torch.equal(sh0, ps[1].detach().to(torch.bfloat16))
    opt = FusedAdam(ps, lr=1e-2, weight_decay=1e-4, clip=1.0)
    ropt = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-4)
    for it in range(3):
        for p, r in zip(ps, ref):
            gr = torch.randn(p.shape, generator=g).to(cuda)
            p.grad, r.grad = gr.clone(), gr.clone()
        opt.step()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        ropt.step()
        torch.cuda.synchronize()
        for p, r in zip(ps, ref):
            assert torch.allclose(p, r, rtol=1e-5, atol=1e-6)
        sh = K.bf16_shadow(ps[1])
        assert sh.data_ptr() == sh0.data_ptr()  # no recast: Adam wrote it
        assert torch.equal(sh, ps[1].detach().to(torch.bfloat16))
    with torch.no_grad():
        ps[1].mul_(2.0)  # any other in-place change invalidates the copy
    assert torch.equal(K.bf16_shadow(ps[1]), ps[1].detach().to(torch.bfloat16))


def test_adam_precomputed_sqsum(cuda):
    """A gradient tagged with its GEMM's per-tile sums of squares (K.tag_sqsum) is not re-read by the
    norm pass; the step matches torch's clip + Adam, and a stale tag (gradient written since) is
    ignored."""
    from src.miaudio import lib as L
    g = torch.Generator().manual_seed(3)
    M, N, Kd = 256, 384, 128
    ps = [torch.nn.Parameter((0.05 * torch.randn(M, N, generator=g)).to(cuda)),
          torch.nn.Parameter(torch.randn(77, generator=g).to(cuda))]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=1e-4, clip=0.5)
    ropt = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-4)
    for it in range(3):
        a = torch.randn(Kd, M, generator=g).to(torch.bfloat16).to(cuda)
        b = torch.randn(Kd, N, generator=g).to(torch.bfloat16).to(cuda)
        dW = torch.empty(M, N, dtype=torch.float32, device=cuda)
        sq = K.sqsum_slots(dW, M, N)
        K.gemm(K.dense(a, L.RC, Kd, M), K.dense(b, L.RC, Kd, N), K.epilogue(dW, N, sqsum=sq), M, N, Kd, L.BF16)
        K.tag_sqsum(ps[0], dW, sq)
        if it == 2:
            dW.mul_(0.5)  # written after the GEMM: the tag no longer describes it
            assert K.valid_sqsum(ps[0], dW) is None
        else:
            assert K.valid_sqsum(ps[0], dW) is sq
            assert K.valid_sqsum(ps[0], dW.clone()) is None
        gb = torch.randn(77, generator=g).to(cuda)
        ps[0].grad, ps[1].grad = dW, gb.clone()
        ref[0].grad, ref[1].grad = dW.clone(), gb.clone()
        opt.step()
        total = torch.nn.utils.clip_grad_norm_(ref, 0.5)
        ropt.step()
        torch.cuda.synchronize()
        assert abs(float(opt.last_total_norm) - float(total)) <= 1e-5 * float(total)
        for p, r in zip(ps, ref):
            assert torch.allclose(p, r, rtol=1e-5, atol=1e-6)
        assert ps[0]._mia_sqsum is None  # consumed


def test_adam_per_parameter_steps_and_table_reuse(cuda):
    """torch.optim.Adam counts steps per parameter: a parameter without a gradient in some step is
    skipped and its bias corrections lag the others'.  The fused step takes per-tensor counts then
    (mia_clip_adam's ``steps`` table) and matches torch; with unchanged pointers the device pointer
    table is not rebuilt."""
    g = torch.Generator().manual_seed(5)
    ps = [torch.nn.Parameter(torch.randn(n, generator=g).to(cuda)) for n in (515, 64, 3)]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=1e-4, clip=0.0)
    ropt = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-4)
    grads = [torch.empty_like(p) for p in ps]  # fixed storage: the table key stays the same
    for it in range(5):
        for i, (p, r) in enumerate(zip(ps, ref)):
            if it == 1 and i == 1:  # parameter 1 misses step 1
                p.grad = r.grad = None
                continue
            grads[i].copy_(torch.randn(p.shape, generator=g).to(cuda))
            p.grad, r.grad = grads[i], grads[i].clone()
        opt.step()
        ropt.step()
        torch.cuda.synchronize()
        for p, r in zip(ps, ref):
            assert torch.allclose(p, r, rtol=1e-5, atol=1e-6), it
    assert [int(opt.state[p]["step"]) for p in ps] == [5, 4, 5]
    # builds: step 0 (3 tensors), step 1 (2 tensors), steps 2-4 (per-tensor counts, same pointers)
    assert opt.table_builds == 3
