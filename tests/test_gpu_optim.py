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
