"""GPU: the deferred FC1 weight gradient (K.defer_weight_grad + mia_gemm_sqsum_only + mia_gemm_adam).

On one GPU under FusedAdam, EnvNet-v2's FC1 weight gradient (envnet_v2.py:51, 4096 x 84480 f32) is never
written: the backward leaves its per-tile sums of squares and FusedAdam.step recomputes the product inside
the Adam GEMM.  The same kernel main loop and the same Adam arithmetic run in both forms, so two EnvNetV2
(bf16) runs from the same weights -- one deferring, one with the gradient materialised (FusedAdam built
after the backward, so the model sees no fused optimizer) -- must end in bit-identical parameters, Adam
moments and global grad norms after every step."""
import pytest
import torch

from oracle.synth import synth_waveform
from tests._util import envnet_with_hash_params

pytestmark = pytest.mark.gpu


def _run(cuda, defer: bool, steps: int, x, y):
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    m = envnet_with_hash_params(cuda, compute_dtype="bf16").train()
    opt = FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-4, clip=1.0)
    if not defer:
        for p in m.parameters():
            p._mia_fused_adam = False
    norms, deferred = [], []
    for _ in range(steps):
        z = m(x)
        _, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=False)
        z.backward(dz)
        fc1 = dict(m.named_parameters())["classifier.1.weight"]
        assert (fc1.grad is None) == defer
        opt.step()
        opt.zero_grad(set_to_none=True)
        norms.append(float(opt.last_total_norm))
        deferred.append(opt.last_deferred)
    torch.cuda.synchronize()
    state = {n: (p.detach().clone(), opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone())
             for n, p in m.named_parameters()}
    return norms, deferred, state


def test_deferred_fc1_wgrad_bit_identical(cuda):
    B = 64
    x = torch.from_numpy(synth_waveform(33, B, 220_500)[:, None, :]).to(cuda)
    y = torch.zeros(B, 50, device=cuda)
    y[torch.arange(B), torch.arange(B) % 50] = 1.0
    n1, d1, s1 = _run(cuda, True, 3, x, y)
    n0, d0, s0 = _run(cuda, False, 3, x, y)
    assert d1 == [1, 1, 1] and d0 == [0, 0, 0]
    assert n1 == n0, (n1, n0)
    for name in s0:
        for a, b in zip(s1[name], s0[name]):
            assert torch.equal(a, b), name


def test_deferred_grad_pending_twice_raises(cuda):
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    m = envnet_with_hash_params(cuda, compute_dtype="bf16").train()
    FusedAdam(m.parameters(), lr=1e-3)
    x = torch.from_numpy(synth_waveform(34, 64, 220_500)[:, None, :]).to(cuda)
    y = torch.zeros(64, 50, device=cuda)
    y[:, 0] = 1.0
    z = m(x)
    _, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=False)
    z.backward(dz)
    z = m(x)
    with pytest.raises(RuntimeError, match="deferred weight gradient is still pending"):
        z.backward(dz)
