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
            p._mia_fused_adam = None
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
    opt = FusedAdam(m.parameters(), lr=1e-3)  # noqa: F841  (alive: the model defers to it)
    x = torch.from_numpy(synth_waveform(34, 64, 220_500)[:, None, :]).to(cuda)
    y = torch.zeros(64, 50, device=cuda)
    y[:, 0] = 1.0
    z = m(x)
    _, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=False)
    z.backward(dz)
    z = m(x)
    with pytest.raises(RuntimeError, match="deferred weight gradient is still pending"):
        z.backward(dz)


def test_torch_adam_after_fused_adam_updates_fc1(cuda):
    """a torch.optim.Adam built after a FusedAdam (still alive) on the same parameters must update
    FC1 on its first step: the global step pre-hook materialises the deferred gradient into p.grad with the
    same GEMM, and the parameter stops deferring.  Its gradient equals a run where no FusedAdam ever existed."""
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    x = torch.from_numpy(synth_waveform(35, 64, 220_500)[:, None, :]).to(cuda)
    y = torch.zeros(64, 50, device=cuda)
    y[torch.arange(64), torch.arange(64) % 50] = 1.0
    grads = []
    for with_fused in (True, False):
        m = envnet_with_hash_params(cuda, compute_dtype="bf16").train()
        fused = FusedAdam(m.parameters(), lr=1e-3) if with_fused else None  # noqa: F841
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        fc1 = dict(m.named_parameters())["classifier.1.weight"]
        before = fc1.detach().clone()
        z = m(x)
        _, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=False)
        z.backward(dz)
        assert (fc1.grad is None) == with_fused  # deferred while the FusedAdam is alive
        opt.step()
        assert fc1.grad is not None and getattr(fc1, "_mia_deferred", None) is None
        assert not torch.equal(fc1.detach(), before)
        assert not K.defers_to_fused_adam(fc1)  # taken over by torch's Adam
        grads.append(fc1.grad.detach().clone())
    torch.testing.assert_close(grads[0], grads[1], rtol=1e-5, atol=1e-9)


def test_fused_adam_collected_stops_deferring(cuda):
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    m = envnet_with_hash_params(cuda, compute_dtype="bf16").train()
    opt = FusedAdam(m.parameters(), lr=1e-3)
    fc1 = dict(m.named_parameters())["classifier.1.weight"]
    assert K.defers_to_fused_adam(fc1)
    del opt
    import gc
    gc.collect()
    assert not K.defers_to_fused_adam(fc1)
