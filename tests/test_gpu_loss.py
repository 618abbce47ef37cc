"""GPU: the fused soft-label loss (mia_soft_ce) and dropout (mia_dropout) on the benched step.

* soft-CE: loss, dlogits and the argmax hit count against the oracle's autograd in float64 of
  ``-(y * log(softmax(z) + 1e-8)).sum(1).mean()`` (reference engine.py:175-176), for logits
  (EnvNet) and for sigmoid probabilities (AST returns sigmoid(head(.)), ast.py:63; the input_sigmoid
  variant folds that sigmoid's backward in), over one-hot, BC-mixed and same-class-Mixup labels.
* dropout (nn.Dropout(0.5), envnet_v2.py:53,57): keep rate ~ 1 - p, kept values scaled by exactly
  1/(1-p), deterministic per seed; inside EnvNetV2 the backward mask is the forward mask (the FC-head
  gradients equal a float64 restatement built from the captured post-dropout activations)."""
import numpy as np
import pytest
import torch

from oracle import train as otrain
from oracle.synth import synth_waveform
from tests._util import envnet_with_hash_params

pytestmark = pytest.mark.gpu


def _labels(B, C, g):
    y = torch.zeros(B, C, dtype=torch.float64)
    lab = torch.randint(0, C, (B,), generator=g)
    y[torch.arange(B), lab] = 1.0
    r = torch.rand(B, generator=g, dtype=torch.float64)
    other = (lab + 1 + torch.randint(0, C - 1, (B,), generator=g)) % C
    for b in range(B):
        if b % 3 == 1:    # BC mixing: r / 1 - r on two different classes
            y[b, lab[b]] = r[b]
            y[b, other[b]] = 1 - r[b]
        elif b % 3 == 2:  # Mixup with a same-class partner: only 1 - lam survives
            y[b, lab[b]] = 1 - r[b]
    return y


@pytest.mark.parametrize("input_sigmoid", [False, True])
@pytest.mark.parametrize("B,C", [(7, 50), (256, 50), (33, 10)])
def test_soft_ce_loss_and_grad(cuda, B, C, input_sigmoid):
    from src.miaudio import kernels as K
    g = torch.Generator().manual_seed(B * 100 + C)
    logits = (torch.randn(B, C, generator=g) * 4).float()
    y = _labels(B, C, g)
    loss, dlogits, correct = K.soft_ce(logits.to(cuda), y.float().to(cuda), input_sigmoid=input_sigmoid)
    z = logits.double().requires_grad_(True)
    ref = otrain.soft_ce(torch.sigmoid(z) if input_sigmoid else z, y)
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 2e-6 * max(1.0, abs(float(ref)))
    torch.testing.assert_close(dlogits.cpu().double(), z.grad, rtol=1e-4, atol=1e-7)
    assert int(correct) == int((logits.argmax(1) == y.argmax(1)).sum())


def test_soft_ce_engine_autograd_path(cuda):
    """LitClassifier._soft_loss -> _FusedSoftCE: loss value and the gradient autograd hands back."""
    from src.training.engine import _FusedSoftCE
    g = torch.Generator().manual_seed(11)
    logits = torch.randn(16, 50, generator=g).to(cuda).requires_grad_(True)
    y = _labels(16, 50, g).float().to(cuda)
    loss = _FusedSoftCE.apply(logits, y)
    (2.5 * loss).backward()
    z = logits.detach().cpu().double().requires_grad_(True)
    ref = otrain.soft_ce(z, y.cpu().double())
    (2.5 * ref).backward()
    assert abs(float(loss) - float(ref)) < 1e-5
    torch.testing.assert_close(logits.grad.cpu().double(), z.grad, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dropout_keep_rate_scale_and_determinism(cuda, dtype):
    from src.miaudio import kernels as K
    n = 1 << 20
    base = (torch.rand(n, generator=torch.Generator().manual_seed(2)) + 1.0).to(dtype).to(cuda)
    for p in (0.5, 0.2):
        x = base.clone()
        K.dropout_(x, p, seed=1234)
        kept = x != 0
        rate = float(kept.float().mean())
        assert abs(rate - (1 - p)) < 4e-3, (p, rate)
        scale = torch.tensor(1.0 / (1.0 - p), dtype=torch.float32)
        exp = (base.float() * scale.to(cuda)).to(dtype)
        assert torch.equal(x[kept], exp[kept])
        x2 = base.clone()
        K.dropout_(x2, p, seed=1234)
        assert torch.equal(x, x2)
        x3 = base.clone()
        K.dropout_(x3, p, seed=1235)
        assert not torch.equal(x3 != 0, kept)
    x = base.clone()
    K.dropout_(x, 0.0, seed=1)
    assert torch.equal(x, base)


def test_envnet_dropout_backward_mask_is_forward_mask(cuda):
    """f32 EnvNetV2 with Dropout(0.5) in train mode: the classifier gradients equal a float64 backward
    through the captured post-ReLU/dropout activations h1, h2 with masks (h != 0) and scale 2."""
    from src.miaudio import kernels as K
    m = envnet_with_hash_params(cuda, dropout=0.5).train()
    m._debug_capture = True
    x = torch.from_numpy(synth_waveform(21, 2, 220_500)[:, None, :]).to(cuda)
    z = m(x)
    s = m._debug
    h0, h1, h2 = s["flat"].double(), s["h1"].double(), s["h2"].double()
    for h in (h1, h2):
        frac = float((h == 0).double().mean())
        assert 0.5 <= frac < 0.95  # dropout zeros (~half) plus ReLU zeros
    y = torch.zeros(2, 50, device=cuda)
    y[0, 3] = 1.0
    y[1, 7] = 1.0
    _, dz, _ = K.soft_ce(z.detach(), y, input_sigmoid=False)
    z.backward(dz)
    W2, W3 = m.classifier[4].weight.detach().double(), m.classifier[7].weight.detach().double()
    dzd = dz.double()
    dW3 = dzd.t() @ h2
    d2 = (dzd @ W3) * (h2 != 0) * 2.0
    dW2 = d2.t() @ h1
    d1 = (d2 @ W2) * (h1 != 0) * 2.0
    rows = torch.arange(0, 4096, 97, device=cuda)
    dW1 = d1[:, rows].t() @ h0
    for got, ref, name in ((m.classifier[7].weight.grad, dW3, "fc3"), (m.classifier[4].weight.grad, dW2, "fc2"),
                           (m.classifier[1].weight.grad[rows], dW1, "fc1")):
        err = float((got.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < 1e-4, (name, err)
    db = d2.sum(0)
    torch.testing.assert_close(m.classifier[4].bias.grad.double(), db, rtol=1e-4, atol=1e-5 * float(db.abs().max()))
