"""CPU: the OCP MX-fp8 restatement (oracle/mx.py) obeys the format's defining properties -- the shared
exponent rule, element rounding within half an E4M3 step of the scaled value, saturation at 448, zero
blocks -- on hand-built blocks (parity with the reference unpinned: the reference has no fp8 path)."""
import torch

from oracle import mx as omx


def test_scale_rule_and_rounding():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 256, generator=g) * torch.pow(2.0, torch.randint(-20, 20, (64, 1), generator=g).float())
    q, s = omx.quantize(x)
    blk = x.reshape(64, 8, 32)
    amax = blk.abs().amax(dim=2)
    e = torch.floor(torch.log2(amax)) - 8
    assert torch.equal(s.to(torch.int64) - 127, e.to(torch.int64))
    deq = omx.dequantize(q, s).reshape(64, 8, 32)
    # e4m3 keeps 3 mantissa bits: |P - x/X| <= 2^-4 * 2^floor(log2|x/X|) (half a step), X = 2^e
    y = blk.double() / torch.pow(2.0, e.double())[..., None]
    step = torch.pow(2.0, torch.floor(torch.log2(y.abs().clamp_min(2.0 ** -9))) - 3)
    err = (deq / torch.pow(2.0, e.double())[..., None] - y).abs()
    sat = y.abs() > 448
    assert bool(((err <= step / 2 + 1e-12) | sat).all())


def test_saturation_and_zero_block():
    x = torch.zeros(2, 32)
    x[1] = torch.linspace(-511.0, 511.0, 32)  # amax 511 -> e = 0: elements past 448 clamp
    q, s = omx.quantize(x)
    assert int(s[0, 0]) == 0 and bool((q[0] == 0).all())
    assert int(s[1, 0]) == 127
    deq = omx.dequantize(q, s)[1]
    assert float(deq.max()) == 448.0 and float(deq.min()) == -448.0


def test_gemm_is_dequantised_product():
    g = torch.Generator().manual_seed(1)
    a, b = torch.randn(5, 64, generator=g), torch.randn(3, 64, generator=g)
    qa, sa = omx.quantize(a)
    qb, sb = omx.quantize(b)
    ref = omx.dequantize(qa, sa) @ omx.dequantize(qb, sb).T
    assert torch.allclose(omx.gemm(qa, sa, qb, sb), ref)
    assert float((ref - a.double() @ b.double().T).abs().max()) < 0.2 * float(ref.abs().max())
