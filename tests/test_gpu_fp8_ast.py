"""GPU: trainer.precision=fp8-mixed (north_star config 5) end to end -- one AST depth-2 train step with the
block linears' forward GEMMs on MX-fp8 operands (mia_mx_quantize + mia_gemm_mxfp8), held against the f32
oracle step and against the bf16 HIP step on the same inputs.  The reference has no fp8 path, so parity is
unpinned; the yardstick is an MX-fp8 EMULATION of the same step -- the oracle AST under bf16 autocast with
its four block linears replaced by oracle.mx.MXLinear (forward on the MX values of the bf16 activation and
the f32 weight, straight-through bf16 backward, the HIP path's recipe).  The HIP fp8 step must be as close
to the f32 step as that emulation is (self-calibrating bounds, as the bf16 e2e tests do against autocast),
and its Adam directions must agree with the f32 step's."""
import os

import pytest
import torch

from oracle import ast as oast
from oracle import mx as omx
from oracle.synth import hash_uniform
from tests.test_gpu_e2e_bf16 import _oracle_step, _rel

pytestmark = pytest.mark.gpu


def _hip_step(cuda, cd, st, hw, hb, x, y):
    from src.miaudio import kernels as K
    from src.models.ast import ASTModel
    from src.training.optim import FusedAdam
    m = ASTModel(num_classes=50, compute_dtype=cd, depth=2)
    m.load_vit_state(st)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    m = m.to(cuda).train()
    probs = m(x)
    loss, dp, _ = K.soft_ce(probs.detach().float().contiguous(), y, input_sigmoid=False)
    probs.backward(dp)
    pmap = dict(m.named_parameters())
    grads = {n: p.grad.detach().clone() for n, p in pmap.items()}
    before = {n: p.detach().clone() for n, p in pmap.items()}
    opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    opt.step()
    deltas = {n: p.detach() - before[n] for n, p in pmap.items()}
    return probs.detach().float(), float(loss), grads, float(opt.last_total_norm), deltas


def test_ast_depth2_fp8_mixed_train_step(cuda):
    os.environ["MIA_QUIET"] = "1"
    B = 4
    st = oast.deit_hash_state(300, depth=2)
    hw, hb = oast.head_hash(901, 50)
    x = torch.from_numpy(hash_uniform(32, (B, 128, 1379))).to(cuda)
    y = torch.zeros(B, 50, device=cuda)
    y[0, 3], y[1, 5], y[1, 2], y[2, 49], y[3, 0], y[3, 1] = 1.0, 0.6, 0.4, 1.0, 0.3, 0.7
    z8, l8, g8, t8, d8 = _hip_step(cuda, "fp8", st, hw, hb, x, y)
    names = list(oast.model_params(st, hw, hb, depth=2))

    def ref(lin, autocast):
        p = {k: v.to(cuda).requires_grad_(True) for k, v in oast.model_params(st, hw, hb, depth=2).items()}
        return _oracle_step(p, names, lambda q: oast.forward(q, x, depth=2, lin=lin), y, autocast)

    z32, l32, g32, t32, d32 = ref(torch.nn.functional.linear, False)
    zo, lo, go, to, do = ref(omx.mx_linear, True)
    gcat = lambda g: torch.cat([g[n].flatten().float() for n in names])  # noqa: E731
    e8, eo = _rel(z8, z32), _rel(zo, z32)
    gn8, gno = abs(t8 - t32) / t32, abs(to - t32) / t32
    gr8, gro = _rel(gcat(g8), gcat(g32)), _rel(gcat(go), gcat(g32))
    agree, n = 0, 0
    for name in names:
        g = g32[name].flatten()
        msk = g.abs() > 0.05 * g.abs().max()
        agree += int((torch.sign(d8[name].flatten()[msk]) == torch.sign(d32[name].flatten()[msk])).sum())
        n += int(msk.sum())
    frac = agree / max(n, 1)
    print(f"[fp8] probs rel-L2 vs f32: hip {e8:.4f}, MX emulation {eo:.4f} (hip vs emulation {_rel(z8, zo):.4f}); "
          f"loss {l8:.5f} / {lo:.5f} / f32 {float(l32):.5f}; grad norm rel err hip {gn8:.4f}, emulation {gno:.4f}; "
          f"grads rel-L2 hip {gr8:.4f}, emulation {gro:.4f}; Adam sign agreement with f32 {frac:.4f} over {n}")
    assert e8 <= 1.5 * eo + 2e-3, (e8, eo)
    assert abs(l8 - float(l32)) <= 2 * abs(lo - float(l32)) + 1e-3
    assert gn8 <= 1.5 * gno + 5e-3, (gn8, gno)
    assert gr8 <= 1.5 * gro + 5e-3, (gr8, gro)
    assert frac >= 0.99, frac
