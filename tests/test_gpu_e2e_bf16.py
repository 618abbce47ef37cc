"""GPU: the BENCHED bf16 train step end to end (verdict r1: the 1e-3 parity holds on the f32 kernel
set; the bf16 bench path runs different kernels).

One full step — forward -> soft-label loss -> backward -> global-norm clip 1.0 -> Adam(1e-4, wd 1e-4)
— of EnvNetV2(compute_dtype="bf16") (B = 4, the golden clips of seed 21 plus two more, golden hash
weights) and of ASTModel(compute_dtype="bf16") at depth 2, against the oracle run on the same device
under torch.autocast(bf16) (the reference's `trainer.precision: bf16-mixed`).  Both are bf16
approximations of the same f32 step, so the yardstick is fixed tolerances on logits, loss, global
grad norm and the Adam deltas (first step ~ -lr * sign(g): sign agreement where |g| is not tiny),
with each tolerance written below, plus the self-calibrating bound: the HIP step's logits and grad
logits are no further from the f32 oracle step than 1.25x the autocast step's distance to it
(measured: 0.098 HIP / 0.112 autocast for EnvNet, 0.0025 / 0.0039 for AST), the grad norm within 2x
of autocast's distance, and the argmax classes equal the f32 step's wherever its top-2 margin is
decided (larger than twice autocast's own logit perturbation)."""
import numpy as np
import pytest
import torch

from oracle import ast as oast
from oracle import envnet as oenv
from oracle import train as otrain
from oracle.synth import hash_uniform, synth_waveform
from tests._util import envnet_with_hash_params, hash_params

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _oracle_step(params, names, fwd, y, autocast: bool):
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        z = fwd(params)
    loss = otrain.soft_ce(z.float(), y)
    loss.backward()
    grads = {n: params[n].grad.detach().clone() for n in names}
    total = float(torch.nn.utils.clip_grad_norm_([params[n] for n in names], 1.0))
    before = {n: params[n].detach().clone() for n in names}
    opt = torch.optim.Adam([params[n] for n in names], lr=1e-4, weight_decay=1e-4)
    opt.step()
    return z.detach().float(), float(loss), grads, total, {n: params[n].detach() - before[n] for n in names}


def _check(tag, z, loss, total, deltas, grads, ref, ref32, tol):
    zr, lr_, gr, tr, dr = ref
    z32, l32, t32 = ref32[0], ref32[1], ref32[3]
    ez, ez32, ea32 = _rel(z, zr), _rel(z, z32), _rel(zr, z32)
    gh32, ga32 = abs(total - t32) / t32, abs(tr - t32) / t32
    print(f"[{tag}] logits rel-L2 vs autocast {ez:.4f} (vs f32 {ez32:.4f}; autocast vs f32 {ea32:.4f})"
          f" loss {loss:.5f}/{lr_:.5f} (f32 {l32:.5f}) gradnorm {total:.5f}/{tr:.5f} (f32 {t32:.5f}: hip {gh32:.5f}, "
          f"autocast {ga32:.5f})")
    assert ez < tol["logits"], ez
    if "logits_f32" in tol:  # a fixed bound against the f32 step itself, beside the self-calibrated one below
        assert ez32 < tol["logits_f32"], ez32
    # the HIP bf16 step is as close to the f32 step as autocast bf16 is (verdict r2)
    assert ez32 <= 1.25 * ea32 + 1e-3, (ez32, ea32)
    # global grad norm: both bf16 steps are within 0.6 % of the f32 one (measured EnvNet 0.53 % HIP,
    # 0.34 % autocast; AST 0.10 % / 0.08 %); the HIP path keeps more intermediates in bf16
    # (pre-BN conv outputs, BN+ReLU applied at the consumer) than autocast does
    assert gh32 <= 2.0 * ga32 + 1e-3, (gh32, ga32)
    # argmax classes equal the f32 step's wherever the f32 top-2 margin exceeds twice the largest
    # logit perturbation autocast bf16 itself causes (random-init logits have near-ties, where any
    # bf16 step may flip a class)
    a32 = z32.argmax(1)
    top2 = z32.topk(2, dim=1).values
    decided = (top2[:, 0] - top2[:, 1]) > 2.0 * float((zr - z32).abs().max())
    print(f"[{tag}] argmax: hip {z.argmax(1).tolist()} autocast {zr.argmax(1).tolist()} f32 {a32.tolist()} "
          f"decided {decided.tolist()}")
    assert torch.equal(z.argmax(1)[decided], a32[decided]), (z.argmax(1), a32, decided)
    # loss and grad norm against the f32 step: within the fixed tolerance, or no further from it than the
    # autocast step is (its distance depends on the bf16 conv algorithms MIOpen picks for the oracle)
    assert abs(loss - l32) <= max(tol["loss"] * abs(l32), 1.25 * abs(lr_ - l32) + 1e-4), (loss, lr_, l32)
    assert abs(total - t32) <= max(tol["gradnorm"] * t32, 2.0 * abs(tr - t32) + 1e-4), (total, tr, t32)
    agree, n = 0, 0
    for name, d in deltas.items():
        g = gr[name].flatten()
        m = g.abs() > 0.05 * g.abs().max()
        if not bool(m.any()):
            continue
        agree += int((torch.sign(d.flatten()[m]) == torch.sign(dr[name].flatten()[m])).sum())
        n += int(m.sum())
    frac = agree / max(n, 1)
    print(f"[{tag}] Adam delta sign agreement {frac:.4f} over {n} entries")
    assert frac >= tol["sign"], frac


def test_envnet_bf16_train_step_vs_autocast_oracle(cuda):
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    B = 4
    x = torch.from_numpy(synth_waveform(21, B, 220_500)[:, None, :]).to(cuda)
    y = torch.zeros(B, 50, device=cuda)
    y[0, 3] = 1.0
    y[1, 7], y[1, 12] = 0.8, 0.2
    y[2, 40] = 1.0
    y[3, 9], y[3, 30] = 0.35, 0.65
    m = envnet_with_hash_params(cuda, compute_dtype="bf16").train()
    names = [n for n, _ in m.named_parameters()]
    z = m(x)
    loss, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=False)
    z.backward(dz)
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    opt.step()
    assert opt.last_precomputed == 2  # FC1/FC2 weight-gradient norms came from their GEMM epilogues
    deltas = {n: p.detach() - before[n] for n, p in m.named_parameters()}

    def ref(autocast):
        p = {k: torch.from_numpy(v.copy()).to(cuda) for k, v in hash_params(100).items()}
        for n in names:
            p[n].requires_grad_(True)
        return _oracle_step(p, names, lambda q: oenv.forward(q, x, training=True, dropout_p=0.0), y, autocast)

    r16, r32 = ref(True), ref(False)
    _check("envnet", z.detach().float(), float(loss), float(opt.last_total_norm), deltas, grads, r16, r32,
           tol={"logits": 0.2, "loss": 0.03, "gradnorm": 0.03, "sign": 0.95})  # measured 0.134 / 0.010 / 0.009 / 0.973


def test_ast_depth2_bf16_train_step_vs_autocast_oracle(cuda):
    import os
    os.environ["MIA_QUIET"] = "1"
    from src.miaudio import kernels as K
    from src.models.ast import ASTModel
    from src.training.optim import FusedAdam
    B = 4
    st = oast.deit_hash_state(300, depth=2)
    hw, hb = oast.head_hash(901, 50)
    m = ASTModel(num_classes=50, compute_dtype="bf16", depth=2)
    m.load_vit_state(st)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    m = m.to(cuda).train()
    x = torch.from_numpy(hash_uniform(32, (B, 128, 1379))).to(cuda)
    y = torch.zeros(B, 50, device=cuda)
    y[0, 3], y[1, 5], y[1, 2], y[2, 49], y[3, 0], y[3, 1] = 1.0, 0.6, 0.4, 1.0, 0.3, 0.7
    probs = m(x)
    loss, dp, _ = K.soft_ce(probs.detach().float().contiguous(), y, input_sigmoid=False)
    probs.backward(dp)
    pmap = dict(m.named_parameters())
    grads = {n: p.grad.detach().clone() for n, p in pmap.items()}
    before = {n: p.detach().clone() for n, p in pmap.items()}
    opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
    opt.step()
    deltas = {n: p.detach() - before[n] for n, p in pmap.items()}
    ref_names = list(oast.model_params(st, hw, hb, depth=2))
    assert set(ref_names) == set(pmap), set(ref_names) ^ set(pmap)

    def ref(autocast):
        p = {k: v.to(cuda).requires_grad_(True) for k, v in oast.model_params(st, hw, hb, depth=2).items()}
        return _oracle_step(p, ref_names, lambda q: oast.forward(q, x, depth=2), y, autocast)

    r16, r32 = ref(True), ref(False)
    _check("ast", probs.detach().float(), float(loss), float(opt.last_total_norm), deltas, grads, r16, r32,
           tol={"logits": 0.015, "loss": 0.002, "gradnorm": 0.006, "sign": 0.99})  # measured 0.0037 / 0.0004 / 0.0015 / 1.0
