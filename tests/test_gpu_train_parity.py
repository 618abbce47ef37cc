"""GPU: multi-step training parity of the benched bf16 path (verdict r2, "What's missing" 4).

One step cannot show drift in the optimizer state, the BN running statistics or the schedule of
updates; this runs N steps of the product path — EnvNetV2(compute_dtype="bf16") and ASTModel(bf16,
depth 2) + soft-label loss + FusedAdam (clip 1.0, Adam lr 1e-4, wd 1e-4, reference
engine.py:147-197,299-310) — and the same N steps of the oracle (torch restatement, reference op
order) under torch.autocast(bf16) (Lightning "bf16-mixed") and in f32, from identical weights, on
the same fixed batches of a learnable synthetic set: class-dependent tones (each class its own
fundamental and harmonic mix, random phase and level, noise; peak-normalised as
prepare_esc50.py:98-101).  Dropout and augmentation are off so the three runs see identical work.

Checked (tolerances below, measured values in the comments):
  * all three runs learn (the loss over the last steps is below the first steps' by a margin);
  * the HIP run's loss curve stays as close to the f32 run as the autocast run does:
    mean |loss_hip - loss_f32| <= 1.5 x mean |loss_autocast - loss_f32| + floor;
  * held-out top-1 accuracy (eval mode: BN running statistics) of the HIP run equals the f32 run's
    within one clip per 16.
"""
import numpy as np
import pytest
import torch

from oracle import ast as oast
from oracle import envnet as oenv
from oracle import logmel as olog
from oracle import train as otrain

pytestmark = pytest.mark.gpu

SR = 44_100


def tone_set(n: int, classes: int, seed: int, T: int = 220_500):
    """n clips of class-dependent harmonic tones (f0 = 110 * 2^(c / 4) Hz, class-specific harmonic
    weights), random phase / level / onset, white noise at -26 dB; peak-normalised."""
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, classes, n)
    t = np.arange(T, dtype=np.float64) / SR
    x = np.empty((n, T), np.float32)
    for i, c in enumerate(labels):
        f0 = 110.0 * 2.0 ** (c / 4.0)
        w = np.array([1.0, 0.5 * (c % 3), 0.3 * (c % 2), 0.2 * (c % 5) / 4])
        s = sum(w[h] * np.sin(2 * np.pi * f0 * (h + 1) * t + rng.uniform(0, 2 * np.pi)) for h in range(4))
        env = np.clip((t - rng.uniform(0, 1.0)) * 8.0, 0.0, 1.0)
        s = rng.uniform(0.3, 1.0) * s * env + 0.05 * rng.standard_normal(T)
        x[i] = (s / np.abs(s).max()).astype(np.float32)
    return torch.from_numpy(x), torch.from_numpy(labels)


def _onehot(lbl, C):
    return torch.nn.functional.one_hot(lbl.long(), C).float()


def _oracle_run(fwd, params, names, batches, steps, autocast, eval_fn, lr=1e-4):
    opt = torch.optim.Adam([params[n] for n in names], lr=lr, weight_decay=1e-4)
    losses = []
    for it in range(steps):
        x, y = batches[it % len(batches)]
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            z = fwd(params, x)
        loss = otrain.soft_ce(z.float(), y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_([params[n] for n in names], 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        acc = eval_fn(params)
    return np.array(losses), acc


def _hip_run(model, batches, steps, eval_fn, input_sigmoid=False, lr=1e-4):
    from src.miaudio import kernels as K
    from src.training.optim import FusedAdam
    opt = FusedAdam(model.parameters(), lr=lr, weight_decay=1e-4, clip=1.0)
    losses = []
    for it in range(steps):
        x, y = batches[it % len(batches)]
        z = model(x)
        loss, dz, _ = K.soft_ce(z.detach().float().contiguous(), y, input_sigmoid=input_sigmoid)
        z.backward(dz)
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
    model.eval()
    with torch.no_grad():
        acc = eval_fn(model)
    model.train()
    return np.array(losses), acc


def _compare(tag, hip, auto, f32, floor, acc_tol, min_drop):
    lh, ah = hip
    la, aa = auto
    lf, af = f32
    dh, da = float(np.abs(lh - lf).mean()), float(np.abs(la - lf).mean())
    k = max(3, len(lh) // 8)
    print(f"[{tag}] loss first/last: hip {lh[:k].mean():.4f}/{lh[-k:].mean():.4f}  autocast "
          f"{la[:k].mean():.4f}/{la[-k:].mean():.4f}  f32 {lf[:k].mean():.4f}/{lf[-k:].mean():.4f}")
    print(f"[{tag}] mean |loss - f32|: hip {dh:.5f}  autocast {da:.5f};  held-out acc hip {ah:.4f} "
          f"autocast {aa:.4f} f32 {af:.4f}")
    for name, l in (("hip", lh), ("autocast", la), ("f32", lf)):
        assert l[-k:].mean() < l[:k].mean() - min_drop, (name, l[:k].mean(), l[-k:].mean())
    assert dh <= 1.5 * da + floor, (dh, da)
    assert abs(ah - af) <= acc_tol, (ah, af)


def test_envnet_bf16_multistep_training_parity(cuda):
    """EnvNet: 100 steps, batch 16 of 128 clips, Adam lr 1e-5.  At the reference's lr 1e-4 this small
    set from the default init is chaotic -- Adam's first steps move every weight by ~lr*sign(g), the
    logits blow up to losses of ~10 and two f32 runs that differ only in summation order end up on
    unrelated trajectories (tools/diag/envnet_curves.py: per seed, the oracle's own autocast and f32
    runs landed 3 nats apart) -- so a curve comparison there measures noise.  At 1e-5 all runs
    converge and stay comparable; the held-out accuracy (eval mode: BN running statistics) is where
    the eval-mode fe_conv3 defect showed (bf16 0.75 vs f32 0.91)."""
    C, B, steps, n = 10, 16, 100, 128
    xtr, ytr = tone_set(n, C, seed=1)
    xte, yte = tone_set(32, C, seed=2)
    batches = [(xtr[i:i + B, None, :].to(cuda), _onehot(ytr[i:i + B], 50).to(cuda)) for i in range(0, n, B)]
    xte, yte = xte[:, None, :].to(cuda), yte.to(cuda)
    lr = 1e-5

    # the reference's own initialisation (envnet_v2.py:63-73 + replace_head), seeded
    from src.models.envnet_v2 import EnvNetV2
    torch.manual_seed(1234)
    init = {k: v.clone() for k, v in EnvNetV2(num_classes=50, dropout=0.0, compute_dtype="bf16").state_dict().items()
            if not k.endswith("num_batches_tracked")}

    def oracle(autocast):
        p = {k: v.to(cuda) for k, v in init.items()}
        names = oenv.trainable_names(p)
        for n_ in names:
            p[n_].requires_grad_(True)

        def ev(q):
            z = torch.cat([oenv.forward(q, xte[i:i + 8], training=False, dropout_p=0.0) for i in range(0, 32, 8)])
            return float((z.float().argmax(1) == yte).float().mean())

        return _oracle_run(lambda q, x: oenv.forward(q, x, training=True, dropout_p=0.0), p, names, batches, steps,
                           autocast, ev, lr=lr)

    m = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype="bf16")
    m.load_state_dict(init, strict=False)
    m = m.to(cuda).train()

    def ev_hip(model):
        z = torch.cat([model(xte[i:i + 8]) for i in range(0, 32, 8)])
        return float((z.float().argmax(1) == yte).float().mean())

    hip = _hip_run(m, batches, steps, ev_hip, lr=lr)
    _compare("envnet", hip, oracle(True), oracle(False), floor=0.02, acc_tol=2 / 32, min_drop=0.5)


def test_ast_depth2_bf16_multistep_training_parity(cuda):
    import os
    os.environ["MIA_QUIET"] = "1"
    from src.models.ast import ASTModel
    C, B, steps = 10, 4, 48
    xtr, ytr = tone_set(32, C, seed=3)
    xte, yte = tone_set(16, C, seed=4)
    spec_tr = olog.logmel(xtr.numpy()).float()  # (n, 128, 1379), the reference's ASTPreprocessor
    spec_te = olog.logmel(xte.numpy()).float().to(cuda)
    batches = [(spec_tr[i:i + B].to(cuda), _onehot(ytr[i:i + B], 50).to(cuda)) for i in range(0, 32, B)]
    yte = yte.to(cuda)
    st = oast.deit_hash_state(300, depth=2)
    hw, hb = oast.head_hash(901, 50)

    def oracle(autocast):
        p = {k: v.to(cuda).requires_grad_(True) for k, v in oast.model_params(st, hw, hb, depth=2).items()}
        names = list(p)

        def ev(q):
            z = torch.cat([oast.forward(q, spec_te[i:i + 4], depth=2) for i in range(0, 16, 4)])
            return float((z.float().argmax(1) == yte).float().mean())

        return _oracle_run(lambda q, x: oast.forward(q, x, depth=2), p, names, batches, steps, autocast, ev)

    m = ASTModel(num_classes=50, compute_dtype="bf16", depth=2)
    m.load_vit_state(st)
    with torch.no_grad():
        m.head.weight.copy_(torch.from_numpy(hw))
        m.head.bias.copy_(torch.from_numpy(hb))
    m = m.to(cuda).train()

    def ev_hip(model):
        z = torch.cat([model(spec_te[i:i + 4]) for i in range(0, 16, 4)])
        return float((z.float().argmax(1) == yte).float().mean())

    hip = _hip_run(m, batches, steps, ev_hip)
    # softmax over sigmoid outputs (ast.py:63 + engine.py:175-176) bounds this loss to [2.94, 3.92]
    _compare("ast", hip, oracle(True), oracle(False), floor=0.005, acc_tol=1 / 16, min_drop=0.02)
