"""Diagnostic: 60-step loss curves (10-step window means) + held-out accuracy of the EnvNet product
path (bf16, f32) and the oracle (autocast, f32) from several seeded inits, the test's data and schedule.
    python tools/diag/envnet_curves.py [seeds] [batch] [steps] [clip samples] [train clips] [lr]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "dl-sound-classification_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import envnet as oenv  # noqa: E402
from tests.test_gpu_train_parity import _hip_run, _onehot, _oracle_run, tone_set  # noqa: E402

seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
T = int(sys.argv[4]) if len(sys.argv) > 4 else 220_500
NTR = int(sys.argv[5]) if len(sys.argv) > 5 else 64
LR = float(sys.argv[6]) if len(sys.argv) > 6 else 1e-4
dev = torch.device("cuda:0")
from src.models.envnet_v2 import EnvNetV2  # noqa: E402

xtr, ytr = tone_set(NTR, 10, seed=1, T=T)
xte, yte = tone_set(32, 10, seed=2, T=T)
batches = [(xtr[i:i + B, None, :].to(dev), _onehot(ytr[i:i + B], 50).to(dev)) for i in range(0, NTR, B)]
xte, yte = xte[:, None, :].to(dev), yte.to(dev)


def curve(l):
    w = max(1, len(l) // 6)
    return " ".join(f"{l[i:i + w].mean():5.2f}" for i in range(0, len(l), w))


for seed in range(seeds):
    torch.manual_seed(1234 + seed)
    init = {k: v.clone() for k, v in EnvNetV2(num_classes=50, dropout=0.0).state_dict().items()
            if not k.endswith("num_batches_tracked")}
    for ac in (True, False):
        p = {k: v.to(dev) for k, v in init.items()}
        names = oenv.trainable_names(p)
        for n in names:
            p[n].requires_grad_(True)

        def ev(q):
            z = torch.cat([oenv.forward(q, xte[i:i + 8], training=False, dropout_p=0.0) for i in range(0, 32, 8)])
            return float((z.float().argmax(1) == yte).float().mean())

        l, a = _oracle_run(lambda q, x: oenv.forward(q, x, training=True, dropout_p=0.0), p, names, batches, steps, ac, ev, lr=LR)
        print(f"seed {seed} oracle {'autocast' if ac else 'f32     '}: {curve(l)}  acc {a:.3f}", flush=True)
    for cd in ("bf16", "f32"):
        m = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd)
        m.load_state_dict(init, strict=False)
        m = m.to(dev).train()

        def ev_hip(model):
            z = torch.cat([model(xte[i:i + 8]) for i in range(0, 32, 8)])
            return float((z.float().argmax(1) == yte).float().mean())

        l, a = _hip_run(m, batches, steps, ev_hip, lr=LR)
        print(f"seed {seed} hip    {cd:8s}: {curve(l)}  acc {a:.3f}", flush=True)
