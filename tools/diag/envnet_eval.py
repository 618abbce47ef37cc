"""Diagnostic: EnvNet eval-mode (BN running statistics) accuracy / logits of the bf16 product path on
the SAME trained weights as the f32 product path and the oracle.  python tools/diag/envnet_eval.py"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "dl-sound-classification_amd")]
import torch  # noqa: E402

from oracle import envnet as oenv  # noqa: E402
from tests.test_gpu_train_parity import _hip_run, _onehot, tone_set  # noqa: E402

dev = torch.device("cuda:0")
from src.models.envnet_v2 import EnvNetV2  # noqa: E402

B = 16
xtr, ytr = tone_set(128, 10, seed=1)
xte, yte = tone_set(32, 10, seed=2)
batches = [(xtr[i:i + B, None, :].to(dev), _onehot(ytr[i:i + B], 50).to(dev)) for i in range(0, 128, B)]
xte, yte = xte[:, None, :].to(dev), yte.to(dev)
torch.manual_seed(1234)
init = {k: v.clone() for k, v in EnvNetV2(num_classes=50, dropout=0.0).state_dict().items()
        if not k.endswith("num_batches_tracked")}


def logits(model, x):
    return torch.cat([model(x[i:i + 8]).float() for i in range(0, x.shape[0], 8)])


for train_cd in ("f32", "bf16"):
    m = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=train_cd)
    m.load_state_dict(init, strict=False)
    m = m.to(dev).train()
    _hip_run(m, batches, 100, lambda mm: 0.0, lr=1e-5)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    res = {}
    for cd in ("f32", "bf16"):
        e = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd)
        e.load_state_dict(sd)
        e = e.to(dev).eval()
        with torch.no_grad():
            res[cd] = logits(e, xte)
    q = {k: v.to(dev) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    with torch.no_grad():
        zo = torch.cat([oenv.forward(q, xte[i:i + 8], training=False, dropout_p=0.0) for i in range(0, 32, 8)]).float()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            za = torch.cat([oenv.forward(q, xte[i:i + 8], training=False, dropout_p=0.0) for i in range(0, 32, 8)]).float()
    for tag, z in (("hip f32", res["f32"]), ("hip bf16", res["bf16"]), ("oracle f32", zo), ("oracle autocast", za)):
        acc = float((z.argmax(1) == yte).float().mean())
        print(f"trained {train_cd}: eval {tag:16s} acc {acc:.3f}  rel vs oracle f32 {float((z - zo).norm() / zo.norm()):.4f}"
              f"  argmax agree {float((z.argmax(1) == zo.argmax(1)).float().mean()):.3f}", flush=True)
    # the train-mode forward on the test clips (batch statistics): isolates the running-statistics path
    for cd in ("f32", "bf16"):
        e = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd)
        e.load_state_dict(sd)
        e = e.to(dev).train()
        with torch.no_grad():
            z = logits(e, xte)
        q2 = {k: v.to(dev).clone() for k, v in sd.items() if not k.endswith("num_batches_tracked")}
        with torch.no_grad():
            zt = torch.cat([oenv.forward(q2, xte[i:i + 8], training=True, dropout_p=0.0) for i in range(0, 32, 8)]).float()
        print(f"trained {train_cd}: train-mode {cd:5s} rel vs oracle {float((z - zt).norm() / zt.norm()):.4f}  acc "
              f"{float((z.argmax(1) == yte).float().mean()):.3f} oracle {float((zt.argmax(1) == yte).float().mean()):.3f}")
        # running statistics written by that forward vs the oracle's
        worst = 0.0
        for k, v in e.state_dict().items():
            if k.endswith("running_var") or k.endswith("running_mean"):
                r = float((v - q2[k]).norm() / (q2[k].norm() + 1e-12))
                worst = max(worst, r)
        print(f"   running stats after 4 train-mode batches: worst rel vs oracle {worst:.4e}")
