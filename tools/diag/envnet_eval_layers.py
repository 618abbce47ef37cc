"""Diagnostic: per-layer eval-mode activations of the bf16 EnvNet path vs the f32 path on the same
trained weights (model._debug_capture).  python tools/diag/envnet_eval_layers.py"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "dl-sound-classification_amd")]
import torch  # noqa: E402

from tests.test_gpu_train_parity import _hip_run, _onehot, tone_set  # noqa: E402

dev = torch.device("cuda:0")
from src.models.envnet_v2 import EnvNetV2  # noqa: E402

B = 16
xtr, ytr = tone_set(64, 10, seed=1)
xte, _ = tone_set(8, 10, seed=2)
batches = [(xtr[i:i + B, None, :].to(dev), _onehot(ytr[i:i + B], 50).to(dev)) for i in range(0, 64, B)]
xte = xte[:, None, :].to(dev)
torch.manual_seed(1234)
m = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype="f32").to(dev).train()
_hip_run(m, batches, 40 if len(sys.argv) < 2 else int(sys.argv[1]), lambda mm: 0.0, lr=1e-5)
sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
for k, v in sd.items():
    if "running" in k:
        print(f"{k:28s} min {float(v.min()):10.4f} max {float(v.max()):10.4f}")
cap = {}
for cd in ("f32", "bf16"):
    e = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd)
    e.load_state_dict(sd)
    e = e.to(dev).eval()
    e._debug_capture = True
    with torch.no_grad():
        z = e(xte).float()
    cap[cd] = (e._debug, z)


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-30))


f, h = cap["f32"][0], cap["bf16"][0]
for k in ("y1", "y2", "X0", "flat", "h1", "h2"):
    if k in f and f[k] is not None and h.get(k) is not None:
        print(f"{k:6s} rel {rel(h[k].reshape(-1), f[k].reshape(-1)):.4e}  |f| {float(f[k].float().abs().max()):.3e}")
for k in ("bn1", "bn2"):
    print(f"{k} scale rel {rel(h[k].scale, f[k].scale):.3e} shift rel {rel(h[k].shift, f[k].shift):.3e}")
for i, (tf, th) in enumerate(zip(f["trunk"], h["trunk"])):
    for k in ("ya", "yb"):
        print(f"trunk{i}.{k} rel {rel(th[k].reshape(-1), tf[k].reshape(-1)):.4e} mean {float(tf[k].float().mean()):.3e} "
              f"std {float(tf[k].float().std()):.3e}")
    for k in ("bna", "bnb"):
        print(f"trunk{i}.{k} scale rel {rel(th[k].scale, tf[k].scale):.3e} shift rel {rel(th[k].shift, tf[k].shift):.3e}")
print(f"logits rel {rel(cap['bf16'][1], cap['f32'][1]):.4e}")
