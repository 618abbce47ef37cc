"""Diagnostic: EnvNet product path vs the oracle over a few Adam steps from the seeded default init
(per-step loss, per-parameter gradient / update agreement).  python tools/diag/envnet_train.py [f32|bf16]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "dl-sound-classification_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import envnet as oenv  # noqa: E402
from oracle import train as otrain  # noqa: E402
from tests.test_gpu_train_parity import _onehot, tone_set  # noqa: E402

cd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
dev = torch.device("cuda:0")
from src.miaudio import kernels as K  # noqa: E402
from src.models.envnet_v2 import EnvNetV2  # noqa: E402
from src.training.optim import FusedAdam  # noqa: E402

torch.manual_seed(1234)
init = {k: v.clone() for k, v in EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd).state_dict().items()
        if not k.endswith("num_batches_tracked")}
xtr, ytr = tone_set(16, 10, seed=1)
B = 8
batches = [(xtr[i:i + B, None, :].to(dev), _onehot(ytr[i:i + B], 50).to(dev)) for i in range(0, 16, B)]

p = {k: v.to(dev) for k, v in init.items()}
names = oenv.trainable_names(p)
for n in names:
    p[n].requires_grad_(True)
opt_o = torch.optim.Adam([p[n] for n in names], lr=1e-4, weight_decay=1e-4)
m = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd)
m.load_state_dict(init, strict=False)
m = m.to(dev).train()
mp = dict(m.named_parameters())
opt_h = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
missing = [n for n in names if n not in mp]
print("oracle names not in model:", missing[:5], "model params not in oracle:", [n for n in mp if n not in names][:5])
for it in range(8):
    x, y = batches[it % 2]
    z = oenv.forward(p, x, training=True, dropout_p=0.0)
    lo = otrain.soft_ce(z.float(), y)
    lo.backward()
    no = float(torch.nn.utils.clip_grad_norm_([p[n] for n in names], 1.0))
    zh = m(x)
    lh, dz, _ = K.soft_ce(zh.detach().float().contiguous(), y, False)
    zh.backward(dz)
    nh = float(torch.sqrt(sum((q.grad.double() ** 2).sum() for q in m.parameters() if q.grad is not None)))
    print(f"step {it}: loss oracle {float(lo):.4f} hip {float(lh):.4f}  logits rel {float((zh.float()-z).norm()/z.norm()):.4f}"
          f"  gradnorm oracle {no:.3f} hip {nh:.3f}")
    if it == 0:
        for n in names:
            go = p[n].grad.double()
            gh = mp[n].grad.double() if mp[n].grad is not None else None
            if gh is None:
                print(f"   {n}: no hip grad")
                continue
            # oracle grads are post-clip: compare directions
            cos = float((go * gh).sum() / (go.norm() * gh.norm() + 1e-30))
            print(f"   {n:28s} |g| oracle(clipped) {float(go.norm()):.3e} hip {float(gh.norm()):.3e} cos {cos:.5f}")
    opt_o.step()
    opt_o.zero_grad(set_to_none=True)
    before = {n: mp[n].detach().clone() for n in names}
    opt_h.step()
    opt_h.zero_grad(set_to_none=True)
    if it < 2:
        worst = max(names, key=lambda n: float((mp[n].detach() - p[n].detach()).norm() / (p[n].detach().norm() + 1e-30)))
        du = {n: float((mp[n].detach() - before[n]).norm()) for n in names}
        print(f"   hip update norm total {np.sqrt(sum(v*v for v in du.values())):.4e}; worst param drift {worst} "
              f"{float((mp[worst].detach() - p[worst].detach()).norm() / p[worst].detach().norm()):.3e}  "
              f"clip coef hip norm {opt_h.last_total_norm}")
