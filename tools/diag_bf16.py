"""Per-stage forward comparison of the EnvNet-v2 bf16 and f32 HIP paths (same weights, same clips,
train-mode BN): relative L2 of every saved activation, to localise a precision loss."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from oracle.synth import synth_waveform  # noqa: E402
from src.models.envnet_v2 import EnvNetV2  # noqa: E402

dev = torch.device("cuda:0")
x = torch.from_numpy(synth_waveform(33, 4, 220_500)[:, None, :]).to(dev)
caps = {}
for cd in ("f32", "bf16"):
    torch.manual_seed(0)
    m = EnvNetV2(num_classes=50, dropout=0.0, compute_dtype=cd).to(dev).train()
    m._debug_capture = True
    z = m(x)
    s = m._debug
    d = {"y1": s["y1"], "y2": s["y2"], "X0": s["X0"], "flat": s["flat"], "h1": s["h1"], "h2": s["h2"], "z": z}
    for i, ts in enumerate(s["trunk"]):
        d[f"t{i}.ya"] = ts["ya"]
        d[f"t{i}.yb"] = ts["yb"]
    for k in ("bn1", "bn2"):
        d[k + ".mean"] = s[k].mean
        d[k + ".invstd"] = s[k].invstd
    caps[cd] = {k: v.detach().double().cpu() for k, v in d.items()}


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


for k in caps["f32"]:
    a, b = caps["bf16"][k], caps["f32"][k]
    print(f"{k:12s} shape={tuple(b.shape)} relL2={rel(a.reshape(b.shape), b):.4e} |f32|={float(b.abs().max()):.3e}")

# PyTorch (MIOpen/hipBLAS) restatement of the reference forward on the same weights: f32 and
# bf16 autocast, to see how much of the bf16/f32 gap is inherent to bf16 activations.
from oracle import envnet as oenv  # noqa: E402

torch.manual_seed(0)
m = EnvNetV2(num_classes=50, dropout=0.0).to(dev).train()
ref = {}
for mode in ("f32", "bf16"):
    params = {k: v.detach().clone() for k, v in m.state_dict().items()}
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "bf16"):
        ref[mode] = oenv.forward(params, x.float(), training=True, dropout_p=0.0).double().cpu()
print("torch  bf16-autocast vs torch f32: z relL2", rel(ref["bf16"], ref["f32"]))
print("ours   f32 vs torch f32          : z relL2", rel(caps["f32"]["z"], ref["f32"]))
print("ours   bf16 vs torch f32         : z relL2", rel(caps["bf16"]["z"], ref["f32"]))
print("ours   bf16 vs torch bf16        : z relL2", rel(caps["bf16"]["z"], ref["bf16"]))
