"""Time clip + Adam (FusedAdam) on the EnvNet-v2 parameter set (363.4 M f32 params, grads resident)."""
import os
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "dl-sound-classification_amd"))
import torch  # noqa: E402
from src.models.envnet_v2 import EnvNetV2  # noqa: E402
from src.training.optim import FusedAdam  # noqa: E402

dev = torch.device("cuda:0")
m = EnvNetV2(num_classes=50).to(dev)
for p in m.parameters():
    p.grad = torch.randn_like(p) * 1e-3
opt = FusedAdam(m.parameters(), lr=1e-4, weight_decay=1e-4, clip=1.0)
for _ in range(3):
    opt.step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
IT = 10
e0.record()
for _ in range(IT):
    opt.step()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / IT
nel = sum(p.numel() for p in m.parameters())
print(f"clip + Adam: {ms:.3f} ms "
      f"({32 * nel / ms / 1e6:.0f} GB/s at 32 B/param)", flush=True)
