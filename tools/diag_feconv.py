"""Which reference channel does each fe_conv2_fwd output channel match?  (GPU diagnostic)"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "dl-sound-classification_amd"))
import torch
import torch.nn.functional as F
from src.miaudio import kernels as K
from src.miaudio import lib as L

dev = torch.device("cuda:0")
n, w1 = 1, 4112
w2 = (w1 - 16) // 2 + 1
g = torch.Generator().manual_seed(1)
y1 = torch.randn(n, w1, 32, generator=g).to(torch.bfloat16)
W = torch.randn(64, 32, 1, 16, generator=g) * 0.05
bias = torch.zeros(64)
wp = K.pack_weight(W.to(dev), L.BF16, 0)
out = torch.zeros((n * w2, 64), dtype=torch.bfloat16, device=dev)
K.fe_conv2_fwd(y1.to(dev).reshape(-1, 32), None, None, wp, bias.to(dev), out, n, w1, w2)
torch.cuda.synchronize()
ref = F.conv1d(y1.double().permute(0, 2, 1), W.to(torch.bfloat16).double()[:, :, 0], stride=2)[0]  # (64, w2)
got = out.double().cpu().view(w2, 64).t()
for c in range(64):
    errs = [(got[c, :64] - ref[r, :64]).abs().max().item() for r in range(64)]
    best = min(range(64), key=lambda r: errs[r])
    # maybe pixel-shifted
    print(c, best, round(errs[best], 4), round(errs[c], 4))
