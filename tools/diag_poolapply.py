"""GPU diagnostic: octet pooled BN apply vs generic on bf16 (prints channel-wise max errors)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "dl-sound-classification_amd"))
import torch
from src.miaudio import kernels as K
dev = torch.device("cuda:0")
n, h, w, c, kh, kw = 2, 1, 640, 64, 1, 64
g = torch.Generator().manual_seed(1)
y = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16).to(dev)
st = K.BNState(torch.zeros(c, device=dev), torch.ones(c, device=dev), torch.ones(c, device=dev), torch.zeros(c, device=dev))
oh, ow = h // kh, w // kw
out = torch.empty(n, oh, ow, c, device=dev, dtype=torch.bfloat16)
am = torch.empty(n, oh, ow, c, dtype=torch.uint8, device=dev)
K.pool_fwd(y, n, h, w, c, kh, kw, st, out, 0, am)
dout = torch.randn(n, oh, ow, c, generator=g).to(dev)
gm, dg, db = K.pool_bwd_gather(dout, 0, am, y, n, h, w, c, kh, kw, st)
dx = torch.full_like(y, 7.0)
K.pool_bn_relu_bwd_apply(gm, am, y, n, h, w, c, kh, kw, None, st, torch.zeros_like(dg), torch.zeros_like(db), dx, None)
torch.cuda.synchronize()
print("dx[0,0,:4,:16]", dx[0, 0, :4, :16].float().cpu())
print("gm[0,0,0,:16]", gm.view(n, oh, ow, c)[0, 0, 0, :16].cpu())
print("am[0,0,0,:16]", am[0, 0, 0, :16].cpu())
print("y[0,0,:4,:8]", y[0, 0, :4, :8].float().cpu())
