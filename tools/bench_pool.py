"""Time the trunk pooled-BN kernels at EnvNet block 0's shape (B = 256: conv4 output 50 x 846 x 32 bf16, pool
(5, 3)): pool_fwd (max of relu(bn(x)) + argmax + raw winners) and pool_bn_relu_bwd_apply (one pass x -> dx);
digests of the outputs so builds can be compared (MIAUDIO_LIB selects the library).
    python tools/bench_pool.py"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
B, H, W, C, kh, kw = 256, 50, 846, 32, 5, 3
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(B, H, W, C, generator=g, device=dev) * 2 + 0.3).to(torch.bfloat16)
gamma = torch.randn(C, generator=g, device=dev)
beta = torch.randn(C, generator=g, device=dev) * 0.5
rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
bn = K.bn_fwd_stats(x, B * H * W, C, gamma, beta, rm, rv, 0.1, 1e-5, True)
OH, OW = H // kh, W // kw
pooled = torch.empty(B, OH, OW, C, dtype=torch.bfloat16, device=dev)
am = torch.empty(B, OH, OW, C, dtype=torch.uint8, device=dev)
win = torch.empty(B, OH, OW, C, dtype=torch.bfloat16, device=dev)
dout = torch.randn(B, OH, OW, C, generator=g, device=dev).to(torch.bfloat16)
dx = torch.empty_like(x)
dbias = torch.empty(C, device=dev)


def fwd():
    K.pool_fwd(x, B, H, W, C, kh, kw, bn, pooled, 0, am, win=win)


fwd()
gm, dg, db = K.pool_bwd_gather(dout, 0, am, x, B, H, W, C, kh, kw, bn, win=win)


def bwd():
    K.pool_bn_relu_bwd_apply(gm, am, x, B, H, W, C, kh, kw, gamma, bn, dg, db, dx, dbias)


def digest(t):
    v = t.reshape(-1).view(torch.int16).to(torch.int64)
    return int((v * torch.arange(1, v.numel() + 1, device=v.device, dtype=torch.int64).remainder(65521)).sum()) & (2**64 - 1)


nbytes = {"pool_fwd": x.numel() * 2 + pooled.numel() * 5, "pool_bn_bwd_apply": x.numel() * 4 + gm.numel() * 4}
for name, fn in (("pool_fwd", fwd), ("pool_bn_bwd_apply", bwd)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10)
    out = pooled if name == "pool_fwd" else dx
    print(f"{name:18s} {best:7.3f} ms  {nbytes[name] / best / 1e6:7.1f} GB/s  digest {digest(out):x}", flush=True)
