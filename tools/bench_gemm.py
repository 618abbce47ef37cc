"""Time the dense bf16 GEMM paths on the AST linear shapes (one process, interleaved rounds).
    MIA_DGEMM256=0|1 python tools/bench_gemm.py"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

T = int(os.environ.get("TOKENS", 105280))
SHAPES = [  # (name, M, N, K, la, lb)
    ("qkv.fwd", T, 2304, 768, L.KC, L.KC), ("fc1.fwd", T, 3072, 768, L.KC, L.KC),
    ("fc2.fwd", T, 768, 3072, L.KC, L.KC), ("proj.fwd", T, 768, 768, L.KC, L.KC),
    ("fc2.dgrad", T, 3072, 768, L.KC, L.RC), ("qkv.dgrad", T, 768, 2304, L.KC, L.RC),
    ("fc1.wgrad", 3072, 768, T, L.RC, L.RC), ("qkv.wgrad", 2304, 768, T, L.RC, L.RC),
]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for name, M, N, Kd, la, lb in SHAPES:
    a = (torch.randn(M, Kd, generator=g, device=dev) if la == L.KC else torch.randn(Kd, M, generator=g, device=dev)).to(torch.bfloat16)
    b = (torch.randn(N, Kd, generator=g, device=dev) if lb == L.KC else torch.randn(Kd, N, generator=g, device=dev)).to(torch.bfloat16)
    A = K.dense(a, la, *a.shape)
    Bo = K.dense(b, lb, *b.shape)
    out = torch.empty(M, N, dtype=torch.bfloat16 if Kd < 10000 else torch.float32, device=dev)
    E = K.epilogue(out, N)
    for _ in range(2):
        K.gemm(A, Bo, E, M, N, Kd, L.BF16)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        K.gemm(A, Bo, E, M, N, Kd, L.BF16)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{name:10s} M={M:6d} N={N:5d} K={Kd:6d}  {ms:7.3f} ms  {2 * M * N * Kd / ms / 1e9:7.1f} TF/s", flush=True)
