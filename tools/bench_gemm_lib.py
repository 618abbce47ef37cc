"""Reference point only: torch.matmul (hipBLASLt) on the AST linear shapes, to size the headroom of
the hand-written dense GEMM (tools/bench_gemm.py).  Not used by the package."""
import os

import torch

T = int(os.environ.get("TOKENS", 105280))
SHAPES = [("qkv.fwd", T, 2304, 768, 0, 0), ("fc1.fwd", T, 3072, 768, 0, 0), ("fc2.fwd", T, 768, 3072, 0, 0),
          ("proj.fwd", T, 768, 768, 0, 0), ("fc2.dgrad", T, 3072, 768, 0, 1), ("qkv.dgrad", T, 768, 2304, 0, 1),
          ("fc1.wgrad", 3072, 768, T, 1, 1), ("qkv.wgrad", 2304, 768, T, 1, 1),
          ("proj.dgrad", T, 768, 768, 0, 1), ("fc1.dgrad", T, 768, 3072, 0, 1), ("proj.wgrad", 768, 768, T, 1, 1),
          ("fc2.wgrad", 768, 3072, T, 1, 1),
          ("envfc1.fwd", 256, 4096, 84480, 0, 0), ("envfc1.dgrad", 256, 84480, 4096, 0, 1),
          ("envfc1.wgrad", 4096, 84480, 256, 1, 1)]
dev = torch.device("cuda:0")
for name, M, N, Kd, la, lb in SHAPES:
    a = torch.randn(Kd, M, device=dev).to(torch.bfloat16).t() if la else torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    b = torch.randn(Kd, N, device=dev).to(torch.bfloat16) if lb else torch.randn(N, Kd, device=dev).to(torch.bfloat16).t()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    for _ in range(2):
        torch.mm(a, b, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.mm(a, b, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"lib {name:10s} M={M:6d} N={N:5d} K={Kd:6d}  {ms:7.3f} ms  {2 * M * N * Kd / ms / 1e9:7.1f} TF/s", flush=True)
