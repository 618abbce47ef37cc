"""Time the flash-attention kernels on the AST shape (1645 tokens, 12 heads, d 64).
    BATCH=64 python tools/bench_attn.py"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import lib as L  # noqa: E402

B, N, H, D = int(os.environ.get("BATCH", 64)), 1645, 12, 64
ITERS = int(os.environ.get("ITERS", 10))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B * N, 3 * H * D, generator=g, device=dev).to(torch.bfloat16)
out = torch.empty(B * N, H * D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B, H, N, dtype=torch.float32, device=dev)
dout = torch.randn(B * N, H * D, generator=g, device=dev).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
lib = L.load()
work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=dev)
s = L.stream_ptr()


def fwd():
    L.check(lib.mia_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), L.BF16, B, N, H, D ** -0.5, s), "fwd")


def bwd():
    L.check(lib.mia_attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dqkv.data_ptr(),
                             work.data_ptr(), L.BF16, B, N, H, D ** -0.5, s), "bwd")


flop_f = 4.0 * B * H * N * N * D
for name, fn, fl in (("fwd", fwd, flop_f), ("bwd", bwd, 2.5 * flop_f)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / ITERS
    print(f"attn.{name} B={B} {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF/s ({100 * fl / ms / 1e9 / 2500:.1f}% of 2.5 PF)", flush=True)
