"""Time the flash-attention kernels on the AST shape (1645 tokens, 12 heads, d 64), optionally A/B against
an experiment build of the same C ABI (ATTN_LIBS=path1,path2: each a shared library exporting mia_attn_fwd /
mia_attn_bwd, e.g. tools/probe/libattn_ref.so built from a previous attention.hip), interleaved rounds in
one process, outputs checked equal to the product library's.  Build a reference with attention.hip's
own flags from the package Makefile (-mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize): without them the
same source runs ~5 % slower and the A/B measures the flags.
    BATCH=256 python tools/bench_attn.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import lib as L  # noqa: E402

B, N, H, D = int(os.environ.get("BATCH", 64)), 1645, 12, 64
ITERS = int(os.environ.get("ITERS", 10))
ROUNDS = int(os.environ.get("ROUNDS", 3))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B * N, 3 * H * D, generator=g, device=dev).to(torch.bfloat16)
out = torch.empty(B * N, H * D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B, H, N, dtype=torch.float32, device=dev)
dout = torch.randn(B * N, H * D, generator=g, device=dev).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
libs = {"product": L.load()}
for path in filter(None, os.environ.get("ATTN_LIBS", "").split(",")):
    x = C.CDLL(str(REPO / path))
    x.mia_attn_fwd.argtypes = L.SIGNATURES["mia_attn_fwd"][1]
    x.mia_attn_bwd.argtypes = L.SIGNATURES["mia_attn_bwd"][1]
    libs[Path(path).stem] = x
work = torch.empty(int(libs["product"].mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=dev)
s = L.stream_ptr()


def fwd(lib):
    L.check(lib.mia_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), L.BF16, B, N, H, D ** -0.5, s), "fwd")


def bwd(lib):
    L.check(lib.mia_attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dqkv.data_ptr(),
                             work.data_ptr(), L.BF16, B, N, H, D ** -0.5, s), "bwd")


ref = {}
for name, lib in libs.items():
    fwd(lib)
    bwd(lib)
    torch.cuda.synchronize()
    got = (out.clone(), lse.clone(), dqkv.clone())
    if not ref:
        ref = got
    else:
        same = all(torch.equal(a, b) for a, b in zip(got, ref))
        print(f"{name}: outputs {'equal to' if same else 'DIFFER from'} the product library's", flush=True)

flop_f = 4.0 * B * H * N * N * D
times = {(n, k): [] for n in libs for k in ("fwd", "bwd")}
for _ in range(ROUNDS):
    for name, lib in libs.items():
        for kind, fn in (("fwd", fwd), ("bwd", bwd)):
            for _ in range(2):
                fn(lib)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(ITERS):
                fn(lib)
            e1.record()
            torch.cuda.synchronize()
            times[(name, kind)].append(e0.elapsed_time(e1) / ITERS)
for (name, kind), ts in times.items():
    ms = min(ts)
    fl = flop_f if kind == "fwd" else 2.0 * flop_f  # backward = 2x forward, recompute not credited
    print(f"{name:12s} attn.{kind} B={B} {ms:7.3f} ms {fl / ms / 1e9:7.1f} TF/s ({100 * fl / ms / 1e9 / 2500:.1f}% "
          f"of 2.5 PF)", flush=True)
