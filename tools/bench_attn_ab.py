"""A/B of the AST training path's attention backward (mia_attn_bwd_saved_q: the two-pass dQ + dK/dV kernels on
the forward's saved Q') against experiment builds of attention.hip (ATTN_LIBS=path1,...), interleaved rounds in
one process, HIP events on the launch stream, outputs compared bit for bit with the product's.
    BATCH=256 ATTN_LIBS=tools/probe/libmia_x.so python tools/bench_attn_ab.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import lib as L  # noqa: E402

B, N, H, D = int(os.environ.get("BATCH", 256)), int(os.environ.get("SEQ", 1645)), 12, 64
ITERS, ROUNDS = int(os.environ.get("ITERS", 5)), int(os.environ.get("ROUNDS", 3))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B * N, 3 * H * D, generator=g, device=dev).to(torch.bfloat16)
out = torch.empty(B * N, H * D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B, H, N, dtype=torch.float32, device=dev)
dout = torch.randn(B * N, H * D, generator=g, device=dev).to(torch.bfloat16)
lib, s = L.load(), L.stream_ptr()
libs = {"product": lib}
for path in filter(None, os.environ.get("ATTN_LIBS", "").split(",")):
    x = C.CDLL(str(REPO / path))
    for name in ("mia_attn_bwd_saved_q", "mia_attn_fwd_save_q"):
        getattr(x, name).restype, getattr(x, name).argtypes = L.SIGNATURES[name]
    libs[Path(path).stem] = x
work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=dev)
L.check(lib.mia_attn_fwd_save_q(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), None, None, work.data_ptr(), B, N, H,
                                D ** -0.5, s), "fwd")
dq = {k: torch.empty_like(qkv) for k in libs}


def run(name):
    L.check(libs[name].mia_attn_bwd_saved_q(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                            dq[name].data_ptr(), work.data_ptr(), B, N, H, D ** -0.5, s), name)


for name in libs:
    run(name)
torch.cuda.synchronize()
for name in libs:
    if name != "product":
        same = torch.equal(dq[name], dq["product"])
        d = (dq[name].float() - dq["product"].float()).abs().max() / dq["product"].float().abs().max()
        print(f"{name}: dqkv {'bit-identical to' if same else 'DIFFERS from'} the product's (max rel {float(d):.3g})",
              flush=True)
times = {n: [] for n in libs}
for _ in range(ROUNDS):
    for name in libs:
        run(name)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ITERS):
            run(name)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / ITERS)
fl = 8.0 * B * H * N * N * D
for name, ts in times.items():
    ms = min(ts)
    print(f"{name:16s} attn bwd (saved Q') B={B} {ms:.4f} ms  {fl / ms / 1e9:.1f} TF/s credited", flush=True)
