"""Time the fused log-mel at the AST shape (B clips of 5 s @ 44.1 kHz -> 128 x 1379), optionally A/B against
other builds of the C ABI (LOGMEL_LIBS=path1,...: shared libraries exporting mia_logmel_fwd, e.g. a previous
logmel.hip built into tools/probe), interleaved rounds in one process, outputs checked equal.
    BATCH=256 ITERS=10 python tools/bench_logmel.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.datasets.features import GpuLogMel  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

B, T = int(os.environ.get("BATCH", 256)), 220500
ITERS = int(os.environ.get("ITERS", 10))
ROUNDS = int(os.environ.get("ROUNDS", 3))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
wav = torch.randn(B, T, generator=g, device=dev) * 0.1
libs = {"product": L.load()}
for path in filter(None, os.environ.get("LOGMEL_LIBS", "").split(",")):
    x = C.CDLL(str(REPO / path))
    for name in ("mia_logmel_fwd", "mia_logmel_workspace_bytes"):
        getattr(x, name).restype, getattr(x, name).argtypes = L.SIGNATURES[name]
    libs[Path(path).stem] = x
mel = GpuLogMel()
ref = None
for name, lib in libs.items():
    out = mel(wav, lib=lib)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    else:
        print(f"{name}: output {'equal to' if torch.equal(out, ref) else 'DIFFERS from'} the product's", flush=True)
out = torch.empty_like(ref)
times = {n: [] for n in libs}
for _ in range(ROUNDS):
    for name, lib in libs.items():
        for _ in range(2):
            mel(wav, out, lib=lib)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ITERS):
            mel(wav, out, lib=lib)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / ITERS)
for name, ts in times.items():
    ms = min(ts)
    print(f"{name:14s} logmel B={B} {ms:.4f} ms  {B * 1588048 / ms / 1e6:.1f} GB/s algorithmic", flush=True)
