"""Time the fused log-mel at the AST shape (B clips of 5 s @ 44.1 kHz -> 128 x 1379).
    BATCH=256 ITERS=10 python tools/bench_logmel.py"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.datasets.features import GpuLogMel  # noqa: E402

B, T = int(os.environ.get("BATCH", 256)), 220500
ITERS = int(os.environ.get("ITERS", 10))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
wav = torch.randn(B, T, generator=g, device=dev) * 0.1
mel = GpuLogMel()
out = mel(wav)
for _ in range(3):
    mel(wav, out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(ITERS):
    mel(wav, out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / ITERS
print(f"logmel B={B} {ms:.4f} ms  {B * 1588048 / ms / 1e9:.1f} GB/s algorithmic", flush=True)
