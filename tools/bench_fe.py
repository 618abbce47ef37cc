"""Time the EnvNet frontend conv kernels at the bench shape (B=256, 5 s clips) in isolation.
    python tools/bench_fe.py"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

dev = torch.device("cuda:0")
B, W1 = 256, 110219
W2 = (W1 - 16) // 2 + 1
g = torch.Generator(device=dev).manual_seed(0)
y1 = torch.randn(B * W1, 32, generator=g, device=dev).to(torch.bfloat16)
dy2 = torch.randn(B * W2, 64, generator=g, device=dev).to(torch.bfloat16)
W = torch.randn(64, 32, 1, 16, generator=g, device=dev) * 0.05
w0 = K.pack_weight(W, L.BF16, 0)
wpar = K.pack_weight(W, L.BF16, 2)
sc = torch.rand(32, generator=g, device=dev) + 0.5
sh = torch.randn(32, generator=g, device=dev)
bias = torch.randn(64, generator=g, device=dev)
y2 = torch.empty(B * W2, 64, dtype=torch.bfloat16, device=dev)
da1 = torch.empty(B * W1, 32, dtype=torch.bfloat16, device=dev)
dw = torch.empty(64, 512, device=dev)
T = 220500
x = torch.randn(B, T, generator=g, device=dev) * 0.1
w1 = (torch.randn(32, 64, generator=g, device=dev) * 0.1).to(torch.bfloat16)
b1 = torch.randn(32, generator=g, device=dev) * 0.1
y1c = torch.empty(B * W1, 32, dtype=torch.bfloat16, device=dev)
H3, W3 = 64, 860  # trunk conv3 input (B, 64, 860) -> (B, 57, 853, 32)
x3 = (torch.randn(B, H3, W3, generator=g, device=dev) * 0.5).to(torch.bfloat16)
w3 = (torch.randn(32, 64, generator=g, device=dev) * 0.1).to(torch.bfloat16)
b3 = torch.randn(32, generator=g, device=dev) * 0.1
y3 = torch.empty(B * (H3 - 7) * (W3 - 7), 32, dtype=torch.bfloat16, device=dev)
runs = {
    "fe_conv3_fwd": lambda: K.fe_conv3_fwd(x3, w3, b3, y3, B, H3, W3, stats=True),
    "fe_conv1_fwd": lambda: K.fe_conv1_fwd(x, w1, b1, y1c, B, T, stats=True),
    "fe_conv2_fwd": lambda: K.fe_conv2_fwd(y1, sc, sh, w0, bias, y2, B, W1, W2),
    "fe_conv2_dgrad": lambda: K.fe_conv2_dgrad(dy2, wpar, da1, B, W1, W2),
    "fe_conv2_wgrad": lambda: K.fe_conv2_wgrad(dy2, y1, sc, sh, dw, B, W1, W2),
    "dgrad+wgrad": lambda: (K.fe_conv2_dgrad(dy2, wpar, da1, B, W1, W2), K.fe_conv2_wgrad(dy2, y1, sc, sh, dw, B, W1, W2)),
}
byts = {"fe_conv3_fwd": x3.numel() * 2 + y3.numel() * 2, "fe_conv1_fwd": x.numel() * 4 + y1c.numel() * 2, "fe_conv2_fwd": (y1.numel() + y2.numel()) * 2, "fe_conv2_dgrad": (dy2.numel() + da1.numel()) * 2,
        "fe_conv2_wgrad": (dy2.numel() + y1.numel()) * 2, "dgrad+wgrad": (2 * dy2.numel() + y1.numel() + da1.numel()) * 2}
flop = 2.0 * B * W2 * 64 * 512
want = set(sys.argv[1:])


def with_ws(fn, on):  # MIA_FECONV_WS A/B (read by the library per call)
    def run():
        os.environ["MIA_FECONV_WS"] = "1" if on else "0"
        fn()
    return run


if os.environ.get("FE_AB"):  # warp-specialised conv2 fwd against the two-workgroup form, alternating
    f = runs.pop("fe_conv2_fwd")
    runs["fe_conv2_fwd"] = with_ws(f, False)
    runs["fe_conv2_fwd_ws"] = with_ws(f, True)
    byts["fe_conv2_fwd_ws"] = byts["fe_conv2_fwd"]
    seq = [(k, runs[k]) for k in ["fe_conv2_fwd", "fe_conv2_fwd_ws"] * 3]
else:
    seq = list(runs.items())


def digest(t):
    v = t.reshape(-1).view(torch.int32).to(torch.int64)
    return int((v * torch.arange(1, v.numel() + 1, device=v.device, dtype=torch.int64).remainder(65521)).sum()) & (2**64 - 1)


for name, fn in seq:
    if want and name not in want:
        continue
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    out = {"fe_conv3_fwd": y3, "fe_conv1_fwd": y1c, "fe_conv2_fwd": y2, "fe_conv2_dgrad": da1,
           "fe_conv2_wgrad": dw}.get(name.removesuffix("_ws"))
    dg = f"digest {digest(out):x}" if out is not None else ""
    print(f"{name:16s} {ms:7.3f} ms  {byts[name] / ms / 1e6:7.1f} GB/s  {flop / ms / 1e9:7.1f} TF/s  {dg}", flush=True)
