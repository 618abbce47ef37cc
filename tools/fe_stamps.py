"""Per-item segment stamps of the frontend conv2 kernels (a -DFE_STAMP build of feconv.hip, linked as
tools/probe/libmia_festamp.so): wave-level s_memtime at the segment boundaries of every item of the first
64 workgroups, for the conv2 forward and backward-data launches at the bench shape.
    MIAUDIO_LIB=$PWD/tools/probe/libmia_festamp.so python tools/fe_stamps.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import numpy as np  # noqa: E402
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
lib = C.CDLL(os.environ["MIAUDIO_LIB"])
lib.mia_fe_stamps_copy.argtypes = [C.c_void_p, C.c_int64]
names = ["load issue", "compute", "epilogue", "store(cook)", "lgkm wait", "barrier"]
for name, fn in (("conv2.fwd", lambda: K.fe_conv2_fwd(y1, sc, sh, w0, bias, y2, B, W1, W2)),
                 ("conv2.dgrad", lambda: K.fe_conv2_dgrad(dy2, wpar, da1, B, W1, W2))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(64 * 4 * 256 * 8, dtype=np.uint64)
    assert lib.mia_fe_stamps_copy(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(64, 4, 256, 8).astype(np.float64)
    ok = st[:, :, :, 6] > 0
    seg = np.diff(st[..., :7], axis=3)
    n = int(ok[0, 0].sum())
    mid = seg[:, :, 2:n - 2, :]
    print(f"{name}: {e0.elapsed_time(e1):.3f} ms (stamp build); items per workgroup {n}")
    for k, nm in enumerate(names):
        v = mid[..., k].ravel()
        print(f"  {nm:12s} median {np.median(v):7.0f}  mean {v.mean():7.0f}  p90 {np.percentile(v, 90):7.0f}")
    item = st[:, :, 3:n - 2, 0] - st[:, :, 2:n - 3, 0]
    print(f"  item total   median {np.median(item):7.0f}  mean {item.mean():7.0f}")
