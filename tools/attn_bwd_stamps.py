"""Per-segment cycle stamps of the one-pass attention backward (a -DCB_STAMP build of attn_bwd.hip, see
tools/probe): wave-level s_memtime at the segment boundaries of every step of the first 256 work items.
    STAMP_LIB=tools/probe/libattn_stamp.so BATCH=256 python tools/attn_bwd_stamps.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.miaudio import lib as L  # noqa: E402

B, N, H, D = int(os.environ.get("BATCH", 256)), int(os.environ.get("SEQ", 1645)), 12, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B * N, 3 * H * D, generator=g, device=dev).to(torch.bfloat16)
out = torch.empty(B * N, H * D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B, H, N, dtype=torch.float32, device=dev)
dout = torch.randn(B * N, H * D, generator=g, device=dev).to(torch.bfloat16)
lib, s = L.load(), L.stream_ptr()
work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=dev)
L.check(lib.mia_attn_fwd_save_q(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), None, None, work.data_ptr(), B, N, H,
                                D ** -0.5, s), "fwd")
x = C.CDLL(str(REPO / os.environ.get("STAMP_LIB", "tools/probe/libattn_stamp.so")))
x.mia_attn_bwd_onepass.argtypes = L.SIGNATURES["mia_attn_bwd_onepass"][1]
x.mia_attn_bwd_chain_bytes.restype = C.c_int64
x.mia_attn_bwd_chain_bytes.argtypes = [C.c_int32] * 3
plain = int(lib.mia_attn_bwd_chain_bytes(B, N, H))
chain = torch.zeros(int(x.mia_attn_bwd_chain_bytes(B, N, H)), dtype=torch.uint8, device=dev)
assert chain.numel() > plain + 256 * 4 * 64 * 16 * 8 - 1, "not a CB_STAMP build"
err = torch.zeros(1, dtype=torch.int32, device=dev)
dq = torch.empty_like(qkv)
ms = []
for _ in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    L.check(x.mia_attn_bwd_onepass(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), dq.data_ptr(),
                                   work.data_ptr(), chain.data_ptr(), err.data_ptr(), B, N, H, D ** -0.5, 1, s), "one")
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
print(f"stamp build: {min(ms):.3f} ms per call, error word {int(err.item())}")
nt = (N + 63) // 64
flags_bytes = plain - B * H * nt * 16384
st = chain[plain:plain + 256 * 4 * 64 * 16 * 8].view(torch.int64).cpu().numpy().reshape(256, 4, 64, 16)[:, :, :nt, :]
st = st.astype(np.float64)
order = [0, 1, 7, 8, 9, 2, 3, 4, 5, 6]  # 7 after the mid-step vmcnt(0), 8 after the flag publish, 9 after the spin
names = ["issue+half0", "vmcnt(0)", "publish", "flag/spin", "run loads", "half1", "link_store", "lgkm wait", "barrier"]
seg = np.diff(st[..., order], axis=3)
mid = seg[:, :, 2:nt - 1, :]
print(f"steps 2..{nt - 2}, 256 work items x 4 waves: median / mean cycles per segment")
for k, n in enumerate(names):
    v = mid[..., k].ravel()
    print(f"  {n:12s} median {np.median(v):8.0f}  mean {v.mean():8.0f}  p90 {np.percentile(v, 90):8.0f}")
step = st[:, :, 3:nt, 0] - st[:, :, 2:nt - 1, 0]
print(f"  step total   median {np.median(step):8.0f}  mean {step.mean():8.0f}")
spun = st[:, :, 2:nt - 1, 10] != 0
print(f"steps whose start-of-step flag was not ready (spun): {spun.mean():.3f}")
for wv in range(4):
    print(f"  wave {wv}: " + " ".join(f"{np.median(mid[:, wv, :, k]):6.0f}" for k in range(len(names))))
print(f"kernel span of item 0 wave 0: {st[0, 0, nt - 1, 6] - st[0, 0, 0, 0]:.0f} cycles")
