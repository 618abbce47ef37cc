"""Time the bf16 attention backward on the AST shape (N 1645, H 12, d 64): the fused one-pass form
(mia_attn_bwd_fused) against the two-kernel form (mia_attn_bwd_two_pass), interleaved rounds in one
process, HIP events on the launch stream; the fused form's error word checked, results compared.
    BATCH=256 python tools/bench_attn_bwd.py"""
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
work = torch.empty(int(lib.mia_attn_bwd_workspace_bytes(L.BF16, B, N, H)), dtype=torch.uint8, device=dev)
L.check(lib.mia_attn_fwd_save_q(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), None, None, work.data_ptr(), B, N, H,
                                D ** -0.5, s), "fwd")
ALT = {}  # experiment builds of attention.hip (ATTN_LIBS=path,...): timed as "one:<stem>"
for path in filter(None, os.environ.get("ATTN_LIBS", "").split(",")):
    import ctypes as C
    x = C.CDLL(str(REPO / path))
    x.mia_attn_bwd_onepass.argtypes = L.SIGNATURES["mia_attn_bwd_onepass"][1]
    ALT["one:" + Path(path).stem] = x
dq = {k: torch.empty_like(qkv) for k in ("fused", "two", "one", *ALT)}
chain = torch.empty(int(lib.mia_attn_bwd_chain_bytes(B, N, H)), dtype=torch.uint8, device=dev)
errs = {}  # one sticky error word per one-pass variant


def run(name):
    if name.startswith("one"):
        err = errs.setdefault(name, torch.zeros(1, dtype=torch.int32, device=dev))
        L.check(ALT.get(name, lib).mia_attn_bwd_onepass(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                         dq[name].data_ptr(), work.data_ptr(), chain.data_ptr(), err.data_ptr(), B, N,
                                         H, D ** -0.5, 1, s), name)
    elif name == "fused":
        L.check(lib.mia_attn_bwd_fused(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                       dq[name].data_ptr(), work.data_ptr(), B, N, H, D ** -0.5, 1, s), name)
    else:
        L.check(lib.mia_attn_bwd_two_pass(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                          dq[name].data_ptr(), work.data_ptr(), B, N, H, D ** -0.5, 1, s), name)


for name in dq:
    run(name)
torch.cuda.synchronize()
off = int(lib.mia_attn_bwd_error_offset(B, N, H))
run("fused")
torch.cuda.synchronize()
print("fused error word", int(work[off:off + 4].view(torch.int32).item()), flush=True)
d = (dq["fused"].float() - dq["two"].float()).abs().max() / dq["two"].float().abs().max()
print(f"fused vs two-pass: max |d| / max {float(d):.3g}", flush=True)
for name in ["one", *ALT]:
    d = (dq[name].float() - dq["two"].float()).abs().max() / dq["two"].float().abs().max()
    print(f"{name} vs two-pass: max |d| / max {float(d):.3g}, error word {int(errs[name].item())}", flush=True)
flop = 8.0 * B * H * N * N * D  # 2x the forward, recompute not credited
for r in range(ROUNDS):
    for name in os.environ.get("VARIANTS", "two,fused,one").split(",") + list(ALT):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(ITERS):
            run(name)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / ITERS
        print(f"round {r} {name:5s} {ms:7.3f} ms  {flop / ms / 1e9:7.1f} TF/s credited  "
              f"{flop / ms / 1e9 / 2500:.3f} of peak", flush=True)
