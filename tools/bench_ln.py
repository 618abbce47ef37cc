"""Time the AST LayerNorm forward (rows = 256 x 1645 tokens, D = 768, f32 in, bf16 out; and the MX-fp8
form) optionally A/B against another build of the same C ABI (LN_LIBS=path,...: a shared library exporting
mia_layernorm_fwd / mia_layernorm_fwd_mx, e.g. tools/probe/libnorm_ref.so from a previous norm.hip),
interleaved rounds in one process, outputs compared with the product library's.
    python tools/bench_ln.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import lib as L  # noqa: E402

dev = torch.device("cuda:0")
R, D = int(os.environ.get("BATCH", 256)) * 1645, 768
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(R, D, generator=g, device=dev) * 2 + 0.3
gamma = torch.rand(D, generator=g, device=dev) + 0.5
beta = torch.randn(D, generator=g, device=dev)
y = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
q = torch.empty(R, D, dtype=torch.uint8, device=dev)
qs = torch.empty(R, D // 32, dtype=torch.uint8, device=dev)
mean = torch.empty(R, device=dev)
rstd = torch.empty(R, device=dev)
libs = {"product": L.load()}
for path in filter(None, os.environ.get("LN_LIBS", "").split(",")):
    lib = C.CDLL(str(REPO / path))
    for n in ("mia_layernorm_fwd", "mia_layernorm_fwd_mx", "mia_layernorm_bwd_colsum"):
        getattr(lib, n).argtypes = L.SIGNATURES[n][1]
    libs[Path(path).stem] = lib
s = L.stream_ptr()


def fwd(lib):
    L.check(lib.mia_layernorm_fwd(x.data_ptr(), L.F32, gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), L.BF16,
                                  mean.data_ptr(), rstd.data_ptr(), R, D, 1e-6, s), "ln")


def fwd_mx(lib):
    L.check(lib.mia_layernorm_fwd_mx(x.data_ptr(), L.F32, gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                                     q.data_ptr(), qs.data_ptr(), mean.data_ptr(), rstd.data_ptr(), R, D, 1e-6, s), "ln_mx")


dyb = (torch.randn(R, D, generator=g, device=dev) * 0.1).to(torch.bfloat16)
dx = torch.zeros(R, D, device=dev)
dx2 = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
dgam, dbet, dcs = (torch.empty(D, device=dev) for _ in range(3))
part = torch.empty(int(libs["product"].mia_layernorm_partial_bytes(R, D)), dtype=torch.uint8, device=dev)


def bwd(lib):
    L.check(lib.mia_layernorm_bwd_colsum(dyb.data_ptr(), L.BF16, x.data_ptr(), L.F32, gamma.data_ptr(), mean.data_ptr(),
                                         rstd.data_ptr(), dx.data_ptr(), L.F32, 1, dx2.data_ptr(), L.BF16,
                                         dgam.data_ptr(), dbet.data_ptr(), dcs.data_ptr(), part.data_ptr(), R, D, s),
            "ln_bwd")


ref = None
for name, lib in libs.items():
    fwd_mx(lib)
    dx.zero_()
    bwd(lib)
    torch.cuda.synchronize()
    got = (y.clone(), q.clone(), qs.clone(), mean.clone(), rstd.clone(), dx.clone(), dgam.clone(), dcs.clone())
    if ref is None:
        ref = got
    else:
        dy = (got[0].float() - ref[0].float()).abs().max().item()
        print(f"{name}: bf16 out max |diff| {dy:.3g}, fp8 bytes differing {int((got[1] != ref[1]).sum())}, "
              f"scales differing {int((got[2] != ref[2]).sum())}, mean max |diff| "
              f"{(got[3] - ref[3]).abs().max().item():.3g}; bwd dx / dgamma / colsum equal: "
              f"{[torch.equal(a, b) for a, b in zip(got[5:], ref[5:])]}", flush=True)
byts = R * D * (4 + 2)
times = {(n, k): [] for n in libs for k in ("ln", "ln_mx", "ln_bwd")}
for _ in range(3):
    for name, lib in libs.items():
        for kind, fn in (("ln", fwd), ("ln_mx", fwd_mx), ("ln_bwd", bwd)):
            fn(lib)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn(lib)
            e1.record()
            torch.cuda.synchronize()
            times[(name, kind)].append(e0.elapsed_time(e1) / 10)
for (name, kind), ts in times.items():
    ms = min(ts)
    b = byts + (R * D + R * D // 32 if kind == "ln_mx" else 0)
    if kind == "ln_bwd":
        b = R * D * (2 + 4 + 4 + 4 + 2)  # dy bf16, x, dx read + write, dx2 bf16
    print(f"{name:14s} {kind:6s} {ms:7.3f} ms {b / ms / 1e6:7.1f} GB/s", flush=True)
