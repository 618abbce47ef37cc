"""Time the EnvNet trunk conv4 row-rolling kernel (mia_trunk_conv8) at the bench shape (B=256: forward
57 x 853 -> 50 x 846 with BN+ReLU staging and BN statistics; backward-data 50 x 846 -> 57 x 853),
optionally A/B against another build of the same C ABI (CONV8_LIBS=path,...: a shared library exporting
mia_trunk_conv8, e.g. tools/probe/libconv8_ref.so built from a previous conv8.hip), interleaved rounds in
one process, outputs checked equal to the product library's.
    python tools/bench_conv8.py"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

dev = torch.device("cuda:0")
B, H, W = int(os.environ.get("BATCH", 256)), 57, 853
OH, OW = H - 7, W - 7
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(B * H * W, 32, generator=g, device=dev) * 0.7).to(torch.bfloat16)
dy = torch.randn(B * OH * OW, 32, generator=g, device=dev).to(torch.bfloat16)
Wt = torch.randn(32, 32, 8, 8, generator=g, device=dev) * 0.03
wp, wf = K.pack_weight(Wt, L.BF16, 0), K.pack_weight(Wt, L.BF16, 1)
sc = torch.rand(32, generator=g, device=dev) + 0.5
sh = torch.randn(32, generator=g, device=dev) * 0.3
bias = torch.randn(32, generator=g, device=dev)
y = torch.empty(B * OH * OW, 32, dtype=torch.bfloat16, device=dev)
dx = torch.empty(B * H * W, 32, dtype=torch.bfloat16, device=dev)
part = torch.empty(1024, 32, 2, device=dev)
libs = {"product": L.load()}
for path in filter(None, os.environ.get("CONV8_LIBS", "").split(",")):
    lib = C.CDLL(str(REPO / path))
    lib.mia_trunk_conv8.argtypes = L.SIGNATURES["mia_trunk_conv8"][1]
    lib.mia_trunk_conv8_dgrad_bn.argtypes = L.SIGNATURES["mia_trunk_conv8_dgrad_bn"][1]
    libs[Path(path).stem] = lib
s = L.stream_ptr()


def fwd(lib):
    L.check(lib.mia_trunk_conv8(x.data_ptr(), sc.data_ptr(), sh.data_ptr(), wp.data_ptr(), bias.data_ptr(),
                                y.data_ptr(), part.data_ptr(), 256, B, H, W, 0, 0, s), "fwd")


bxr = (torch.randn(B * H * W, 32, generator=g, device=dev) * 0.7).to(torch.bfloat16)
bn = K.BNState(torch.zeros(32, device=dev), torch.ones(32, device=dev), sc, sh)
gbeta = torch.empty(2, 32, device=dev)


def dgrad_bn(lib):
    L.check(lib.mia_trunk_conv8_dgrad_bn(dy.data_ptr(), wf.data_ptr(), dx.data_ptr(), 256, B, OH, OW, bxr.data_ptr(),
                                         sc.data_ptr(), sh.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                                         gbeta[0].data_ptr(), gbeta[1].data_ptr(), part.data_ptr(), s), "dgrad_bn")


def dgrad(lib):
    L.check(lib.mia_trunk_conv8(dy.data_ptr(), None, None, wf.data_ptr(), None, dx.data_ptr(), None, 256, B, OH, OW,
                                7, 7, s), "dgrad")


ref = None
for name, lib in libs.items():
    fwd(lib)
    dgrad(lib)
    torch.cuda.synchronize()
    got = (y.clone(), dx.clone(), part.clone())
    dgrad_bn(lib)
    torch.cuda.synchronize()
    got += (dx.clone(), gbeta.clone())
    if ref is None:
        ref = got
    else:
        print(f"{name}: outputs {'equal to' if all(torch.equal(a, b) for a, b in zip(got, ref)) else 'DIFFER from'} "
              f"the product library's", flush=True)
flop = 2.0 * B * OH * OW * 32 * 2048
KINDS = [("fwd", fwd), ("dgrad", dgrad), ("dgbn", dgrad_bn)]
times = {(n, k): [] for n in libs for k, _ in KINDS}
for _ in range(int(os.environ.get("ROUNDS", 3))):
    for name, lib in libs.items():
        for kind, fn in KINDS:
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
    if not ts:
        continue
    ms = min(ts)
    print(f"{name:16s} conv8.{kind:5s} {ms:7.3f} ms {flop / ms / 1e9:7.1f} TF/s", flush=True)
