"""A/B timing of an experiment GEMM library in tools/probe (default libmgexp.so, entry points
mgexp_gemm / mgexp_workspace_bytes; MGLIB=libmg2.so MGSYM=mg2 for the 2-workgroups-per-CU variant)
against the product kernel (mia_gemm, variant "p") on the AST shapes, interleaved rounds in one process;
each variant's output is checked against mia_gemm's (bit for bit, or the max relative difference when the
K split differs).
    make -C tools/probe && TOKENS=421120 python tools/bench_mgexp.py "p,0,1" [shape ...]
mgexp flags: 1 no start stagger, 2 LDS-staged bf16 epilogue, 4 no epilogue traffic, 8 paired 16-B bf16 stores."""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

sys.path.insert(0, str(REPO / "tools"))
from bench_gemm import SHAPES  # noqa: E402

T = int(os.environ.get("TOKENS", 421120))
REPS = int(os.environ.get("REPS", 5))
ROUNDS = int(os.environ.get("ROUNDS", 3))
variants = [v if v == "p" else int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "p,0").split(",")]
want = set(sys.argv[2:])
X = C.CDLL(str(REPO / "tools" / "probe" / os.environ.get("MGLIB", "libmgexp.so")))
SYM = os.environ.get("MGSYM", "mgexp")
P = C.POINTER
XG = getattr(X, SYM + "_gemm")
XW = getattr(X, SYM + "_workspace_bytes")
XG.argtypes = [C.c_int, P(L.MiaOperand), P(L.MiaOperand), P(L.MiaEpilogue), C.c_int64, C.c_int64, C.c_int64,
               C.c_void_p, C.c_void_p]
XW.restype = C.c_int64
XW.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for name, M, N, Kd, la, lb, epi in SHAPES:
    if want and name not in want:
        continue
    a = (torch.randn(M, Kd, generator=g, device=dev) if la == L.KC else torch.randn(Kd, M, generator=g, device=dev))
    a = a.to(torch.bfloat16)
    b = (torch.randn(N, Kd, generator=g, device=dev) if lb == L.KC else torch.randn(Kd, N, generator=g, device=dev))
    b = b.to(torch.bfloat16)
    A = K.dense(a, la, *a.shape)
    Bo = K.dense(b, lb, *b.shape)
    bias = torch.randn(N, generator=g, device=dev)
    odt = torch.float32 if epi in ("f32", "residual") else torch.bfloat16
    extra = {}
    if epi == "residual":
        extra = dict(act=L.ACT_ADD_AUX, bias=bias, aux=torch.randn(M, N, generator=g, device=dev), ldaux=N)
    elif epi == "gelu_save":
        extra = dict(act=L.ACT_GELU_SAVE, bias=bias, aux=torch.empty(M, N, dtype=torch.bfloat16, device=dev), ldaux=N)
    elif epi == "dgelu":
        extra = dict(act=L.DACT_GELU, aux=torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16), ldaux=N,
                     colsum=torch.empty(N, device=dev))
    elif epi == "bias":
        extra = dict(bias=bias)
    ref = torch.empty(M, N, dtype=odt, device=dev)
    K.gemm(A, Bo, K.epilogue(ref, N, **extra), M, N, Kd, L.BF16)
    out = torch.empty(M, N, dtype=odt, device=dev)
    E = K.epilogue(out, N, **extra)
    ws = torch.empty(max(256, XW(M, N, Kd, 1 if epi == "dgelu" else 0)), dtype=torch.uint8,
                     device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def run(f):
        if f == "p":
            K.gemm(A, Bo, E, M, N, Kd, L.BF16)
            return
        rc = XG(f, A, Bo, E, M, N, Kd, ws.data_ptr(), st)
        assert rc == 0, rc

    times = {f: [] for f in variants}
    for f in variants:
        run(f)
        torch.cuda.synchronize()
        if f == "p" or not f & 4:
            if not torch.equal(out, ref):
                d = float((out.float() - ref.float()).abs().max() / ref.float().abs().max())
                print(f"  variant {f}: output differs from mia_gemm (max rel {d:.3e})")
    for _ in range(ROUNDS):
        for f in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REPS):
                run(f)
            e1.record()
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) / REPS)
    flop = 2 * M * N * Kd
    print(f"{name:11s} {epi:9s} " + "  ".join(f"[{f}] {min(times[f]):6.3f} ms {flop / min(times[f]) / 1e9:6.0f} TF"
                                           for f in variants), flush=True)
    del a, b, A, Bo, E, out, ref, ws, extra
    torch.cuda.empty_cache()
