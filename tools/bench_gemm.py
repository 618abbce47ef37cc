"""Time mia_gemm on the AST linear shapes with the epilogues the AST step uses (one process).
    TOKENS=421120 python tools/bench_gemm.py [name[@mx][:epilogue[+mxq]] ...]
(an explicit epilogue overrides the shape's own: plain, bias, gelu, gelu_save, gelu_save_d, dgelu, dmul, dmul_nocs,
residual, f32 -- the epilogue ablations of one shape; "+mxq" adds the epilogue's MX-fp8 copy of the bf16 output;
"@mx" runs the shape on MX-fp8 operands (mia_gemm_mxfp8_ex), as fp8-mixed does)
Prints ms and TFLOP/s per shape (random bf16 operands; HIP events on the launch stream)."""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

T = int(os.environ.get("TOKENS", 421120))  # the bench step: 256 clips x 1645 tokens
REPS = int(os.environ.get("REPS", 10))
ROT = int(os.environ.get("ROT", 1))  # >1: rotate through ROT fresh copies of A and the outputs (cold TLB / caches)
# >0: a streaming copy of that many MiB between the timed launches (each launch timed alone), as a training
# step runs memory-bound kernels between its GEMMs
GAP_MB = int(os.environ.get("GAP_MB", 0))
# (name, M, N, K, la, lb, epilogue kind)
SHAPES = [
    ("qkv.fwd", T, 2304, 768, L.KC, L.KC, "bias"), ("proj.fwd", T, 768, 768, L.KC, L.KC, "residual"),
    ("fc1.fwd", T, 3072, 768, L.KC, L.KC, "gelu_save"), ("fc2.fwd", T, 768, 3072, L.KC, L.KC, "residual"),
    ("fc2.dgrad", T, 3072, 768, L.KC, L.RC, "dgelu"), ("fc1.dgrad", T, 768, 3072, L.KC, L.RC, "plain"),
    ("proj.dgrad", T, 768, 768, L.KC, L.RC, "plain"), ("qkv.dgrad", T, 768, 2304, L.KC, L.RC, "plain"),
    ("fc2.wgrad", 768, 3072, T, L.RC, L.RC, "f32"), ("fc1.wgrad", 3072, 768, T, L.RC, L.RC, "f32"),
    ("proj.wgrad", 768, 768, T, L.RC, L.RC, "f32"), ("qkv.wgrad", 2304, 768, T, L.RC, L.RC, "f32"),
]

def main():
    want = sys.argv[1:] or [s[0] for s in SHAPES]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    total = 0.0
    table = {s[0]: s for s in SHAPES}
    for w in want:
        name, _, over = w.partition(":")
        name, _, prec = name.partition("@")
        _, M, N, Kd, la, lb, epi = table[name]
        epi = over or epi
        epi, _, mxq = epi.partition("+")
        a = (torch.randn(M, Kd, generator=g, device=dev) if la == L.KC else torch.randn(Kd, M, generator=g, device=dev))
        a = a.to(torch.bfloat16)
        b = (torch.randn(N, Kd, generator=g, device=dev) if lb == L.KC else torch.randn(Kd, N, generator=g, device=dev))
        b = b.to(torch.bfloat16)
        A = K.dense(a, la, *a.shape)
        Bo = K.dense(b, lb, *b.shape)
        bias = torch.randn(N, generator=g, device=dev)
        if epi == "f32":
            out = torch.empty(M, N, dtype=torch.float32, device=dev)
            E = K.epilogue(out, N)
        elif epi == "residual":
            out = torch.empty(M, N, dtype=torch.float32, device=dev)
            res = torch.randn(M, N, generator=g, device=dev)
            E = K.epilogue(out, N, act=L.ACT_ADD_AUX, bias=bias, aux=res, ldaux=N)
        elif epi == "gelu_save":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            u = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            E = K.epilogue(out, N, act=L.ACT_GELU_SAVE, bias=bias, aux=u, ldaux=N)
        elif epi == "gelu_save_d":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            u = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            E = K.epilogue(out, N, act=L.ACT_GELU_SAVE_D, bias=bias, aux=u, ldaux=N)
        elif epi == "gelu":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            E = K.epilogue(out, N, act=L.ACT_GELU, bias=bias)
        elif epi in ("dgelu", "dmul", "dmul_nocs"):
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            u = torch.randn(M, N, generator=g, device=dev).to(torch.bfloat16)
            cs = torch.empty(N, device=dev) if epi != "dmul_nocs" else None
            E = K.epilogue(out, N, act=L.DACT_GELU if epi == "dgelu" else L.DACT_MUL, aux=u, ldaux=N, colsum=cs)
        else:
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            E = K.epilogue(out, N, bias=bias if epi == "bias" else None)
        if ROT > 1:  # the same shape / epilogue on ROT separate A / output / aux buffers, used round robin
            sets = []
            for _ in range(ROT):
                a2 = a.clone()
                o2 = torch.empty_like(out)
                E2 = K.epilogue(o2, N, act=E.act, bias=bias if E.bias else None,
                                aux=(torch.empty_like(out) if E.aux else None), ldaux=E.ldaux,
                                colsum=(torch.empty(N, device=dev) if E.colsum else None))
                sets.append((K.dense(a2, la, *a2.shape), E2, a2))
        if mxq:
            q = K.mx_empty(M, N, dev)
            E.mx_q, E.mx_scales = q.q.data_ptr(), q.scales.data_ptr()
            E._keep = E._keep + (q,)
        if prec == "mx":
            qa = K.mx_quantize(a) if la == L.KC else K.mx_quantize_t(a)
            qb = K.mx_quantize(b) if lb == L.KC else K.mx_quantize_t(b)
            path = "mx"
            run = lambda: K.gemm_mxfp8(qa, qb, E)  # noqa: E731
        elif ROT > 1:
            path = L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1)
            it = [0]

            def run():
                A2, E2, _ = sets[it[0] % ROT]
                it[0] += 1
                K.gemm(A2, Bo, E2, M, N, Kd, L.BF16)
        else:
            path = L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1)
            run = lambda: K.gemm(A, Bo, E, M, N, Kd, L.BF16)  # noqa: E731
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        if GAP_MB > 0:
            src = torch.empty(GAP_MB << 20, dtype=torch.uint8, device=dev)
            dst = torch.empty_like(src)
            evs = []
            for _ in range(REPS):
                L.check(L.load().mia_stream_copy(src.data_ptr(), dst.data_ptr(), src.numel(), L.stream_ptr()), "copy")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                evs.append((e0, e1))
            torch.cuda.synchronize()
            ms = sum(a.elapsed_time(b) for a, b in evs) / REPS
            del src, dst
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REPS):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / REPS
        total += ms
        digest = ""
        if os.environ.get("CHECKSUM"):  # outputs of this build, to compare builds bit for bit across processes
            import hashlib
            h = hashlib.sha1(out.cpu().contiguous().view(torch.uint8).numpy().tobytes())
            if epi in ("gelu_save", "gelu_save_d"):
                h.update(u.cpu().contiguous().view(torch.uint8).numpy().tobytes())
            if E.colsum:
                h.update(cs.cpu().numpy().tobytes())
            digest = "  sha1 " + h.hexdigest()[:16]
        print(f"path {path} {name:11s} {epi + ('+mxq' if mxq else ''):15s} M={M:6d} N={N:5d} K={Kd:6d}  {ms:7.3f} ms  "
              f"{2 * M * N * Kd / ms / 1e9:7.1f} TF/s{digest}", flush=True)
        del a, b, A, Bo, E, out
        torch.cuda.empty_cache()
    print(f"total {total:.3f} ms per block (x12 per step)")


if __name__ == "__main__":
    main()
