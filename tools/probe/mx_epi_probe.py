# NOTE: written against the round-2 MX-fp8 attempt (mia_mxfp8_quant / MIA_FP8_MX operands), which was not
# kept; the findings are in DESIGN.md section 9 and profiles/r02_mxfp8_ast_attempt_tests.log.
"""Which MX-fp8 hipBLASLt shapes have an algorithm (ROCm 7.2, gfx950): M granularity, K = 768 + 96
(bias carried as three extra K blocks).  (Bias epilogues: none -- 'rocRoller does not support bias'.)"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "dl-sound-classification_amd"))
import torch  # noqa: E402
from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

dev = torch.device("cuda:0")
for M in (1040, 1056, 1088, 1152, 1280, 3290, 3328, 421120):
    for N, Kd in ((768, 768), (2304, 864), (768, 3168)):
        a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        w = torch.randn(N, Kd, device=dev) * 0.05
        qa, sa = K.mxfp8_quant(a, M, Kd)
        qw, sw = K.mxfp8_quant(w, N, Kd)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        try:
            K.gemm(K.dense_mx(qa, sa, M, Kd), K.dense_mx(qw, sw, N, Kd), K.epilogue(out, N), M, N, Kd, L.FP8_MX)
            torch.cuda.synchronize()
            r = "ok"
        except RuntimeError as e:
            r = "FAIL " + str(e)[-40:]
        print(f"M={M} N={N} K={Kd}: {r}", flush=True)
        del a, qa, sa, out
