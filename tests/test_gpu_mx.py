"""GPU: MX-fp8 (north_star config 5, trainer.precision=fp8-mixed) -- the quantiser byte for byte against the
OCP MX restatement in oracle/mx.py, and the hand-written v_mfma_scale_f32_16x16x128_f8f6f4 GEMM against the
float64 product of the dequantised operands with every epilogue the AST forward uses.  Parity with the
reference is unpinned (the reference has no fp8 path); these pin the kernels to the published format.
Tolerances: f32 outputs 1e-4 of max |C| (the scaled MFMA's internal sum is not f32-exact); bf16 outputs one bf16 rounding
(2^-8 relative) of max |C|."""
import pytest
import torch

from oracle import mx as omx
from src.miaudio import kernels as K
from src.miaudio import lib as L

pytestmark = pytest.mark.gpu


def _blocky(rows, cols, g, dtype):
    """Values whose 32-blocks span many binades, with zero blocks, saturating blocks and subnormal-scale
    blocks, so every branch of the scale rule is exercised."""
    x = torch.randn(rows, cols, generator=g)
    mag = torch.pow(2.0, torch.randint(-30, 30, (rows, cols // 32), generator=g).float())
    x = (x.reshape(rows, cols // 32, 32) * mag[..., None]).reshape(rows, cols)
    x[0, :32] = 0.0
    x[1 % rows, 32:64] = 1e-39 if dtype == torch.float32 else 0.0
    x[2 % rows, :32] = torch.linspace(-511.0, 511.0, 32)  # amax in [256, 512): elements past 448 saturate
    return x.to(dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols", [(3, 32), (77, 768), (1024, 3072), (5, 96)])
def test_mx_quantize_matches_oracle(cuda, dtype, rows, cols):
    g = torch.Generator().manual_seed(rows * 31 + cols)
    x = _blocky(rows, cols, g, dtype)
    mxt = K.mx_quantize(x.to(cuda))
    torch.cuda.synchronize()
    q_ref, s_ref = omx.quantize(x)
    assert torch.equal(mxt.scales.cpu(), s_ref)
    assert torch.equal(mxt.q.cpu(), q_ref)


def _mx_pair(M, N, Kd, g):
    a = torch.randn(M, Kd, generator=g) * torch.rand(M, 1, generator=g) * 4
    b = torch.randn(N, Kd, generator=g) * 0.05
    qa, sa = omx.quantize(a)
    qb, sb = omx.quantize(b)
    return qa, sa, qb, sb


def _to(cuda, *ts):
    return [t.to(cuda) for t in ts]


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 128), (1000, 768, 768), (513, 2304, 768), (777, 768, 3072),
                                    (300, 3072, 768)])
@pytest.mark.parametrize("epi", ["bf16_bias", "f32_plain", "f32_residual", "gelu_save", "gelu", "gelu_save_d"])
def test_gemm_mxfp8_vs_float64(cuda, M, N, Kd, epi):
    g = torch.Generator().manual_seed(M + 3 * N + 7 * Kd)
    qa, sa, qb, sb = _mx_pair(M, N, Kd, g)
    ref = omx.gemm(qa, sa, qb, sb)
    bias = torch.randn(N, generator=g)
    A = K.MXTensor(*_to(cuda, qa, sa))
    B = K.MXTensor(*_to(cuda, qb, sb))
    if epi == "f32_plain":
        out = torch.empty(M, N, device=cuda)
        K.gemm_mxfp8(A, B, K.epilogue(out, N))
        want = ref
    elif epi == "f32_residual":
        res = torch.randn(M, N, generator=g)
        out = torch.empty(M, N, device=cuda)
        K.gemm_mxfp8(A, B, K.epilogue(out, N, act=L.ACT_ADD_AUX, bias=bias.to(cuda), aux=res.to(cuda), ldaux=N))
        want = ref + bias.double() + res.double()
    elif epi == "bf16_bias":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        K.gemm_mxfp8(A, B, K.epilogue(out, N, bias=bias.to(cuda)))
        want = ref + bias.double()
    else:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        u = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        act = {"gelu_save": L.ACT_GELU_SAVE, "gelu_save_d": L.ACT_GELU_SAVE_D}.get(epi, L.ACT_GELU)
        saves = epi != "gelu"
        K.gemm_mxfp8(A, B, K.epilogue(out, N, act=act, bias=bias.to(cuda), aux=u if saves else None,
                                      ldaux=N if saves else 0))
        pre = (ref + bias.double()).to(torch.bfloat16).double()  # the Linear output rounds to bf16 first
        want = torch.nn.functional.gelu(pre)
        if epi == "gelu_save":
            torch.cuda.synchronize()
            du = (u.cpu().double() - pre).abs().max() / pre.abs().max()
            assert float(du) <= 2.0 ** -7, f"saved pre-activation off by {float(du):.3e}"  # one bf16 ulp
        elif epi == "gelu_save_d":  # gelu'(u) of the bf16 pre-activation, rounded to bf16
            torch.cuda.synchronize()
            x = pre.clone().requires_grad_(True)
            torch.nn.functional.gelu(x).backward(torch.ones_like(x))
            dd = (u.cpu().double() - x.grad).abs().max() / x.grad.abs().max()
            # u may round to the neighbouring bf16 (f32 accumulation order), gelu'' <= 0.49 amplifies it
            assert float(dd) <= 1e-2, f"saved gelu' off by {float(dd):.3e}"
    torch.cuda.synchronize()
    got = out.cpu().double()
    err = float((got - want).abs().max() / want.abs().max())
    # f32 outputs: the scaled e4m3 MFMA does not sum its 128 products exactly in f32 (measured 3.7e-5 of
    # max |C| at K = 128 against the float64 product of the same dequantised operands)
    tol = 1e-4 if out.dtype == torch.float32 else 2.0 ** -8
    assert err <= tol, f"{epi} {M}x{N}x{Kd}: rel err {err:.3e} > {tol:.1e}"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols", [(32, 3), (768, 77), (3072, 768), (96, 1000)])
def test_mx_quantize_t_is_quantize_of_the_transpose(cuda, dtype, rows, cols):
    """mia_mx_quantize_t (the fp8 backward-data operand W^T) byte for byte = the oracle's quantisation of x^T."""
    g = torch.Generator().manual_seed(rows * 7 + cols)
    x = _blocky(cols, rows, g, dtype).t().contiguous()  # blocks of 32 along the rows of x = rows of x^T
    mxt = K.mx_quantize_t(x.to(cuda))
    torch.cuda.synchronize()
    q_ref, s_ref = omx.quantize(x.t().contiguous())
    assert torch.equal(mxt.scales.cpu(), s_ref)
    assert torch.equal(mxt.q.cpu(), q_ref)


@pytest.mark.parametrize("M,N,Kd", [(1000, 3072, 768), (513, 768, 3072), (300, 768, 768)])
def test_gemm_mxfp8_dact_mul_colsum_vs_float64(cuda, M, N, Kd):
    """The fp8 backward-data of fc2 (x the saved gelu'(u), column sums of the stored bf16 values = fc1's bias
    gradient) on mia_gemm_mxfp8_ex against the float64 product of the dequantised operands."""
    g = torch.Generator().manual_seed(M * 5 + N + Kd)
    qa, sa, qb, sb = _mx_pair(M, N, Kd, g)
    ref = omx.gemm(qa, sa, qb, sb)
    d = (torch.rand(M, N, generator=g) * 1.2 - 0.1).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    cs = torch.empty(N, device=cuda)
    K.gemm_mxfp8(K.MXTensor(*_to(cuda, qa, sa)), K.MXTensor(*_to(cuda, qb, sb)),
                 K.epilogue(out, N, act=L.DACT_MUL, aux=d.to(cuda), ldaux=N, colsum=cs))
    torch.cuda.synchronize()
    want = ref * d.double()
    got = out.cpu().double()
    err = float((got - want).abs().max() / want.abs().max())
    # two bf16 roundings: the product is rounded into the epilogue's bf16 image before the multiply (as in
    # the bf16 kernel), the result again on store
    assert err <= 2.0 ** -7, f"{M}x{N}x{Kd}: rel err {err:.3e}"
    # the column sums are of the stored (rounded) values, in a fixed order
    cerr = float((cs.cpu().double() - got.sum(0)).abs().max() / got.abs().sum(0).max())
    assert cerr <= 1e-5, f"colsum rel err {cerr:.3e}"


def test_gemm_mxfp8_colsum_needs_the_dact_mul_epilogue(cuda):
    a = K.MXTensor(torch.zeros(256, 128, dtype=torch.uint8, device=cuda), torch.zeros(256, 4, dtype=torch.uint8,
                                                                                       device=cuda))
    out = torch.empty(256, 256, dtype=torch.bfloat16, device=cuda)
    cs = torch.empty(256, device=cuda)
    with pytest.raises(RuntimeError, match="gemm_mxfp8"):
        K.gemm_mxfp8(a, a, K.epilogue(out, 256, colsum=cs))


def test_gemm_mxfp8_rejects_bad_shapes(cuda):
    a = K.MXTensor(torch.zeros(256, 96, dtype=torch.uint8, device=cuda), torch.zeros(256, 3, dtype=torch.uint8,
                                                                                      device=cuda))
    out = torch.empty(256, 256, device=cuda)
    with pytest.raises(RuntimeError, match="multiple of 128"):
        K.gemm_mxfp8(a, a, K.epilogue(out, 256))


@pytest.mark.parametrize("rows,D", [(5, 768), (300, 768), (7, 384)])
def test_layernorm_fwd_mx_equals_quantised_bf16_output(cuda, rows, D):
    """mia_layernorm_fwd_mx: the bf16 y equals mia_layernorm_fwd's, and its MX copy equals
    mia_mx_quantize(y) byte for byte (the qkv / fc1 A operand under fp8-mixed)."""
    from src.models.ast_hip import _ln
    g = torch.Generator().manual_seed(rows + D)
    x = (torch.randn(rows, D, generator=g) * 3 + 1).to(cuda)
    w = (1 + 0.1 * torch.randn(D, generator=g)).to(cuda)
    b = (0.1 * torch.randn(D, generator=g)).to(cuda)
    y0, m0, r0, _ = _ln(x, w, b, torch.bfloat16, rows, D)
    y1, m1, r1, yq = _ln(x, w, b, torch.bfloat16, rows, D, mx=True)
    ref = K.mx_quantize(y0)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(m0, m1) and torch.equal(r0, r1)
    assert torch.equal(yq.scales, ref.scales) and torch.equal(yq.q, ref.q)


@pytest.mark.parametrize("B,N,H", [(2, 1645, 12), (1, 77, 2)])
def test_attn_fwd_mx_equals_quantised_bf16_output(cuda, B, N, H):
    """mia_attn_fwd_mx: the bf16 output equals mia_attn_fwd's and its MX copy equals mia_mx_quantize of it
    (the proj A operand under fp8-mixed)."""
    g = torch.Generator().manual_seed(N + H)
    qkv = torch.randn(B * N, 3 * H * 64, generator=g).to(torch.bfloat16).to(cuda)
    lib = L.load()
    out0 = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device=cuda)
    out1 = torch.empty_like(out0)
    lse0 = torch.empty(B, H, N, device=cuda)
    lse1 = torch.empty_like(lse0)
    q = K.mx_empty(B * N, H * 64, cuda)
    L.check(lib.mia_attn_fwd(qkv.data_ptr(), out0.data_ptr(), lse0.data_ptr(), L.BF16, B, N, H, 0.125,
                             L.stream_ptr()), "attn")
    L.check(lib.mia_attn_fwd_mx(qkv.data_ptr(), out1.data_ptr(), lse1.data_ptr(), q.q.data_ptr(),
                                q.scales.data_ptr(), B, N, H, 0.125, L.stream_ptr()), "attn_mx")
    ref = K.mx_quantize(out0)
    torch.cuda.synchronize()
    assert torch.equal(out0, out1) and torch.equal(lse0, lse1)
    assert torch.equal(q.scales, ref.scales) and torch.equal(q.q, ref.q)


@pytest.mark.parametrize("mode", ["bf16_gemm", "mx_gemm"])
def test_gelu_save_epilogue_mx_copy(cuda, mode):
    """The GELU_SAVE epilogue's MX copy of gelu(u) equals mia_mx_quantize of the bf16 gelu(u) it stores,
    on the bf16 256x256 kernel and on the MX kernel (fc1 feeding fc2 under fp8-mixed)."""
    M, N, Kd = 700, 3072, 768
    g = torch.Generator().manual_seed(5)
    a = torch.randn(M, Kd, generator=g)
    w = torch.randn(N, Kd, generator=g) * 0.05
    bias = (0.1 * torch.randn(N, generator=g)).to(cuda)
    gu = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    u = torch.empty_like(gu)
    q = K.mx_empty(M, N, cuda)
    E = K.epilogue(gu, N, act=L.ACT_GELU_SAVE, bias=bias, aux=u, ldaux=N, mx=q)
    if mode == "bf16_gemm":
        ab, wb = a.to(torch.bfloat16).to(cuda), w.to(torch.bfloat16).to(cuda)
        K.gemm(K.dense(ab, L.KC, M, Kd), K.dense(wb, L.KC, N, Kd), E, M, N, Kd, L.BF16)
    else:
        K.gemm_mxfp8(K.mx_quantize(a.to(cuda)), K.mx_quantize(w.to(cuda)), E)
    ref = K.mx_quantize(gu)
    torch.cuda.synchronize()
    assert torch.equal(q.scales, ref.scales) and torch.equal(q.q, ref.q)


@pytest.mark.parametrize("rows", [5, 300])
def test_layernorm_bwd_mx_equals_quantised_bf16_dx2(cuda, rows):
    """mia_layernorm_bwd_colsum_mx (fp8-mixed backward): dx, dx2, dgamma, dbeta and the column sums equal
    mia_layernorm_bwd_colsum's, and the MX copy equals mia_mx_quantize(dx2) byte for byte (the proj / fc2
    backward-data A operand)."""
    from src.models.ast_hip import _ln_bwd
    D = 768
    g = torch.Generator().manual_seed(rows + 11)
    x = (torch.randn(rows, D, generator=g) * 3 + 1).to(cuda)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-6)
    w = (1 + 0.1 * torch.randn(D, generator=g)).to(cuda)
    dy = torch.randn(rows, D, generator=g).to(torch.bfloat16).to(cuda)
    base = torch.randn(rows, D, generator=g).to(cuda)
    out = []
    for mx in (False, True):
        dx = base.clone()
        dx2 = torch.empty(rows, D, dtype=torch.bfloat16, device=cuda)
        q = K.mx_empty(rows, D, cuda) if mx else None
        out.append((dx, dx2, q, *_ln_bwd(dy, x, w, mean, rstd, dx, rows, D, True, dx2=dx2, dx2_mx=q)))
    ref = K.mx_quantize(out[0][1])
    torch.cuda.synchronize()
    for a, b in zip(out[0][:2] + out[0][3:], out[1][:2] + out[1][3:]):
        assert torch.equal(a, b)
    q = out[1][2]
    assert torch.equal(q.scales, ref.scales) and torch.equal(q.q, ref.q)


@pytest.mark.parametrize("mode", ["bf16_gemm", "mx_gemm"])
def test_dact_mul_epilogue_mx_copy(cuda, mode):
    """The fc2 backward-data epilogue (x saved gelu'(u), column sums) with an MX copy of its stored bf16
    output (fc1's fp8 backward-data A operand): the copy equals mia_mx_quantize of the stored values, and
    the bf16 output and column sums are unchanged by asking for it."""
    M, N, Kd = 700, 3072, 768
    g = torch.Generator().manual_seed(5)
    d = (torch.rand(M, N, generator=g) * 1.2 - 0.1).to(torch.bfloat16).to(cuda)
    res = []
    for with_mx in (False, True):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        cs = torch.empty(N, device=cuda)
        q = K.mx_empty(M, N, cuda) if with_mx else None
        E = K.epilogue(out, N, act=L.DACT_MUL, aux=d, ldaux=N, colsum=cs, mx=q)
        if mode == "mx_gemm":
            qa, sa, qb, sb = _mx_pair(M, N, Kd, torch.Generator().manual_seed(9))
            K.gemm_mxfp8(K.MXTensor(*_to(cuda, qa, sa)), K.MXTensor(*_to(cuda, qb, sb)), E)
        else:
            gg = torch.Generator().manual_seed(9)
            a = torch.randn(M, Kd, generator=gg).to(torch.bfloat16).to(cuda)
            b = (torch.randn(Kd, N, generator=gg) * 0.05).to(torch.bfloat16).to(cuda)
            K.gemm(K.dense(a, L.KC, M, Kd), K.dense(b, L.RC, Kd, N), E, M, N, Kd, L.BF16)
        res.append((out, cs, q))
    ref = K.mx_quantize(res[1][0])
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert torch.equal(res[1][2].scales, ref.scales) and torch.equal(res[1][2].q, ref.q)

