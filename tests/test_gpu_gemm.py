"""GPU: the implicit-GEMM MFMA kernel against a float64 PyTorch reference of the same op
(dense GEMM in every layout, conv fwd / dgrad / wgrad gathers, pre-ops, epilogues, split-K).
Tolerances: f32 compute 1e-5 rel (exact-f32 MFMA), bf16 compute 2e-2 rel (bf16 operands)."""
import pytest
import torch
import torch.nn.functional as F

from src.miaudio import kernels as K
from src.miaudio import lib as L

pytestmark = pytest.mark.gpu
TOL = {L.F32: 1e-5, L.BF16: 2e-2}


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _mat(layout, rows_logical, k, dt, dev, g):
    """Return (tensor, operand) for a logical [rows][k] matrix stored per layout."""
    src = torch.randn(rows_logical, k, generator=g).to(dt)
    if layout == L.KC:
        t = src.contiguous().to(dev)
        return src, K.dense(t, L.KC, rows_logical, k), t
    t = src.t().contiguous().to(dev)
    return src, K.dense(t, L.RC, k, rows_logical), t


@pytest.mark.parametrize("cd", [L.F32, L.BF16])
@pytest.mark.parametrize("la,lb", [(L.KC, L.KC), (L.KC, L.RC), (L.RC, L.KC), (L.RC, L.RC)])
@pytest.mark.parametrize("M,N,Kd", [(256, 128, 96), (37, 50, 200), (300, 32, 64), (64, 600, 40), (130, 70, 8)])
def test_dense_layouts(cuda, cd, la, lb, M, N, Kd):
    g = torch.Generator().manual_seed(M * 7 + N + Kd)
    dt = torch.float32 if cd == L.F32 else torch.bfloat16
    a, A, ta = _mat(la, M, Kd, dt, cuda, g)
    b, Bo, tb = _mat(lb, N, Kd, dt, cuda, g)
    out = torch.empty(M, N, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(out, N), M, N, Kd, cd)
    torch.cuda.synchronize()
    ref = a.double() @ b.double().t()
    assert rel(out.cpu(), ref) < TOL[cd]


@pytest.mark.parametrize("split", [1, 3, 8])
def test_split_k_bias_relu_bf16_out(cuda, split):
    g = torch.Generator().manual_seed(1)
    M, N, Kd = 200, 300, 1000
    a = torch.randn(M, Kd, generator=g)
    w = torch.randn(N, Kd, generator=g)
    bias = torch.randn(N, generator=g)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    ta, tw, tb = a.to(cuda), w.to(cuda), bias.to(cuda)
    K.gemm(K.dense(ta, L.KC, M, Kd), K.dense(tw, L.KC, N, Kd), K.epilogue(out, N, act=L.ACT_RELU, bias=tb),
           M, N, Kd, L.F32, split_k=split)
    torch.cuda.synchronize()
    ref = torch.relu(a.double() @ w.double().t() + bias.double())
    assert rel(out.float().cpu(), ref) < 1e-2


def test_dact_nz_and_accumulate(cuda):
    g = torch.Generator().manual_seed(2)
    M, N, Kd = 64, 96, 48
    a = torch.randn(M, Kd, generator=g)
    w = torch.randn(N, Kd, generator=g)
    aux = torch.relu(torch.randn(M, N, generator=g))
    base = torch.randn(M, N, generator=g)
    out = base.clone().to(cuda)
    K.gemm(K.dense(a.to(cuda), L.KC, M, Kd), K.dense(w.to(cuda), L.KC, N, Kd),
           K.epilogue(out, N, act=L.DACT_NZ, aux=aux.to(cuda), ldaux=N, act_scale=2.0, accumulate=True), M, N, Kd,
           L.F32)
    torch.cuda.synchronize()
    ref = base.double() + (a.double() @ w.double().t()) * (aux != 0).double() * 2.0
    assert rel(out.cpu(), ref) < 1e-5


def _conv_case(cuda, cd, n, cin, cout, h, w, kh, kw, sw, pre):
    g = torch.Generator().manual_seed(n * 100 + cin + kw)
    dt = torch.float32 if cd == L.F32 else torch.bfloat16
    x = torch.randn(n, h, w, cin, generator=g).to(dt)
    wt = torch.randn(cout, cin, kh, kw, generator=g) / (cin * kh * kw) ** 0.5
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.1
    oh, ow = h - kh + 1, (w - kw) // sw + 1
    xin = x.double()
    if pre:
        xin = torch.relu(xin * sc.double() + sh.double())
    ref = F.conv2d(xin.permute(0, 3, 1, 2), wt.double(), stride=(1, sw)).permute(0, 2, 3, 1)
    return x, wt, sc, sh, oh, ow, ref


@pytest.mark.parametrize("cd", [L.F32, L.BF16])
@pytest.mark.parametrize("case", [
    (2, 32, 32, 12, 40, 8, 8, 1, True),   # trunk 8x8 with fused BN+ReLU
    (2, 32, 64, 1, 300, 1, 16, 2, True),  # frontend conv2 (stride 2)
    (3, 64, 128, 4, 30, 1, 2, 1, False),  # trunk (1,2)
    (2, 1, 32, 16, 60, 8, 8, 1, False),   # 1-channel 8x8 (CONVROW)
])
def test_conv_fwd_dgrad_wgrad(cuda, cd, case):
    n, cin, cout, h, w, kh, kw, sw, pre = case
    x, wt, sc, sh, oh, ow, ref = _conv_case(cuda, cd, n, cin, cout, h, w, kh, kw, sw, pre)
    tx = x.contiguous().to(cuda)
    tsc, tsh = sc.to(cuda), sh.to(cuda)
    wp = K.pack_weight(wt.contiguous().to(cuda), cd, 0)
    out = torch.empty(n * oh * ow, cout, dtype=torch.float32, device=cuda)
    rowk = cin % 8 != 0
    preop = L.PRE_AFFINE_RELU if pre else L.PRE_NONE
    A = K.conv(tx, L.KC, n, h, w, cin, oh, ow, kh, kw, sw=sw, pre=preop, scale=tsc, shift=tsh, row_kind=rowk)
    K.gemm(A, K.dense(wp, L.KC, cout, kh * kw * cin), K.epilogue(out, cout), n * oh * ow, cout, kh * kw * cin, cd)
    torch.cuda.synchronize()
    assert rel(out.view(n, oh, ow, cout).cpu(), ref) < TOL[cd] * 2

    # wgrad: dW = dy^T im2col(x)
    g = torch.Generator().manual_seed(7)
    dy = torch.randn(n, oh, ow, cout, generator=g).to(x.dtype)
    xin = x.double()
    if pre:
        xin = torch.relu(xin * sc.double() + sh.double())
    xr = xin.permute(0, 3, 1, 2).requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=(1, sw))
    yr.backward(dy.double().permute(0, 3, 1, 2))
    P = n * oh * ow
    tdy = dy.contiguous().to(cuda)
    dW = torch.empty(cout, kh * kw * cin, dtype=torch.float32, device=cuda)
    Bop = K.conv(tx, L.RC, n, h, w, cin, oh, ow, kh, kw, sw=sw, pre=preop, scale=tsc, shift=tsh, row_kind=rowk)
    K.gemm(K.dense(tdy, L.RC, P, cout), Bop, K.epilogue(dW, kh * kw * cin), cout, kh * kw * cin, P, cd)
    gw = torch.empty(cout, cin, kh, kw, device=cuda)
    K.unpack_ohwi_grad(dW, (cout, cin, kh, kw), gw)
    torch.cuda.synchronize()
    assert rel(gw.cpu(), wr.grad) < TOL[cd] * 2

    # dgrad (stride 1, cin % 8 == 0): conv of padded dy with the flipped kernel
    if sw == 1 and cin % 8 == 0:
        wf = K.pack_weight(wt.contiguous().to(cuda), cd, 1)
        dx = torch.empty(n * h * w, cin, dtype=torch.float32, device=cuda)
        Kd = kh * kw * cout
        K.gemm(K.conv(tdy, L.KC, n, oh, ow, cout, h, w, kh, kw, ph=kh - 1, pw=kw - 1), K.dense(wf, L.KC, cin, Kd),
               K.epilogue(dx, cin), n * h * w, cin, Kd, cd)
        torch.cuda.synchronize()
        gref = xr.grad.permute(0, 2, 3, 1)  # gradient w.r.t. the conv input (after the pre-op)
        assert rel(dx.view(n, h, w, cin).cpu(), gref) < TOL[cd] * 2


@pytest.mark.parametrize("cd", [L.F32, L.BF16])
def test_stride2_parity_dgrad(cuda, cd):
    """Frontend conv2 dgrad as two stride-1 parity convolutions with a row-map epilogue."""
    g = torch.Generator().manual_seed(3)
    n, cin, cout, W1, kw = 2, 32, 64, 301, 16
    W2 = (W1 - kw) // 2 + 1
    dt = torch.float32 if cd == L.F32 else torch.bfloat16
    wt = torch.randn(cout, cin, 1, kw, generator=g) / 20
    dy = torch.randn(n, 1, W2, cout, generator=g).to(dt)
    xr = torch.zeros(n, cin, 1, W1, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wt.double(), stride=(1, 2)).backward(dy.double().permute(0, 3, 1, 2))
    tdy = dy.contiguous().to(cuda)
    wpar = K.pack_weight(wt.contiguous().to(cuda), cd, 2).view(2, -1)
    dx = torch.empty(n * W1, cin, dtype=torch.float32, device=cuda)
    for par in (0, 1):
        Tp = (W1 - par + 1) // 2
        K.gemm(K.conv(tdy, L.KC, n, 1, W2, cout, 1, Tp, 1, kw // 2, pw=kw // 2 - 1), K.dense(wpar[par], L.KC, cin, 512),
               K.epilogue(dx, cin, rowmap=(Tp, W1, 2, par)), n * Tp, cin, 512, cd)
    torch.cuda.synchronize()
    assert rel(dx.view(n, W1, cin).cpu(), xr.grad[:, :, 0].permute(0, 2, 1)) < TOL[cd] * 2


@pytest.mark.parametrize("cd", [L.F32, L.BF16])
def test_single_channel_dgrad_rowsplit(cuda, cd):
    """1-channel 8x8 conv dgrad via the (ky) row-split GEMM + col2im_rows."""
    g = torch.Generator().manual_seed(4)
    n, cout, H, W, kh, kw = 2, 32, 20, 50, 8, 8
    ha, wa = H - kh + 1, W - kw + 1
    dt = torch.float32 if cd == L.F32 else torch.bfloat16
    wt = torch.randn(cout, 1, kh, kw, generator=g) / 8
    dy = torch.randn(n, ha, wa, cout, generator=g).to(dt)
    xr = torch.zeros(n, 1, H, W, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wt.double()).backward(dy.double().permute(0, 3, 1, 2))
    tdy = dy.contiguous().to(cuda)
    wr = K.pack_weight(wt.contiguous().to(cuda), cd, 3)
    Pm = torch.empty(n * ha * W, kh, dtype=torch.float32, device=cuda)
    K.gemm(K.conv(tdy, L.KC, n, ha, wa, cout, ha, W, 1, kw, pw=kw - 1), K.dense(wr, L.KC, kh, kw * cout),
           K.epilogue(Pm, kh), n * ha * W, kh, kw * cout, cd)
    dx = torch.empty(n, H, W, dtype=torch.float32, device=cuda)
    K.col2im_rows(Pm, n, ha, W, kh, dx)
    torch.cuda.synchronize()
    assert rel(dx.cpu(), xr.grad[:, 0]) < TOL[cd] * 2


@pytest.mark.parametrize("case", [
    # n, cin, cout, h, w, kh, kw, sw, pre, src dtype
    (2, 32, 32, 10, 600, 8, 8, 1, True, torch.bfloat16),    # conv4 shape: several 256-px tiles + tail
    (2, 32, 32, 9, 300, 8, 8, 1, False, torch.float32),     # f32 storage, bf16 compute
    (2, 32, 64, 1, 3001, 1, 16, 2, True, torch.bfloat16),   # conv2: stride 2, de-interleaved window
    (2, 32, 32, 1, 1001, 1, 16, 2, False, torch.float32),   # stride 2, N = 32
    (2, 64, 64, 3, 700, 1, 8, 1, False, torch.bfloat16),    # C = 64, N = 64
    (2, 64, 32, 2, 555, 1, 8, 1, True, torch.bfloat16),     # C = 64, N = 32 (parity-dgrad shape)
])
def test_rowconv_path(cuda, case):
    """The row-window direct conv (mia_gemm_path == 1) against a float64 conv2d."""
    n, cin, cout, h, w, kh, kw, sw, pre, sdt = case
    g = torch.Generator().manual_seed(h * w + cin)
    x = torch.randn(n, h, w, cin, generator=g).to(torch.bfloat16).to(sdt)
    wt = (torch.randn(cout, cin, kh, kw, generator=g) / (cin * kh * kw) ** 0.5).to(torch.bfloat16).float()
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.1
    bias = torch.randn(cout, generator=g)
    oh, ow = h - kh + 1, (w - kw) // sw + 1
    xin = x.double()
    if pre:
        xin = torch.relu(xin * sc.double() + sh.double())
    ref = F.conv2d(xin.permute(0, 3, 1, 2), wt.double(), bias.double(), stride=(1, sw)).permute(0, 2, 3, 1)
    tx = x.contiguous().to(cuda)
    wp = K.pack_weight(wt.contiguous().to(cuda), L.BF16, 0)
    preop = L.PRE_AFFINE_RELU if pre else L.PRE_NONE
    A = K.conv(tx, L.KC, n, h, w, cin, oh, ow, kh, kw, sw=sw, pre=preop, scale=sc.to(cuda), shift=sh.to(cuda))
    Bo = K.dense(wp, L.KC, cout, kh * kw * cin)
    Kd = kh * kw * cin
    assert L.load().mia_gemm_path(A, Bo, n * oh * ow, cout, Kd, L.BF16, 1) == 1
    for odt in (torch.float32, torch.bfloat16):
        out = torch.empty(n * oh * ow, cout, dtype=odt, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, cout, bias=bias.to(cuda)), n * oh * ow, cout, Kd, L.BF16)
        torch.cuda.synchronize()
        assert rel(out.float().view(n, oh, ow, cout).cpu(), ref) < 2e-2


def test_rowconv_padded_dgrad(cuda):
    """conv4 dgrad through the row-window path: padded dY (ph = pw = 7) x flipped weights."""
    g = torch.Generator().manual_seed(11)
    n, cin, cout, h, w, kh, kw = 2, 32, 32, 12, 400, 8, 8
    oh, ow = h - kh + 1, w - kw + 1
    wt = (torch.randn(cout, cin, kh, kw, generator=g) / 40).to(torch.bfloat16).float()
    dy = torch.randn(n, oh, ow, cout, generator=g).to(torch.bfloat16)
    xr = torch.zeros(n, cin, h, w, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wt.double()).backward(dy.double().permute(0, 3, 1, 2))
    wf = K.pack_weight(wt.contiguous().to(cuda), L.BF16, 1)
    A = K.conv(dy.contiguous().to(cuda), L.KC, n, oh, ow, cout, h, w, kh, kw, ph=kh - 1, pw=kw - 1)
    Bo = K.dense(wf, L.KC, cin, kh * kw * cout)
    assert L.load().mia_gemm_path(A, Bo, n * h * w, cin, kh * kw * cout, L.BF16, 1) == 1
    dx = torch.empty(n * h * w, cin, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(dx, cin), n * h * w, cin, kh * kw * cout, L.BF16)
    torch.cuda.synchronize()
    assert rel(dx.view(n, h, w, cin).cpu(), xr.grad.permute(0, 2, 3, 1)) < 2e-2


@pytest.mark.parametrize("case", [
    # n, cin, cout, h, w, kh, kw, sw, pre, dtype
    (2, 32, 32, 12, 700, 8, 8, 1, True, torch.bfloat16),    # conv4 wgrad
    (2, 32, 64, 1, 3001, 1, 16, 2, True, torch.bfloat16),   # conv2 wgrad (stride 2)
    (3, 32, 64, 4, 300, 1, 4, 1, True, torch.bfloat16),     # trunk conv5 (1x4, 32 -> 64)
    (3, 64, 64, 4, 300, 1, 4, 1, False, torch.bfloat16),    # trunk conv6 (1x4, 64 -> 64)
    (2, 32, 32, 9, 333, 8, 8, 1, False, torch.float32),     # f32 storage
    (2, 32, 32, 1, 901, 1, 16, 2, False, torch.bfloat16),   # stride 2, Cout 32
])
def test_rowwgrad_path(cuda, case):
    """The row-window weight-gradient kernel (mia_gemm_path == 2) against float64 autograd."""
    n, cin, cout, h, w, kh, kw, sw, pre, dt = case
    g = torch.Generator().manual_seed(h * w + cout)
    x = torch.randn(n, h, w, cin, generator=g).to(torch.bfloat16).to(dt)
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.1
    oh, ow = h - kh + 1, (w - kw) // sw + 1
    dy = torch.randn(n, oh, ow, cout, generator=g).to(torch.bfloat16).to(dt)
    xin = x.double()
    if pre:
        xin = torch.relu(xin * sc.double() + sh.double())
    wr = torch.zeros(cout, cin, kh, kw, dtype=torch.float64, requires_grad=True)
    F.conv2d(xin.permute(0, 3, 1, 2), wr, stride=(1, sw)).backward(dy.double().permute(0, 3, 1, 2))
    P, Kc = n * oh * ow, kh * kw * cin
    preop = L.PRE_AFFINE_RELU if pre else L.PRE_NONE
    A = K.dense(dy.contiguous().to(cuda), L.RC, P, cout)
    Bo = K.conv(x.contiguous().to(cuda), L.RC, n, h, w, cin, oh, ow, kh, kw, sw=sw, pre=preop,
                scale=sc.to(cuda), shift=sh.to(cuda))
    assert L.load().mia_gemm_path(A, Bo, cout, Kc, P, L.BF16, 2) == 2
    dW = torch.empty(cout, Kc, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(dW, Kc), cout, Kc, P, L.BF16)
    gw = torch.empty(cout, cin, kh, kw, device=cuda)
    K.unpack_ohwi_grad(dW, (cout, cin, kh, kw), gw)
    torch.cuda.synchronize()
    assert rel(gw.cpu(), wr.grad) < 2e-2


@pytest.mark.parametrize("dydt", [torch.bfloat16, torch.float32])
def test_tapwgrad_conv1(cuda, dydt):
    """Frontend conv1 weight gradient (1x64 taps, stride 2 over the waveform) through path 3."""
    g = torch.Generator().manual_seed(21)
    n, T = 3, 2 * 3001 + 64
    W1 = (T - 64) // 2 + 1
    x = torch.randn(n, T, generator=g)
    dy = torch.randn(n, W1, 32, generator=g).to(torch.bfloat16).to(dydt)
    wr = torch.zeros(32, 1, 1, 64, dtype=torch.float64, requires_grad=True)
    xb = x.to(torch.bfloat16).double()  # the kernel rounds the waveform to bf16 like the fwd operand
    F.conv2d(xb.view(n, 1, 1, T), wr, stride=(1, 2)).backward(dy.double().permute(0, 2, 1).unsqueeze(2))
    A = K.dense(dy.contiguous().to(cuda), L.RC, n * W1, 32)
    Bo = K.conv(x.to(cuda), L.RC, n, 1, T // 2, 2, 1, W1, 1, 32, row_kind=True)
    assert L.load().mia_gemm_path(A, Bo, 32, 64, n * W1, L.BF16, 2) == 3
    dW = torch.empty(32, 64, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(dW, 64), 32, 64, n * W1, L.BF16)
    torch.cuda.synchronize()
    assert rel(dW.cpu(), wr.grad.view(32, 64)) < 1e-2


@pytest.mark.parametrize("xdt", [torch.bfloat16, torch.float32])
def test_tapwgrad_conv3(cuda, xdt):
    """Trunk conv3 weight gradient (1 -> 32 channels, 8x8) through path 3."""
    g = torch.Generator().manual_seed(22)
    n, H, W = 2, 20, 600
    ha, wa = H - 7, W - 7
    x = torch.randn(n, H, W, generator=g).to(torch.bfloat16).to(xdt)
    dy = torch.randn(n, ha, wa, 32, generator=g).to(torch.bfloat16)
    wr = torch.zeros(32, 1, 8, 8, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double().unsqueeze(1), wr).backward(dy.double().permute(0, 3, 1, 2))
    A = K.dense(dy.contiguous().to(cuda), L.RC, n * ha * wa, 32)
    Bo = K.conv(x.contiguous().to(cuda), L.RC, n, H, W, 1, ha, wa, 8, 8, row_kind=True)
    assert L.load().mia_gemm_path(A, Bo, 32, 64, n * ha * wa, L.BF16, 2) == 3
    dW = torch.empty(32, 64, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(dW, 64), 32, 64, n * ha * wa, L.BF16)
    torch.cuda.synchronize()
    assert rel(dW.cpu(), wr.grad.view(32, 64)) < 1e-2


@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_tapconv_conv1_fwd(cuda, odt):
    """Frontend conv1 forward (1x64 taps, stride 2, bias) through path 4."""
    g = torch.Generator().manual_seed(31)
    n, T = 3, 2 * 3001 + 64
    W1 = (T - 64) // 2 + 1
    x = torch.randn(n, T, generator=g)
    wt = (torch.randn(32, 1, 1, 64, generator=g) / 8).to(torch.bfloat16).float()
    bias = torch.randn(32, generator=g)
    ref = F.conv2d(x.to(torch.bfloat16).double().view(n, 1, 1, T), wt.double(), bias.double(), stride=(1, 2))
    ref = ref[:, :, 0].permute(0, 2, 1)
    wp = K.pack_weight(wt.contiguous().to(cuda), L.BF16, 0)
    A = K.conv(x.to(cuda), L.KC, n, 1, T // 2, 2, 1, W1, 1, 32, row_kind=True)
    Bo = K.dense(wp, L.KC, 32, 64)
    assert L.load().mia_gemm_path(A, Bo, n * W1, 32, 64, L.BF16, 1) == 4
    out = torch.empty(n * W1, 32, dtype=odt, device=cuda)
    K.gemm(A, Bo, K.epilogue(out, 32, bias=bias.to(cuda)), n * W1, 32, 64, L.BF16)
    torch.cuda.synchronize()
    assert rel(out.float().view(n, W1, 32).cpu(), ref) < 1e-2


@pytest.mark.parametrize("xdt", [torch.bfloat16, torch.float32])
def test_tapconv_conv3_fwd(cuda, xdt):
    """Trunk conv3 forward (1 -> 32 channels, 8x8) through path 4."""
    g = torch.Generator().manual_seed(32)
    n, H, W = 2, 20, 700
    ha, wa = H - 7, W - 7
    x = torch.randn(n, H, W, generator=g).to(torch.bfloat16).to(xdt)
    wt = (torch.randn(32, 1, 8, 8, generator=g) / 8).to(torch.bfloat16).float()
    bias = torch.randn(32, generator=g)
    ref = F.conv2d(x.double().unsqueeze(1), wt.double(), bias.double()).permute(0, 2, 3, 1)
    wp = K.pack_weight(wt.contiguous().to(cuda), L.BF16, 0)
    A = K.conv(x.contiguous().to(cuda), L.KC, n, H, W, 1, ha, wa, 8, 8, row_kind=True)
    Bo = K.dense(wp, L.KC, 32, 64)
    assert L.load().mia_gemm_path(A, Bo, n * ha * wa, 32, 64, L.BF16, 1) == 4
    out = torch.empty(n * ha * wa, 32, dtype=torch.bfloat16, device=cuda)
    K.gemm(A, Bo, K.epilogue(out, 32, bias=bias.to(cuda)), n * ha * wa, 32, 64, L.BF16)
    torch.cuda.synchronize()
    assert rel(out.float().view(n, ha, wa, 32).cpu(), ref) < 1e-2


@pytest.mark.parametrize("la,lb", [(L.KC, L.KC), (L.KC, L.RC), (L.RC, L.KC), (L.RC, L.RC)])
@pytest.mark.parametrize("M,N,Kd,split", [(256, 256, 128, 1), (296, 200, 192, 1), (128, 1000, 512, 1),
                                          (256, 384, 4096, 4), (64, 72, 64, 1)])
def test_dgemm_path(cuda, la, lb, M, N, Kd, split):
    """The LDS-DMA dense bf16 GEMM (mia_gemm_path == 5) against float64, every layout pair."""
    g = torch.Generator().manual_seed(M + N + Kd)
    a, A, ta = _mat(la, M, Kd, torch.bfloat16, cuda, g)
    b, Bo, tb = _mat(lb, N, Kd, torch.bfloat16, cuda, g)
    assert L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, split) == 5
    bias = torch.randn(N, generator=g)
    out = torch.empty(M, N, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(out, N, bias=bias.to(cuda)), M, N, Kd, L.BF16, split_k=split)
    torch.cuda.synchronize()
    ref = a.double() @ b.double().t() + bias.double()
    assert rel(out.cpu(), ref) < 1e-3


def _gelu_grad(x):
    x = x.double().requires_grad_(True)
    F.gelu(x).backward(torch.ones_like(x))
    return x.grad


@pytest.mark.parametrize("act", ["relu", "gelu_save", "dact_gelu", "add_aux", "gelu_save_d", "dact_mul"])
def test_dgemm_epilogues(cuda, act):
    g = torch.Generator().manual_seed(5)
    M, N, Kd = 320, 256, 256
    a = torch.randn(M, Kd, generator=g).to(torch.bfloat16)
    w = torch.randn(N, Kd, generator=g).to(torch.bfloat16)
    aux = torch.randn(M, N, generator=g).to(torch.bfloat16)
    A, Bo = K.dense(a.to(cuda), L.KC, M, Kd), K.dense(w.to(cuda), L.KC, N, Kd)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    z = a.double() @ w.double().t()
    taux = aux.to(cuda).clone()
    code = {"relu": L.ACT_RELU, "gelu_save": L.ACT_GELU_SAVE, "dact_gelu": L.DACT_GELU, "add_aux": L.ACT_ADD_AUX,
            "gelu_save_d": L.ACT_GELU_SAVE_D, "dact_mul": L.DACT_MUL}[act]
    K.gemm(A, Bo, K.epilogue(out, N, act=code, aux=None if act == "relu" else taux, ldaux=N), M, N, Kd, L.BF16)
    torch.cuda.synchronize()
    if act == "relu":
        ref = torch.relu(z)
    elif act == "gelu_save":
        ref = F.gelu(z)
        assert rel(taux.float().cpu(), z) < 1e-2  # pre-activation saved into aux
    elif act == "gelu_save_d":
        ref = F.gelu(z)
        assert rel(taux.float().cpu(), _gelu_grad(z)) < 1e-2  # gelu'(pre-activation) saved into aux
    elif act == "dact_gelu":
        ref = z * _gelu_grad(aux)
    elif act == "dact_mul":
        ref = z * aux.double()
    else:
        ref = z + aux.double()
    assert rel(out.float().cpu(), ref) < 1e-2


@pytest.mark.parametrize("act", ["gelu_save_d", "dact_mul"])
@pytest.mark.parametrize("cd", [L.F32, L.BF16])
def test_gelu_derivative_epilogues_generic(cuda, act, cd):
    """GELU_SAVE_D / DACT_MUL on the generic tile kernel (f32 compute, f32 aux -- the AST f32 path -- and a
    ragged bf16 shape): aux = gelu'(u), out = gelu(u); out = acc * aux."""
    g = torch.Generator().manual_seed(9)
    M, N, Kd = 130, 70, 40
    dt = torch.float32 if cd == L.F32 else torch.bfloat16
    a = torch.randn(M, Kd, generator=g).to(dt)
    w = torch.randn(N, Kd, generator=g).to(dt)
    aux = torch.randn(M, N, generator=g).to(dt)
    taux = aux.to(cuda).clone()
    out = torch.empty(M, N, dtype=dt, device=cuda)
    code = L.ACT_GELU_SAVE_D if act == "gelu_save_d" else L.DACT_MUL
    K.gemm(K.dense(a.to(cuda), L.KC, M, Kd), K.dense(w.to(cuda), L.KC, N, Kd), K.epilogue(out, N, act=code, aux=taux,
           ldaux=N), M, N, Kd, cd)
    torch.cuda.synchronize()
    z = a.double() @ w.double().t()
    tol = TOL[cd] if cd == L.BF16 else 1e-5
    if act == "gelu_save_d":
        assert rel(out.cpu(), F.gelu(z)) < tol
        assert rel(taux.cpu(), _gelu_grad(z)) < tol
    else:
        assert rel(out.cpu(), z * aux.double()) < tol


@pytest.mark.parametrize("n,oh,ow", [(2, 57, 853), (3, 10, 121), (1, 57, 129)])
def test_conv1ch_dgrad_bf16(cuda, n, oh, ow):
    """Single-input-channel 8x8 conv backward-data (EnvNet trunk conv3) vs float64 conv_transpose2d
    of the same bf16-rounded operands."""
    g = torch.Generator().manual_seed(oh * 1000 + ow)
    dy = torch.randn(n, oh, ow, 32, generator=g).to(torch.bfloat16)
    w = torch.randn(32, 1, 8, 8, generator=g) * 0.1
    out = torch.empty(n, oh + 7, ow + 7, dtype=torch.bfloat16, device=cuda)
    K.conv1ch_dgrad(dy.to(cuda).reshape(-1, 32), w.to(cuda), n, oh, ow, out)
    torch.cuda.synchronize()
    wb = w.to(torch.bfloat16).double()
    ref = F.conv_transpose2d(dy.double().permute(0, 3, 1, 2), wb)[:, 0]
    assert rel(out.float().cpu(), ref) < 1e-2


def _big_operands(cuda, la, lb, M, N, Kd, seed):
    g = torch.Generator(device=cuda).manual_seed(seed)
    a = torch.randn(M, Kd, generator=g, device=cuda).to(torch.bfloat16)
    b = torch.randn(N, Kd, generator=g, device=cuda).to(torch.bfloat16)
    ta = a.contiguous() if la == L.KC else a.t().contiguous()
    tb = b.contiguous() if lb == L.KC else b.t().contiguous()
    A = K.dense(ta, L.KC, M, Kd) if la == L.KC else K.dense(ta, L.RC, Kd, M)
    Bo = K.dense(tb, L.KC, N, Kd) if lb == L.KC else K.dense(tb, L.RC, Kd, N)
    return a, b, A, Bo, g


@pytest.mark.parametrize("la,lb", [(L.KC, L.KC), (L.KC, L.RC), (L.RC, L.KC), (L.RC, L.RC)])
@pytest.mark.parametrize("M,N,Kd", [(4096, 768, 768), (4136, 2304, 512), (8192, 264, 3072), (8200, 520, 1024)])
def test_mgemm_layouts(cuda, la, lb, M, N, Kd):
    """The 256x256 8-wave kernel (path 7, csrc/mgemm.hip) on every layout pair -- k-contiguous operands
    read with ds_read_b128, k-by-m operands with ds_read_b64_tr_b16 -- ragged M (rows past M read as
    zeros through the buffer range) and N (a 264-wide output: a partial column tile), bias + bf16 out,
    vs a PyTorch fp32 matmul of the same bf16 operands.  Nothing is written outside the output."""
    a, b, A, Bo, g = _big_operands(cuda, la, lb, M, N, Kd, M + N + Kd + 7 * la + 3 * lb)
    assert L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1) == 7
    bias = torch.randn(N, generator=g, device=cuda)
    ref = a.float() @ b.float().t() + bias
    full = torch.full((M + 3, N + 8), float("nan"), dtype=torch.bfloat16, device=cuda)
    out = full[:M, :N]
    K.gemm(A, Bo, K.epilogue(out, N + 8, bias=bias), M, N, Kd, L.BF16)
    torch.cuda.synchronize()
    assert torch.isnan(full[M:].float()).all() and torch.isnan(full[:, N:].float()).all()
    assert rel(out.float(), ref) < 1e-2


@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_mgemm_ragged_n_not_multiple_of_8(cuda, odt):
    """N % 8 == 4 with a bf16 output -- the 256x256 kernel stores 8 bf16 per lane guarded by
    n < N only, so such shapes must leave it (bf16) while an f32 output (4 per lane) may stay; nothing is
    written past N in either case, and the rows after each output row keep their values."""
    M, N, Kd = 4096, 260, 768
    a, b, A, Bo, g = _big_operands(cuda, L.KC, L.KC, M, N, Kd, 23)
    path = L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1)
    ref = a.float() @ b.float().t()
    full = torch.full((M + 1, N + 12), float("nan"), dtype=odt, device=cuda)
    out = full[:M, :N]
    K.gemm(A, Bo, K.epilogue(out, N + 12), M, N, Kd, L.BF16)
    torch.cuda.synchronize()
    assert torch.isnan(full[M:].float()).all() and torch.isnan(full[:, N:].float()).all(), path
    assert rel(out.float(), ref) < (1e-5 if odt == torch.float32 else 1e-2)
    # contiguous output (ldc = N): the 4 columns past a row's end are the next row's first 4
    out2 = torch.empty(M, N, dtype=odt, device=cuda)
    K.gemm(A, Bo, K.epilogue(out2, N), M, N, Kd, L.BF16)
    torch.cuda.synchronize()
    assert rel(out2.float(), ref) < (1e-5 if odt == torch.float32 else 1e-2)


@pytest.mark.parametrize("case", ["plain_f32", "residual_f32", "bias_bf16", "gelu", "gelu_save", "dact_gelu",
                                  "gelu_save_d", "dact_mul"])
def test_mgemm_epilogues(cuda, case):
    """The fused epilogues of the AST linears on the 256x256 kernel: f32 output, residual add into f32
    with bias (proj / fc2 forward), bias only (qkv forward), exact-erf GELU, GELU_SAVE with bias (fc1
    forward: gelu(u) and the saved u) and dGELU with the column sums of the stored values (fc2
    backward-data: times gelu'(u); the sums are fc1's bias gradient) -- vs float64 / fp32 torch."""
    M, N, Kd = 8192 + 37, 768 if case not in ("dact_gelu", "dact_mul") else 3072, 768
    a, b, A, Bo, g = _big_operands(cuda, L.KC, L.KC, M, N, Kd, 11)
    z = a.float() @ b.float().t()
    bias = torch.randn(N, generator=g, device=cuda)
    cs = None
    if case == "plain_f32":
        out = torch.empty(M, N, dtype=torch.float32, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N), M, N, Kd, L.BF16)
        ref = z
    elif case == "residual_f32":
        res = torch.randn(M, N, generator=g, device=cuda)
        out = torch.empty(M, N, dtype=torch.float32, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.ACT_ADD_AUX, bias=bias, aux=res, ldaux=N), M, N, Kd, L.BF16)
        ref = z + bias + res
    elif case == "bias_bf16":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, bias=bias), M, N, Kd, L.BF16)
        ref = z + bias
    elif case == "gelu":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.ACT_GELU, bias=bias), M, N, Kd, L.BF16)
        ref = F.gelu(z + bias)
    elif case == "gelu_save":
        u = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.ACT_GELU_SAVE, bias=bias, aux=u, ldaux=N), M, N, Kd, L.BF16)
        ref = F.gelu(z + bias)
        torch.cuda.synchronize()
        assert rel(u.float(), z + bias) < 1e-2
    elif case == "gelu_save_d":  # fc1 forward keeping gelu'(u) for the backward: gelu' of the bf16 u
        d = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.ACT_GELU_SAVE_D, bias=bias, aux=d, ldaux=N), M, N, Kd, L.BF16)
        ref = F.gelu(z + bias)
        torch.cuda.synchronize()
        assert rel(d.float(), _gelu_grad((z + bias).to(torch.bfloat16))) < 1e-2  # u may round to the next bf16
    elif case == "dact_mul":  # fc2 backward-data times the saved gelu'(u), column sums of the stored values
        d = (torch.rand(M, N, generator=g, device=cuda) * 1.2 - 0.1).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        cs = torch.full((N,), float("nan"), device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.DACT_MUL, aux=d, ldaux=N, colsum=cs), M, N, Kd, L.BF16)
        ref = z.double() * d.double()
    else:
        u = (torch.randn(M, N, generator=g, device=cuda) * 2).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        cs = torch.full((N,), float("nan"), device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.DACT_GELU, aux=u, ldaux=N, colsum=cs), M, N, Kd, L.BF16)
        x = u.double().requires_grad_(True)
        F.gelu(x).backward(torch.ones_like(x))
        ref = z.double() * x.grad
    torch.cuda.synchronize()
    tol = 1e-4 if out.dtype == torch.float32 else 1e-2
    assert rel(out.float(), ref) < tol
    if cs is not None:
        assert rel(cs, out.double().sum(0)) < 1e-5  # the sums of exactly what was stored


@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,Kd", [(768, 2304, 69632 + 100), (2304, 768, 16384), (768, 768, 421120 // 8)])
def test_mgemm_wgrad_split_k(cuda, odt, M, N, Kd):
    """Weight-gradient shapes (both operands k-by-m, K = tokens, few output tiles): the kernel's own
    split-K (a fixed function of the shape) into f32 slabs, summed in slice order -- vs a PyTorch fp32
    matmul of the same bf16 operands; a K tail that is not a multiple of 64 (k-rows past K read as
    zeros), a strided output (ldc > N, nothing written past N), bit-identical from call to call."""
    a, b, A, Bo, g = _big_operands(cuda, L.RC, L.RC, M, N, Kd, 17)
    assert L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1) == 7
    ref = a.float() @ b.float().t()
    full = torch.full((M, N + 64), float("nan"), dtype=odt, device=cuda)
    out = full[:, :N]
    outs = []
    for _ in range(2):
        K.gemm(A, Bo, K.epilogue(out, N + 64), M, N, Kd, L.BF16)
        torch.cuda.synchronize()
        outs.append(out.clone())
    assert torch.isnan(full[:, N:].float()).all()
    assert torch.equal(outs[0], outs[1])
    assert rel(out.float(), ref) < (1e-5 if odt == torch.float32 else 1e-2)


@pytest.mark.parametrize("lb", [L.RC, L.KC])
@pytest.mark.parametrize("M,N,Kd", [(2304, 768, 16384 + 40), (768 + 8, 768, 421120 // 8), (520, 264, 300)])
def test_gemm_a_colsum(cuda, lb, M, N, Kd):
    """MiaEpilogue.a_colsum (the bias gradient of a weight-gradient GEMM dW = dy^T x, A = dy k-by-m):
    summed inside the 256x256 kernel from the A tiles (split-K partials in slice order; M not a multiple
    of the tile, a K tail that is not a multiple of 64) and, on the other paths (a small shape), a
    column-sum pass over A -- vs float64 sums of A, the GEMM output unchanged, bit-identical per call."""
    if lb == L.KC:
        Kd -= Kd % 64  # a k-contiguous B takes whole 64-k tiles
    a, b, A, Bo, g = _big_operands(cuda, L.RC, lb, M, N, Kd, 23)
    big = M >= 768
    assert (L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1) == 7) == big
    out = torch.empty(M, N, dtype=torch.float32, device=cuda)
    ref_out = torch.empty_like(out)
    K.gemm(A, Bo, K.epilogue(ref_out, N), M, N, Kd, L.BF16)
    res = []
    for _ in range(2):
        cs = torch.full((M,), float("nan"), device=cuda)
        K.gemm(A, Bo, K.epilogue(out, N, a_colsum=cs), M, N, Kd, L.BF16)
        torch.cuda.synchronize()
        res.append(cs)
    assert torch.equal(out, ref_out)
    assert torch.equal(res[0], res[1])
    assert rel(res[0], a.double().sum(1)) < 1e-5


@pytest.mark.parametrize("case", ["dact_gelu", "plain"])
def test_mgemm_output_colsum(cuda, case):
    """MiaEpilogue.colsum on both routes: fused into the 256x256 kernel's dGELU epilogue (AST fc1 bias
    behind the fc2 dgrad) and, for an epilogue it does not fuse it into (the 128x128 dense kernel at a
    small token count), a column-sum pass over the output in the caller's workspace -- equal to float64
    sums of what was stored."""
    M, N, Kd = (8192 + 37, 3072, 768) if case == "dact_gelu" else (900, 640, 256)
    a, b, A, Bo, g = _big_operands(cuda, L.KC, L.KC, M, N, Kd, 13)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    cs = torch.full((N,), float("nan"), device=cuda)
    if case == "dact_gelu":
        u = (torch.randn(M, N, generator=g, device=cuda) * 2).to(torch.bfloat16)
        K.gemm(A, Bo, K.epilogue(out, N, act=L.DACT_GELU, aux=u, ldaux=N, colsum=cs), M, N, Kd, L.BF16)
    else:
        assert L.load().mia_gemm_path(A, Bo, M, N, Kd, L.BF16, 1) == 5
        K.gemm(A, Bo, K.epilogue(out, N, colsum=cs), M, N, Kd, L.BF16)
    torch.cuda.synchronize()
    assert rel(cs, out.double().sum(0)) < 1e-5


def test_wgrad8_many_items(cuda):
    """Rolling-window 8x8 wgrad (trunk conv4) with more (clip, chunk) items than blocks, ragged
    column chunks: vs a PyTorch fp32 autograd weight gradient of the same bf16 operands."""
    n, c, h, w = 70, 32, 20, 400
    g = torch.Generator(device=cuda).manual_seed(11)
    x = torch.randn(n, h, w, c, generator=g, device=cuda).to(torch.bfloat16)
    sc = torch.rand(c, generator=g, device=cuda) + 0.5
    sh = torch.randn(c, generator=g, device=cuda) * 0.1
    oh, ow = h - 7, w - 7
    dy = torch.randn(n, oh, ow, c, generator=g, device=cuda).to(torch.bfloat16)
    xin = torch.relu(x.float() * sc + sh).to(torch.bfloat16).float()
    wr = torch.zeros(c, c, 8, 8, device=cuda, requires_grad=True)
    F.conv2d(xin.permute(0, 3, 1, 2), wr).backward(dy.float().permute(0, 3, 1, 2))
    P, Kc = n * oh * ow, 64 * c
    A = K.dense(dy, L.RC, P, c)
    Bo = K.conv(x, L.RC, n, h, w, c, oh, ow, 8, 8, pre=L.PRE_AFFINE_RELU, scale=sc, shift=sh)
    dW = torch.empty(c, Kc, dtype=torch.float32, device=cuda)
    K.gemm(A, Bo, K.epilogue(dW, Kc), c, Kc, P, L.BF16)
    gw = torch.empty(c, c, 8, 8, device=cuda)
    K.unpack_ohwi_grad(dW, (c, c, 8, 8), gw)
    torch.cuda.synchronize()
    assert rel(gw, wr.grad) < 1e-2


@pytest.mark.parametrize("n,w1,pre", [(2, 20001, True), (3, 4112, False), (300, 600, True)])
def test_fe_conv2_fwd(cuda, n, w1, pre):
    """Persistent weight-stationary EnvNet conv2 forward (1x16, stride 2, 32->64, BN1+ReLU applied
    while staging) vs float64 conv1d of the same bf16-rounded operands; ragged last item, more
    items than workgroups (n=300)."""
    w2 = (w1 - 16) // 2 + 1
    g = torch.Generator().manual_seed(w1 + n)
    y1 = torch.randn(n, w1, 32, generator=g).to(torch.bfloat16)
    W = torch.randn(64, 32, 1, 16, generator=g) * 0.05
    bias = torch.randn(64, generator=g)
    sc = torch.rand(32, generator=g) + 0.5
    sh = torch.randn(32, generator=g) * 0.3
    wp = K.pack_weight(W.to(cuda), L.BF16, 0)
    out = torch.full((n * w2, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
    K.fe_conv2_fwd(y1.to(cuda).reshape(-1, 32), sc.to(cuda) if pre else None, sh.to(cuda) if pre else None,
                   wp, bias.to(cuda), out, n, w1, w2)
    torch.cuda.synchronize()
    a = y1.float()
    if pre:
        a = torch.relu(a * sc + sh).to(torch.bfloat16).float()
    ref = F.conv1d(a.double().permute(0, 2, 1), W.to(torch.bfloat16).double()[:, :, 0], bias.double(), stride=2)
    got = out.float().cpu().view(n, w2, 64).permute(0, 2, 1).double()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max() / ref.abs().max() < 1e-2
    assert rel(got, ref) < 5e-3


@pytest.mark.parametrize("n,w1", [(1, 300), (2, 20001), (300, 600)])
def test_fe_conv2_fwd_forms_bit_identical(cuda, monkeypatch, n, w1):
    """The warp-specialised conv2 forward (default) and the two-workgroup form (MIA_FECONV_WS=0) run the same
    MFMA sequence per output: bit-identical outputs, including a ragged last item and more items than CUs."""
    w2 = (w1 - 16) // 2 + 1
    g = torch.Generator().manual_seed(w1 + 7 * n)
    y1 = torch.randn(n * w1, 32, generator=g).to(torch.bfloat16).to(cuda)
    W = torch.randn(64, 32, 1, 16, generator=g) * 0.05
    bias = torch.randn(64, generator=g).to(cuda)
    sc = (torch.rand(32, generator=g) + 0.5).to(cuda)
    sh = (torch.randn(32, generator=g) * 0.3).to(cuda)
    wp = K.pack_weight(W.to(cuda), L.BF16, 0)
    outs = []
    for form in ("1", "0"):
        monkeypatch.setenv("MIA_FECONV_WS", form)
        out = torch.full((n * w2, 64), float("nan"), dtype=torch.bfloat16, device=cuda)
        K.fe_conv2_fwd(y1, sc, sh, wp, bias, out, n, w1, w2)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("n,w1", [(2, 20001), (3, 4112), (300, 601)])
def test_fe_conv2_dgrad(cuda, n, w1):
    """Backward-data of the same conv (both output parities from one staged dY window) vs float64
    conv_transpose1d; odd and even input widths (the last odd pixel has no parity-1 partner)."""
    w2 = (w1 - 16) // 2 + 1
    g = torch.Generator().manual_seed(w1 * 3 + n)
    dy = torch.randn(n, w2, 64, generator=g).to(torch.bfloat16)
    W = torch.randn(64, 32, 1, 16, generator=g) * 0.05
    wpar = K.pack_weight(W.to(cuda), L.BF16, 2)
    out = torch.full((n * w1, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    K.fe_conv2_dgrad(dy.to(cuda).reshape(-1, 64), wpar, out, n, w1, w2)
    torch.cuda.synchronize()
    ref = F.conv_transpose1d(dy.double().permute(0, 2, 1), W.to(torch.bfloat16).double()[:, :, 0], stride=2)
    ref = F.pad(ref, (0, w1 - ref.shape[-1]))  # pixels no output window reaches get zero gradient
    got = out.float().cpu().view(n, w1, 32).permute(0, 2, 1).double()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max() / ref.abs().max() < 1e-2
    assert rel(got, ref) < 5e-3


@pytest.mark.parametrize("n,w1,pre", [(2, 20001, True), (3, 4112, False), (300, 601, True)])
def test_fe_conv2_wgrad(cuda, n, w1, pre):
    """Gradient-stationary EnvNet conv2 weight gradient (BN1+ReLU applied while staging the input
    window) vs a float64 restatement on the same bf16-rounded operands; ragged last item, more
    items than workgroups (n=300)."""
    w2 = (w1 - 16) // 2 + 1
    g = torch.Generator().manual_seed(w1 * 7 + n)
    y1 = torch.randn(n, w1, 32, generator=g).to(torch.bfloat16)
    dy = (torch.randn(n, w2, 64, generator=g) * 0.1).to(torch.bfloat16)
    sc = torch.rand(32, generator=g) + 0.5
    sh = torch.randn(32, generator=g) * 0.3
    dw = torch.full((64, 512), float("nan"), device=cuda)
    K.fe_conv2_wgrad(dy.to(cuda).reshape(-1, 64), y1.to(cuda).reshape(-1, 32), sc.to(cuda) if pre else None,
                     sh.to(cuda) if pre else None, dw, n, w1, w2)
    torch.cuda.synchronize()
    a = y1.float()
    if pre:
        a = torch.relu(a * sc + sh).to(torch.bfloat16).float()
    cols = a.double().unfold(1, 16, 2)  # (n, w2, 32, 16): [b][o][ci][kx]
    ref = torch.einsum("boc,boik->cki", dy.double(), cols)  # [co][kx][ci]
    got = dw.double().cpu().view(64, 16, 32)
    assert torch.isfinite(got).all()
    assert rel(got, ref) < 1e-3


@pytest.mark.parametrize("B,H,W,cin,cout", [(3, 4, 37, 64, 128), (2, 10, 67, 256, 256), (8, 10, 138, 128, 256)])
def test_trunk_w2_dense(cuda, B, H, W, cin, cout):
    """(1, 2) conv (EnvNet trunk blocks 3-4) as dense GEMMs: forward over every input pixel with
    overlapping im2col rows whose epilogue drops each row's last column (drop-mode row map; the last case
    runs on the 256x256 kernel, the others on the 128x128 one with ragged edge tiles), and the backward in
    both forms -- dY laid on the input grid + overlapping views (mia_pad_w2, the default) and the
    interleaved shifted copy -- vs float64 restatements on the same bf16 operands; BN+ReLU
    materialisation."""
    g = torch.Generator().manual_seed(W + cin)
    x = torch.randn(B * H * W, cin, generator=g).to(torch.bfloat16)
    dy = (torch.randn(B * H * (W - 1), cout, generator=g) * 0.1).to(torch.bfloat16)
    Wt = torch.randn(cout, cin, 1, 2, generator=g) * 0.05
    bias = torch.randn(cout, generator=g)
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.3
    st = K.BNState(torch.zeros(cin, device=cuda), torch.ones(cin, device=cuda), sc.to(cuda), sh.to(cuda))
    a = torch.empty(B * H * W + 1, cin, dtype=torch.bfloat16, device=cuda)[: B * H * W]
    K.bn_relu_apply(x.to(cuda), B * H * W, cin, st, a)
    wpk = K.pack_weight(Wt.to(cuda), L.BF16, 0)
    y = torch.full((B * H * (W - 1), cout), float("nan"), dtype=torch.bfloat16, device=cuda)
    K.conv_w2_fwd(a, B * H, W, cin, wpk, bias.to(cuda), y)
    dw = torch.full((cout, 2 * cin), float("nan"), device=cuda)
    dx = torch.full((B * H * W, cin), float("nan"), dtype=torch.bfloat16, device=cuda)
    K.trunk_bwd_w2(dy.to(cuda), a, B * H, W, cout, cin, wpk, dw, dx)  # shifted-copy form (no wflip)
    dw2 = torch.full((cout, 2 * cin), float("nan"), device=cuda)
    dx2 = torch.full((B * H * W, cin), float("nan"), dtype=torch.bfloat16, device=cuda)
    apad = a.as_strided((cin,), (1,), a.storage_offset() + B * H * W * cin)
    apad.fill_(float("nan"))  # the input-grid form must zero the pad pixel it multiplies by a zero gradient
    K.trunk_bwd_w2(dy.to(cuda), a, B * H, W, cout, cin, wpk, dw2, dx2, wflip=K.pack_weight(Wt.to(cuda), L.BF16, 1))
    torch.cuda.synchronize()
    ar = torch.relu(x.float() * sc + sh).to(torch.bfloat16)
    # fused multiply-add in the kernel vs mul+add here: at most one bf16 rounding step apart
    assert torch.allclose(a.cpu().float(), ar.float(), rtol=8e-3, atol=1e-6)
    a4 = a.cpu().double().view(B * H, W, cin)
    d4 = dy.double().view(B * H, W - 1, cout)
    wb = Wt.to(torch.bfloat16).double()[:, :, 0, :]  # (co, ci, kx)
    yref = sum(torch.einsum("rxi,oi->rxo", a4[:, kx:kx + W - 1], wb[:, :, kx]) for kx in range(2)) + bias.double()
    assert rel(y.double().cpu().view(B * H, W - 1, cout), yref) < 1e-2
    ref = torch.stack([torch.einsum("rxo,rxi->oi", d4, a4[:, kx:kx + W - 1]) for kx in range(2)], 1)  # (co, kx, ci)
    dxref = torch.zeros(B * H, W, cin, dtype=torch.float64)
    for kx in range(2):
        dxref[:, kx:kx + W - 1] += torch.einsum("rxo,oi->rxi", d4, wb[:, :, kx])
    for dwx, dxx in ((dw, dx), (dw2, dx2)):
        got = dwx.double().cpu().view(cout, 2, cin)
        assert torch.isfinite(got).all()
        assert rel(got, ref) < 1e-3
        assert rel(dxx.double().cpu().view(B * H, W, cin), dxref) < 1e-2


def _tile_sqsums(out, M, N):
    nbm, nbn = -(-M // 128), -(-N // 128)
    ref = torch.zeros(nbm * nbn, dtype=torch.float64)
    o = out.double().cpu()
    for bm in range(nbm):
        for bn in range(nbn):
            ref[bm * nbn + bn] = o[bm * 128:(bm + 1) * 128, bn * 128:(bn + 1) * 128].square().sum()
    return ref


@pytest.mark.parametrize("cd,M,N,Kd,split,la", [
    (L.BF16, 384, 512, 256, 1, L.RC),   # dense kernel, full tiles (staged-tile epilogue)
    (L.BF16, 200, 328, 128, 1, L.RC),   # dense kernel, ragged edge tiles (generic epilogue)
    (L.BF16, 256, 384, 1024, 4, L.RC),  # split-K: per-tile pass after the reduce
    (L.BF16, 256, 256, 192, 1, L.KC),   # another layout on the dense kernel
    (L.F32, 150, 260, 40, 1, L.KC),     # tile kernel: per-tile pass
])
def test_sqsum_epilogue(cuda, cd, M, N, Kd, split, la):
    """MiaEpilogue.sqsum (EnvNet FC wgrad -> clip norm): per-128x128-tile sums of squares of exactly
    the values stored, on every path (fused in the dense kernel, a separate pass elsewhere)."""
    g = torch.Generator().manual_seed(M + N + split)
    dt = torch.float32 if cd == L.F32 else torch.bfloat16
    a, A, ta = _mat(la, M, Kd, dt, cuda, g)
    b, Bo, tb = _mat(L.RC, N, Kd, dt, cuda, g)
    out = torch.empty(M, N, dtype=torch.float32, device=cuda)
    sq = K.sqsum_slots(out, M, N)
    sq.fill_(float("nan"))
    K.gemm(A, Bo, K.epilogue(out, N, sqsum=sq), M, N, Kd, cd, split_k=split)
    torch.cuda.synchronize()
    assert rel(out.cpu(), a.double() @ b.double().t()) < TOL[cd]
    ref = _tile_sqsums(out, M, N)
    assert torch.isfinite(sq).all()
    assert torch.allclose(sq.cpu(), ref, rtol=1e-5, atol=0)


def test_sqsum_needs_plain_f32(cuda):
    out = torch.empty(128, 128, dtype=torch.bfloat16, device=cuda)
    sq = torch.empty(1, dtype=torch.float64, device=cuda)
    x = torch.randn(128, 64, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        K.gemm(K.dense(x, L.KC, 128, 64), K.dense(x, L.KC, 128, 64), K.epilogue(out, 128, sqsum=sq), 128, 128, 64,
               L.BF16)
