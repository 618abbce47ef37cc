"""GPU: BatchNorm statistics / backward and the fused BN+ReLU+max-pool kernels against float64
torch autograd on the same inputs (so the ReLU masks agree exactly)."""
import pytest
import torch
import torch.nn.functional as F

from src.miaudio import kernels as K
from src.miaudio import lib as L

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("C", [32, 64, 256])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_stats_and_backward(cuda, C, dt):
    g = torch.Generator().manual_seed(C)
    P = 5000
    y = (torch.randn(P, C, generator=g) * 3 + 2).to(dt)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.2
    rm, rv = torch.zeros(C), torch.ones(C)
    ty = y.to(cuda)
    trm, trv = rm.to(cuda), rv.to(cuda)
    st = K.bn_fwd_stats(ty, P, C, gamma.to(cuda), beta.to(cuda), trm, trv, 0.1, 1e-5, True)
    yd = y.double()
    mu, var = yd.mean(0), yd.var(0, unbiased=False)
    assert rel(st.mean, mu) < 1e-5
    assert rel(1.0 / st.invstd.double() ** 2 - 1e-5, var) < 1e-4
    assert rel(trv, 0.9 + 0.1 * yd.var(0, unbiased=True)) < 1e-4
    # backward of relu(bn(y)) given dact
    dact = torch.randn(P, C, generator=g).to(dt)
    yr = yd.clone().requires_grad_(True)
    gr = gamma.double().requires_grad_(True)
    br = beta.double().requires_grad_(True)
    z = F.batch_norm(yr, None, None, gr, br, True, 0.0, 1e-5)
    torch.relu(z).backward(dact.double())
    tact = dact.to(cuda)
    dz = torch.empty_like(tact)
    dg, db = K.bn_relu_bwd_reduce(tact, dz, ty, P, C, st)
    dx = torch.empty_like(tact)
    dbias = torch.empty(C, device=cuda)
    K.bn_bwd_apply(dz, ty, dx, P, C, gamma.to(cuda), st, dg, db, dbias)
    torch.cuda.synchronize()
    tol = 2e-5 if dt == torch.float32 else 2e-2
    assert rel(dg, gr.grad) < tol * 5 and rel(db, br.grad) < tol * 5
    assert rel(dx.float(), yr.grad) < tol * 10
    assert float(dbias.abs().max()) < 1e-2 * float(yr.grad.abs().sum(0).max())


@pytest.mark.parametrize("geom", [(2, 1, 640, 64, 1, 64, 1), (2, 50, 846, 32, 5, 3, 0), (3, 10, 66, 256, 1, 2, 2)])
def test_pool_fwd_bwd(cuda, geom):
    n, h, w, c, kh, kw, layout = geom
    g = torch.Generator().manual_seed(h * w)
    y = torch.randn(n, h, w, c, generator=g)
    scale = torch.rand(c, generator=g) + 0.5
    shift = torch.randn(c, generator=g) * 0.3
    st = K.BNState(torch.zeros(c, device=cuda), torch.ones(c, device=cuda), scale.to(cuda), shift.to(cuda))
    oh, ow = h // kh, w // kw
    out = torch.empty({0: (n, oh, ow, c), 1: (n, c, ow), 2: (n, c, oh, ow)}[layout], device=cuda)
    am = torch.empty(n, oh, ow, c, dtype=torch.uint8, device=cuda)
    ty = y.to(cuda)
    K.pool_fwd(ty, n, h, w, c, kh, kw, st, out, layout, am)
    a = torch.relu(y.double() * scale.double() + shift.double()).permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(a, (kh, kw), (kh, kw))
    ref_l = {0: ref.permute(0, 2, 3, 1), 1: ref[:, :, 0, :], 2: ref}[layout]
    torch.cuda.synchronize()
    assert rel(out, ref_l) < 1e-6
    dout = torch.randn(ref_l.shape, generator=g)
    ref_l.backward(dout.double())
    # kernel gives dz (grad of the BN output z, relu-masked); torch gives grad of a = relu(z)
    dz = torch.empty_like(ty)
    dg, db = K.pool_bwd_bn_relu_reduce(dout.to(cuda), layout, am, ty, n, h, w, c, kh, kw, st, dz)
    torch.cuda.synchronize()
    zmask = (y.double() * scale.double() + shift.double() > 0).permute(0, 3, 1, 2)
    gz = (a.grad * zmask).permute(0, 2, 3, 1)
    assert rel(dz, gz) < 1e-6
    assert rel(db, gz.sum(dim=(0, 1, 2))) < 1e-5
    # sparse reductions (dz=None) agree with the dense pass; the fused apply equals the two-pass one
    gm, dg2, db2 = K.pool_bwd_gather(dout.to(cuda), layout, am, ty, n, h, w, c, kh, kw, st)
    gamma = (torch.rand(c, generator=g) + 0.5).to(cuda)
    dx_ref = torch.empty_like(ty)
    K.bn_bwd_apply(dz, ty, dx_ref, n * h * w, c, gamma, st, dg, db)
    dx = torch.empty_like(ty)
    dbias = torch.empty(c, device=cuda)
    K.pool_bn_relu_bwd_apply(gm, am, ty, n, h, w, c, kh, kw, gamma, st, dg2, db2, dx, dbias)
    torch.cuda.synchronize()
    assert rel(dg2, dg) < 1e-5 and rel(db2, db) < 1e-5
    assert rel(dx, dx_ref) < 1e-5
    assert rel(dbias, dx_ref.double().sum(dim=(0, 1, 2))) < 1e-4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_relu_bwd_masked_apply(cuda, dt):
    """bn_relu_bwd_apply (mask recomputed from x) == reduce-with-dz + bn_bwd_apply."""
    g = torch.Generator().manual_seed(3)
    P, C = 5000, 64
    y = torch.randn(P, C, generator=g).to(dt).to(cuda)
    dact = torch.randn(P, C, generator=g).to(dt).to(cuda)
    st = K.BNState(torch.randn(C, generator=g).to(cuda) * 0.1, (torch.rand(C, generator=g) + 0.5).to(cuda),
                   (torch.rand(C, generator=g) + 0.5).to(cuda), (torch.randn(C, generator=g) * 0.3).to(cuda))
    gamma = (torch.rand(C, generator=g) + 0.5).to(cuda)
    dz = torch.empty_like(dact)
    dg, db = K.bn_relu_bwd_reduce(dact, dz, y, P, C, st)
    dg2, db2 = K.bn_relu_bwd_reduce(dact, None, y, P, C, st)
    dx_ref = torch.empty_like(dact)
    K.bn_bwd_apply(dz, y, dx_ref, P, C, gamma, st, dg, db)
    dx = torch.empty_like(dact)
    dbias = torch.empty(C, device=cuda)
    K.bn_relu_bwd_apply(dact, y, dx, P, C, gamma, st, dg2, db2, dbias)
    torch.cuda.synchronize()
    assert torch.equal(dg, dg2) and torch.equal(db, db2)
    assert torch.equal(dx, dx_ref)
    # dbias sums the f32 values before the store rounds them (bf16: compare against the rounded sum loosely)
    assert rel(dbias, dx_ref.double().sum(0)) < (1e-4 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("n,t", [(3, 220500), (2, 9000)])
def test_fe_conv1_wgrad_bn_fused(cuda, n, t):
    """One-pass BN1+ReLU backward + conv1 weight/bias gradient (linear form) vs the two-pass path
    (bn_relu_bwd_reduce -> bn_relu_bwd_apply -> bf16 dS1 -> tap wgrad GEMM) and a float64
    restatement."""
    w1 = (t - 64) // 2 + 1
    P = n * w1
    g = torch.Generator(device=cuda).manual_seed(t + n)
    x = torch.randn(n, t, generator=g, device=cuda) * 0.1
    y1 = (torch.randn(P, 32, generator=g, device=cuda) * 0.7 + 0.2).to(torch.bfloat16)
    da = (torch.randn(P, 32, generator=g, device=cuda) * 1e-3).to(torch.bfloat16)
    gamma = torch.rand(32, generator=g, device=cuda) + 0.5
    beta = torch.randn(32, generator=g, device=cuda) * 0.1
    bn = K.bn_fwd_stats(y1, P, 32, gamma, beta, None, None, 0.1, 1e-5, True)
    dg, db = K.bn_relu_bwd_reduce(da, None, y1, P, 32, bn)
    dw = torch.empty(32, 64, device=cuda)
    dbias = torch.empty(32, device=cuda)
    dg1, db1 = K.fe_conv1_wgrad_bn(x, da, y1, n, t, gamma, bn, dw, dbias)
    # unfused reference path
    dx = torch.empty_like(da)
    dbias_u = torch.empty(32, device=cuda)
    K.bn_relu_bwd_apply(da, y1, dx, P, 32, gamma, bn, dg, db, dbias_u)
    dw_u = torch.empty(32, 64, device=cuda)
    K.gemm(K.dense(dx, L.RC, P, 32), K.conv(x, L.RC, n, 1, t // 2, 2, 1, w1, 1, 32, row_kind=True),
           K.epilogue(dw_u, 64), 32, 64, P, L.BF16)
    torch.cuda.synchronize()
    # one-pass linear form: same BN reductions as the reduce kernel (summation order aside); dW
    # differs from the two-pass path only by the bf16 rounding of dS1 that the linear form avoids
    assert rel(dg1, dg) < 1e-5 and rel(db1, db) < 1e-5
    assert rel(dw, dw_u) < 1e-2
    scale_b = dx.float().abs().sum(0).max()
    assert (dbias - dbias_u).abs().max() < 1e-3 * scale_b
    # float64 restatement
    y = y1.double()
    z = y * bn.scale.double() + bn.shift.double()
    dz = torch.where(z > 0, da.double(), torch.zeros_like(z))
    xhat = (y - bn.mean.double()) * bn.invstd.double()
    mdz, mdzx = dz.mean(0), (dz * xhat).mean(0)
    d64 = gamma.double() * bn.invstd.double() * (dz - mdz - xhat * mdzx)
    cols = x.double().unfold(1, 64, 2)  # (n, w1, 64)
    ref = torch.einsum("npc,npk->ck", d64.view(n, w1, 32), cols)
    assert rel(dw.double(), ref) < 1e-2
    assert rel(dg1.double(), (dz * xhat).sum(0)) < 1e-4 and rel(db1.double(), dz.sum(0)) < 1e-4


@pytest.mark.parametrize("n,t", [(3, 220500), (5, 9000)])
def test_fe_conv1_fwd_with_bn_stats(cuda, n, t):
    """Wave-persistent conv1 (1x64, stride 2) vs float64 conv1d of the same bf16 operands, and the BN1
    statistics it accumulates (shifted about the bias) == mia_bn_fwd_stats over its own output,
    running statistics included."""
    w1 = (t - 64) // 2 + 1
    g = torch.Generator(device=cuda).manual_seed(t * 3 + n)
    x = torch.randn(n, t, generator=g, device=cuda) * 0.1
    W = torch.randn(32, 1, 1, 64, generator=g, device=cuda) * 0.1
    bias = torch.randn(32, generator=g, device=cuda) * 0.5
    wp = K.pack_weight(W, L.BF16, 0)
    y1 = torch.empty(n * w1, 32, dtype=torch.bfloat16, device=cuda)
    part, nblk = K.fe_conv1_fwd(x, wp, bias, y1, n, t, stats=True)
    gamma = torch.rand(32, generator=g, device=cuda) + 0.5
    beta = torch.randn(32, generator=g, device=cuda)
    rm1, rv1 = torch.zeros(32, device=cuda), torch.ones(32, device=cuda)
    rm2, rv2 = rm1.clone(), rv1.clone()
    st = K.bn_finalize_shifted(part, nblk, n * w1, 32, bias, gamma, beta, rm1, rv1, 0.1, 1e-5)
    ref_st = K.bn_fwd_stats(y1, n * w1, 32, gamma, beta, rm2, rv2, 0.1, 1e-5, True)
    torch.cuda.synchronize()
    ref = F.conv1d(x.to(torch.bfloat16).double()[:, None], W.to(torch.bfloat16).double()[:, :, 0], bias.double(),
                   stride=2)
    got = y1.double().view(n, w1, 32).permute(0, 2, 1)
    assert (got - ref).abs().max() / ref.abs().max() < 1e-2
    for a, b in ((st.mean, ref_st.mean), (st.invstd, ref_st.invstd), (st.scale, ref_st.scale),
                 (st.shift, ref_st.shift), (rm1, rm2), (rv1, rv2)):
        assert torch.allclose(a, b, rtol=2e-5, atol=2e-6), (a - b).abs().max()


@pytest.mark.parametrize("geom", [(2, 1, 640, 64, 1, 64), (3, 1, 1001, 64, 1, 64), (2, 6, 67, 32, 2, 8),
                                  (2, 50, 846, 32, 5, 3), (3, 11, 68, 32, 5, 3), (2, 10, 67, 64, 1, 2),
                                  (2, 5, 33, 256, 2, 4)])
def test_pool_bn_bwd_apply_octets_bf16(cuda, geom):
    """bf16 pooled BN backward with kw % 8 == 0 (row-octet kernel: one cell lookup per 8 pixels) and
    kw = 2..4 (run kernel: one cell lookup per kw-pixel run of a row; the trunk's (5, 3) and (1, 2)
    pools), with ragged rows and columns (pixels past the last whole cell) vs a float64 restatement:
    dx = BN backward of the max-pool's routed, ReLU-masked gradient."""
    n, h, w, c, kh, kw = geom
    g = torch.Generator().manual_seed(h * w + c)
    y = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16)
    scale = torch.rand(c, generator=g) + 0.5
    shift = torch.randn(c, generator=g) * 0.3
    mean = torch.randn(c, generator=g) * 0.1
    invstd = torch.rand(c, generator=g) + 0.5
    st = K.BNState(mean.to(cuda), invstd.to(cuda), scale.to(cuda), shift.to(cuda))
    oh, ow = h // kh, w // kw
    out = torch.empty(n, oh, ow, c, device=cuda, dtype=torch.bfloat16)
    am = torch.empty(n, oh, ow, c, dtype=torch.uint8, device=cuda)
    ty = y.to(cuda)
    K.pool_fwd(ty, n, h, w, c, kh, kw, st, out, 0, am)
    dout = torch.randn(n, oh, ow, c, generator=g).to(torch.bfloat16)  # same dtype as the activations
    gm, dg, db = K.pool_bwd_gather(dout.to(cuda), 0, am, ty, n, h, w, c, kh, kw, st)
    gamma = (torch.rand(c, generator=g) + 0.5)
    dx = torch.empty_like(ty)
    dbias = torch.empty(c, device=cuda)
    K.pool_bn_relu_bwd_apply(gm, am, ty, n, h, w, c, kh, kw, gamma.to(cuda), st, dg, db, dx, dbias)
    torch.cuda.synchronize()
    # float64 restatement: route dout to the argmax of relu(z) per cell, mask, BN backward
    yd = y.double()
    a = torch.relu(yd * scale.double() + shift.double()).permute(0, 3, 1, 2).requires_grad_(True)
    F.max_pool2d(a, (kh, kw), (kh, kw)).backward(dout.double().permute(0, 3, 1, 2))
    zmask = (yd * scale.double() + shift.double() > 0)
    dz = a.grad.permute(0, 2, 3, 1) * zmask
    P = n * h * w
    xhat = (yd - mean.double()) * invstd.double()
    ref = gamma.double() * invstd.double() * (dz - dz.sum((0, 1, 2)) / P - xhat * (dz * xhat).sum((0, 1, 2)) / P)
    assert rel(dx.double().cpu(), ref) < 1e-2
    assert rel(dg.double().cpu(), (dz * xhat).sum((0, 1, 2))) < 1e-4
    assert rel(db.double().cpu(), dz.sum((0, 1, 2))) < 1e-4


@pytest.mark.parametrize("n,h,wd", [(3, 64, 860), (5, 12, 100)])
def test_fe_conv3_fwd_with_bn_stats(cuda, n, h, wd):
    """Wave-persistent trunk conv3 (1 -> 32, 8x8) vs float64 conv2d of the same bf16 operands, and
    its fused BN statistics == mia_bn_fwd_stats over its own output (running statistics included)."""
    g = torch.Generator(device=cuda).manual_seed(h * wd + n)
    x = (torch.randn(n, h, wd, generator=g, device=cuda) * 0.5).to(torch.bfloat16)
    W = torch.randn(32, 1, 8, 8, generator=g, device=cuda) * 0.1
    bias = torch.randn(32, generator=g, device=cuda) * 0.5
    wp = K.pack_weight(W, L.BF16, 0)
    oh, ow = h - 7, wd - 7
    y = torch.full((n * oh * ow, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    part, nblk = K.fe_conv3_fwd(x, wp, bias, y, n, h, wd, stats=True)
    gamma = torch.rand(32, generator=g, device=cuda) + 0.5
    beta = torch.randn(32, generator=g, device=cuda)
    rm1, rv1 = torch.zeros(32, device=cuda), torch.ones(32, device=cuda)
    rm2, rv2 = rm1.clone(), rv1.clone()
    st = K.bn_finalize_shifted(part, nblk, n * oh * ow, 32, bias, gamma, beta, rm1, rv1, 0.1, 1e-5)
    ref_st = K.bn_fwd_stats(y, n * oh * ow, 32, gamma, beta, rm2, rv2, 0.1, 1e-5, True)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double()[:, None], W.to(torch.bfloat16).double(), bias.double())
    got = y.double().view(n, oh, ow, 32).permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max() / ref.abs().max() < 1e-2
    for a, b in ((st.mean, ref_st.mean), (st.invstd, ref_st.invstd), (st.scale, ref_st.scale),
                 (st.shift, ref_st.shift), (rm1, rm2), (rv1, rv2)):
        assert torch.allclose(a, b, rtol=2e-5, atol=2e-6), (a - b).abs().max()


@pytest.mark.parametrize("n,h,wd", [(2, 57, 853), (3, 10, 40), (2, 9, 12)])
def test_trunk_conv8_fwd_with_bn_stats(cuda, n, h, wd):
    """Row-rolling conv4 kernel (32 -> 32, 8x8, BN+ReLU applied on staging) vs float64 conv2d of the
    same bf16 operands, and its fused BN statistics == mia_bn_fwd_stats over its own output."""
    g = torch.Generator(device=cuda).manual_seed(h * wd + n)
    x = (torch.randn(n, h, wd, 32, generator=g, device=cuda) * 0.7 + 0.1).to(torch.bfloat16)
    scale = torch.rand(32, generator=g, device=cuda) + 0.5
    shift = torch.randn(32, generator=g, device=cuda) * 0.3
    W = torch.randn(32, 32, 8, 8, generator=g, device=cuda) * 0.03
    bias = torch.randn(32, generator=g, device=cuda) * 0.5
    wp = K.pack_weight(W, L.BF16, 0)
    oh, ow = h - 7, wd - 7
    y = torch.full((n * oh * ow, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    part, nblk = K.trunk_conv8(x, wp, y, n, h, wd, scale=scale, shift=shift, bias=bias, stats=True)
    gamma = torch.rand(32, generator=g, device=cuda) + 0.5
    beta = torch.randn(32, generator=g, device=cuda)
    rm1, rv1 = torch.zeros(32, device=cuda), torch.ones(32, device=cuda)
    rm2, rv2 = rm1.clone(), rv1.clone()
    st = K.bn_finalize_shifted(part, nblk, n * oh * ow, 32, bias, gamma, beta, rm1, rv1, 0.1, 1e-5)
    ref_st = K.bn_fwd_stats(y, n * oh * ow, 32, gamma, beta, rm2, rv2, 0.1, 1e-5, True)
    torch.cuda.synchronize()
    a = torch.relu(x.float() * scale + shift).to(torch.bfloat16).double().permute(0, 3, 1, 2)
    ref = F.conv2d(a, W.to(torch.bfloat16).double(), bias.double())
    got = y.double().view(n, oh, ow, 32).permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    assert rel(got, ref) < 1e-2
    for u, v in ((st.mean, ref_st.mean), (st.invstd, ref_st.invstd), (st.scale, ref_st.scale),
                 (st.shift, ref_st.shift), (rm1, rm2), (rv1, rv2)):
        assert torch.allclose(u, v, rtol=2e-5, atol=2e-6), (u - v).abs().max()


@pytest.mark.parametrize("n,h,wd", [(2, 50, 846), (3, 3, 30), (1, 1, 1)])
def test_trunk_conv8_dgrad(cuda, n, h, wd):
    """conv4 backward-data on the row-rolling kernel (dY zero-padded by 7, flipped weights) vs float64
    conv_transpose2d; covers dY maps shorter than the kernel."""
    g = torch.Generator(device=cuda).manual_seed(h + wd + n)
    dy = torch.randn(n, h, wd, 32, generator=g, device=cuda).to(torch.bfloat16)
    W = torch.randn(32, 32, 8, 8, generator=g, device=cuda) * 0.03
    wf = K.pack_weight(W, L.BF16, 1)
    dx = torch.full((n * (h + 7) * (wd + 7), 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    K.trunk_conv8(dy, wf, dx, n, h, wd, ph=7, pw=7)
    torch.cuda.synchronize()
    ref = F.conv_transpose2d(dy.double().permute(0, 3, 1, 2), W.to(torch.bfloat16).double())
    got = dx.double().view(n, h + 7, wd + 7, 32).permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    assert rel(got, ref) < 1e-2


@pytest.mark.parametrize("n,h,wd", [(2, 50, 846), (3, 3, 30), (1, 1, 1), (5, 17, 70)])
def test_trunk_conv8_dgrad_bn_reduce(cuda, n, h, wd):
    """conv4 backward-data with the ReLU+BN backward sums in its epilogue: dx bit-identical to the plain
    backward-data kernel, (dgamma, dbeta) == mia_bn_relu_bwd_reduce over that dx and == float64 sums."""
    g = torch.Generator(device=cuda).manual_seed(3 * h + wd + n)
    dy = torch.randn(n, h, wd, 32, generator=g, device=cuda).to(torch.bfloat16)
    W = torch.randn(32, 32, 8, 8, generator=g, device=cuda) * 0.03
    wf = K.pack_weight(W, L.BF16, 1)
    P = n * (h + 7) * (wd + 7)
    bx = (torch.randn(P, 32, generator=g, device=cuda) * 1.3 + 0.2).to(torch.bfloat16)
    gamma = torch.rand(32, generator=g, device=cuda) + 0.5
    beta = torch.randn(32, generator=g, device=cuda) * 0.5
    bn = K.bn_fwd_stats(bx, P, 32, gamma, beta, None, None, 0.1, 1e-5, True)
    dx0 = torch.full((P, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    dx1 = torch.full((P, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    K.trunk_conv8(dy, wf, dx0, n, h, wd, ph=7, pw=7)
    dg, db = K.trunk_conv8_dgrad_bn(dy, wf, dx1, n, h, wd, bx, bn)
    rg, rb = K.bn_relu_bwd_reduce(dx0, None, bx, P, 32, bn)
    torch.cuda.synchronize()
    assert torch.equal(dx0.view(torch.int16), dx1.view(torch.int16))
    xd = bx.double()
    m = (bx.float() * bn.scale + bn.shift > 0).double()
    gd = dx0.double() * m
    ref_b = gd.sum(0)
    ref_g = (gd * (xd - bn.mean.double()) * bn.invstd.double()).sum(0)
    tol_b = 1e-5 * dx0.double().abs().sum(0) + 1e-6
    tol_g = 1e-5 * (gd * (xd - bn.mean.double()) * bn.invstd.double()).abs().sum(0) + 1e-6
    for got, ref, tol in ((db, ref_b, tol_b), (dg, ref_g, tol_g), (rb, ref_b, tol_b), (rg, ref_g, tol_g)):
        assert ((got.double() - ref).abs() <= tol).all(), (got.double() - ref).abs().max()


@pytest.mark.parametrize("n,h,wd", [(2, 64, 860), (3, 9, 40), (1, 8, 12)])
def test_conv3_wgrad_bn_equals_apply_then_wgrad(cuda, n, h, wd):
    """conv3 weight gradient with the ReLU+BN backward formed while staging dY (in place) == the separate
    bn_relu_bwd_apply pass followed by conv3_wgrad: dY and dW bit-identical, the bias gradient to f32 order."""
    g = torch.Generator(device=cuda).manual_seed(h * 5 + wd + n)
    x = torch.randn(n, h, wd, generator=g, device=cuda).to(torch.bfloat16)
    oh, ow = h - 7, wd - 7
    P = n * oh * ow
    da = torch.randn(P, 32, generator=g, device=cuda).to(torch.bfloat16)
    ya = (torch.randn(P, 32, generator=g, device=cuda) * 1.2 + 0.1).to(torch.bfloat16)
    gamma = torch.rand(32, generator=g, device=cuda) + 0.5
    beta = torch.randn(32, generator=g, device=cuda) * 0.5
    bn = K.bn_fwd_stats(ya, P, 32, gamma, beta, None, None, 0.1, 1e-5, True)
    dg, db = K.bn_relu_bwd_reduce(da, None, ya, P, 32, bn)
    dy0 = torch.empty_like(da)
    db0 = torch.empty(32, device=cuda)
    K.bn_relu_bwd_apply(da, ya, dy0, P, 32, gamma, bn, dg, db, db0)
    dw0 = torch.full((32, 64), float("nan"), device=cuda)
    K.conv3_wgrad(x, dy0, dw0, n, h, wd)
    dy1 = da.clone()
    dw1 = torch.full((32, 64), float("nan"), device=cuda)
    db1 = torch.full((32,), float("nan"), device=cuda)
    K.conv3_wgrad_bn(x, dy1, ya, dy1, dw1, db1, n, h, wd, gamma, bn, dg, db)
    torch.cuda.synchronize()
    assert torch.equal(dy0.view(torch.int16), dy1.view(torch.int16))
    assert torch.equal(dw0, dw1)
    tol = 1e-5 * dy0.float().abs().sum(0) + 1e-6
    assert ((db0 - db1).abs() <= tol).all(), (db0 - db1).abs().max()


@pytest.mark.parametrize("n,h,wd", [(2, 64, 860), (3, 9, 40), (1, 8, 12)])
def test_conv3_wgrad(cuda, n, h, wd):
    """Wave-persistent conv3 (1 -> 32, 8x8) weight gradient vs float64 torch on the same bf16 operands."""
    g = torch.Generator(device=cuda).manual_seed(h * 7 + wd + n)
    x = torch.randn(n, h, wd, generator=g, device=cuda).to(torch.bfloat16)
    oh, ow = h - 7, wd - 7
    dy = torch.randn(n, oh, ow, 32, generator=g, device=cuda).to(torch.bfloat16)
    dw = torch.full((32, 64), float("nan"), device=cuda)
    K.conv3_wgrad(x, dy, dw, n, h, wd)
    torch.cuda.synchronize()
    xd = x.double()[:, None].requires_grad_(True)
    w = torch.zeros(32, 1, 8, 8, dtype=torch.float64, device=cuda, requires_grad=True)
    F.conv2d(xd, w).backward(dy.double().permute(0, 3, 1, 2))
    ref = w.grad.view(32, 64)
    assert torch.isfinite(dw).all()
    assert rel(dw, ref) < 1e-4


@pytest.mark.parametrize("n,h,w,kw,C", [(3, 1, 55102, 64, 64), (2, 1, 300, 64, 64), (2, 1, 70, 7, 64),
                                        (2, 1, 64 * 130, 64, 64), (2, 10, 279, 2, 64), (2, 10, 139, 2, 128),
                                        (3, 1, 1000, 16, 64), (2, 1, 200, 72, 64), (4, 1, 16640 // 8, 64, 64)])
def test_pool_raw_stats_matches_pool_fwd(cuda, n, h, w, kw, C):
    """One-pass maxpool-on-raw-winners + BN statistics (then relu(bn(winner))) == BN statistics pass +
    maxpool of relu(bn(x)); argmax equal wherever the pooled value is positive (elsewhere the routed
    gradient is 0 either way).  Negative and zero gammas exercise the min / first-position winners."""
    g = torch.Generator(device=cuda).manual_seed(n * w + kw)
    x = (torch.randn(n, h, w, C, generator=g, device=cuda) * 2 + 0.3).to(torch.bfloat16)
    gamma = torch.randn(C, generator=g, device=cuda)
    gamma[5] = 0.0
    beta = torch.randn(C, generator=g, device=cuda) * 0.5
    kshift = torch.randn(C, generator=g, device=cuda) * 0.1
    ow = w // kw
    rm1, rv1 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    rm2, rv2 = rm1.clone(), rv1.clone()
    win = torch.empty(n, h, ow, C, dtype=torch.bfloat16, device=cuda)
    am1 = torch.empty(n, h, ow, C, dtype=torch.uint8, device=cuda)
    part, nb = K.pool_raw_stats(x, n, h, w, C, 1, kw, gamma, kshift, win, am1)
    st1 = K.bn_finalize_shifted(part, nb, n * h * w, C, kshift, gamma, beta, rm1, rv1, 0.1, 1e-5)
    out1 = torch.empty(n, h, ow, C, dtype=torch.bfloat16, device=cuda)
    K.pool_apply(win, n, h, ow, C, st1, out1, 0)
    if h == 1 and C == 64:  # the transposed trunk image (layout 1, the tiled kernel): the same values, bit for bit
        out1t = torch.full((n, C, ow), float("nan"), dtype=torch.bfloat16, device=cuda)
        K.pool_apply(win, n, h, ow, C, st1, out1t, 1)
        torch.cuda.synchronize()
        assert torch.equal(out1t, out1[:, 0].permute(0, 2, 1))
    st2 = K.bn_fwd_stats(x, n * h * w, C, gamma, beta, rm2, rv2, 0.1, 1e-5, True)
    out2 = torch.empty(n, h, ow, C, dtype=torch.bfloat16, device=cuda)
    am2 = torch.empty(n, h, ow, C, dtype=torch.uint8, device=cuda)
    K.pool_fwd(x, n, h, w, C, 1, kw, st2, out2, 0, am2)
    torch.cuda.synchronize()
    for a, b in ((st1.mean, st2.mean), (st1.invstd, st2.invstd), (rm1, rm2), (rv1, rv2)):
        assert torch.allclose(a, b, rtol=2e-5, atol=2e-6), (a - b).abs().max()
    assert (out1.float() - out2.float()).abs().max() <= 2e-2 * out2.float().abs().max()
    pos = out2 > 0
    assert torch.equal(am1[pos], am2[pos])
    # every window: the first position of the max of sign(gamma) * x, and the raw value there, bit for bit
    xw = x[:, :, :ow * kw].reshape(n, h, ow, kw, C)
    ref_am = (xw.float() * torch.sign(gamma)).argmax(dim=3)
    assert torch.equal(am1.long(), ref_am)
    ref_win = torch.gather(xw, 3, ref_am.unsqueeze(3)).squeeze(3)
    assert torch.equal(win.view(torch.int16), ref_win.view(torch.int16))


@pytest.mark.parametrize("geom", [(2, 1, 640, 64, 1, 64), (3, 1, 1001, 64, 1, 64)])
def test_pool_bwd_gather_raw_winners_bit_identical(cuda, geom):
    """The frontend backward reads the forward's raw winners (pool_raw_stats `win`) instead of
    gathering y2 at the argmax: gm, dgamma, dbeta must be bit-identical to the gathered version."""
    n, h, w, c, kh, kw = geom
    g = torch.Generator().manual_seed(w + 7)
    y = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16).to(cuda)
    gamma = (torch.rand(c, generator=g) - 0.3).to(cuda)  # mixed signs: min- and max-winners
    kshift = (torch.randn(c, generator=g) * 0.1).to(cuda)
    oh, ow = h // kh, w // kw
    win = torch.empty(n, oh, ow, c, dtype=torch.bfloat16, device=cuda)
    am = torch.empty(n, oh, ow, c, dtype=torch.uint8, device=cuda)
    K.pool_raw_stats(y, n, h, w, c, kh, kw, gamma, kshift, win, am)
    st = K.BNState((torch.randn(c, generator=g) * 0.1).to(cuda), (torch.rand(c, generator=g) + 0.5).to(cuda),
                   gamma.clone(), (torch.randn(c, generator=g) * 0.3).to(cuda))
    dout = torch.randn(n, c, oh * ow, generator=g).to(torch.bfloat16).to(cuda)
    ref = K.pool_bwd_gather(dout, 1, am, y, n, h, w, c, kh, kw, st)
    ref = [t.clone() for t in ref]
    got = K.pool_bwd_gather(dout, 1, am, y, n, h, w, c, kh, kw, st, win=win)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("geom", [(2, 10, 33, 32, 5, 3), (3, 2, 41, 64, 1, 2)])
def test_pool_fwd_raw_winners_feed_gather_bit_identical(cuda, geom, dtype):
    """pool_fwd's optional raw-winner output (trunk pools) == x at the argmax, and the gather reading
    it is bit-identical to the gather over x."""
    n, h, w, c, kh, kw = geom
    g = torch.Generator().manual_seed(h * w)
    y = torch.randn(n, h, w, c, generator=g).to(dtype).to(cuda)
    st = K.BNState((torch.randn(c, generator=g) * 0.1).to(cuda), (torch.rand(c, generator=g) + 0.5).to(cuda),
                   (torch.rand(c, generator=g) - 0.3).to(cuda), (torch.randn(c, generator=g) * 0.3).to(cuda))
    oh, ow = h // kh, w // kw
    out = torch.empty(n, oh, ow, c, dtype=dtype, device=cuda)
    am = torch.empty(n, oh, ow, c, dtype=torch.uint8, device=cuda)
    win = torch.empty(n, oh, ow, c, dtype=dtype, device=cuda)
    K.pool_fwd(y, n, h, w, c, kh, kw, st, out, 0, am, win=win)
    a = am.long().cpu()
    iy = torch.arange(oh)[None, :, None, None] * kh + a // kw
    ix = torch.arange(ow)[None, None, :, None] * kw + a % kw
    yc = y.cpu()
    exp = yc[torch.arange(n)[:, None, None, None], iy, ix, torch.arange(c)[None, None, None, :]]
    assert torch.equal(win.cpu(), exp)
    dout = torch.randn(n, oh, ow, c, generator=g).to(dtype).to(cuda)
    ref = [t.clone() for t in K.pool_bwd_gather(dout, 0, am, y, n, h, w, c, kh, kw, st)]
    got = K.pool_bwd_gather(dout, 0, am, y, n, h, w, c, kh, kw, st, win=win)
    torch.cuda.synchronize()
    for u, v in zip(got, ref):
        assert torch.equal(u, v)


@pytest.mark.parametrize("kind", ["conv1", "conv3", "conv8"])
def test_wave_conv_eval_mode_equals_training_mode(cuda, kind):
    """The eval-mode launches (no BN statistics) of the wave-persistent EnvNet convs write the same
    output, bit for bit, as their training-mode launches on the same operands."""
    g = torch.Generator(device=cuda).manual_seed(77)
    bias = torch.randn(32, generator=g, device=cuda) * 0.5
    if kind == "conv1":
        n, t = 3, 9000
        x = torch.randn(n, t, generator=g, device=cuda) * 0.1
        wp = K.pack_weight(torch.randn(32, 1, 1, 64, generator=g, device=cuda) * 0.1, L.BF16, 0)
        P = n * ((t - 64) // 2 + 1)

        def run(y, stats):
            return K.fe_conv1_fwd(x, wp, bias, y, n, t, stats=stats)
    elif kind == "conv3":
        n, h, wd = 3, 64, 860
        x = (torch.randn(n, h, wd, generator=g, device=cuda) * 0.5).to(torch.bfloat16)
        wp = K.pack_weight(torch.randn(32, 1, 8, 8, generator=g, device=cuda) * 0.1, L.BF16, 0)
        P = n * (h - 7) * (wd - 7)

        def run(y, stats):
            return K.fe_conv3_fwd(x, wp, bias, y, n, h, wd, stats=stats)
    else:
        n, h, wd = 2, 57, 853
        x = (torch.randn(n, h, wd, 32, generator=g, device=cuda) * 0.7 + 0.1).to(torch.bfloat16)
        scale = torch.rand(32, generator=g, device=cuda) + 0.5
        shift = torch.randn(32, generator=g, device=cuda) * 0.3
        wp = K.pack_weight(torch.randn(32, 32, 8, 8, generator=g, device=cuda) * 0.03, L.BF16, 0)
        P = n * (h - 7) * (wd - 7)

        def run(y, stats):
            return K.trunk_conv8(x, wp, y, n, h, wd, scale=scale, shift=shift, bias=bias, stats=stats)
    ya = torch.full((P, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    yb = torch.full((P, 32), float("nan"), dtype=torch.bfloat16, device=cuda)
    run(ya, True)
    run(yb, False)
    torch.cuda.synchronize()
    assert torch.isfinite(yb.float()).all()
    assert torch.equal(ya, yb), float((ya.float() - yb.float()).abs().max())
