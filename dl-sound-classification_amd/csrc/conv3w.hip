// Weight gradient of the EnvNet-v2 trunk conv3 (Conv2d(1, 32, (8, 8)), reference
// src/models/envnet_v2.py:31), bf16 MFMA, gfx950:
//
//   dW[co][ky*8 + kx] = sum_{b, oy, ox} dY[b][oy][ox][co] * x[b][oy+ky][ox+kx]
//
// Wave-persistent, no barriers (the mirror of fe_conv3_kernel): a wave owns (clip, output row,
// 32 output columns) items.  Per item it stages the 8 input rows x 40 samples it needs into a
// per-wave LDS strip as four copies shifted by 0..3 samples (so the 8 consecutive samples of any
// tap are two aligned ds_read_b64) and the [32 px][32 co] dY tile (64-B rows, read transposed with
// ds_read_b64_tr_b16 as the A operand dY^T).  K = the 32 pixels (2 k-steps), N = the 64 taps
// (2 tiles): 4 MFMAs per item into 32 accumulator registers kept across all items; the next item's
// loads are in flight while the current one computes.  dY is read from HBM exactly once; each wave
// writes one f32 slab and a fixed-order reduce sums the slabs (bit-reproducible).
#include "common.h"

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

struct W3Args {
  const bf16* x;   // (n, h, wd) 1-channel image
  const bf16* dy;  // (n, h-7, wd-7, 32); BN: the gradient of relu(bn(ya)) (dA)
  float* part;     // [waves][32][64]
  int n, h, wd, oh, ow, nseg;
  // BN (mia_conv3_wgrad_bn): dY = the ReLU+BN backward of dA (mia_bn_relu_bwd_apply's arithmetic), formed while
  // staging, written to dyo and summed per channel into bpart [waves][32] (the conv bias gradient)
  const bf16* ya;
  bf16* dyo;
  float* bpart;
  const float *gamma, *scale, *shift, *mean, *invstd, *dgamma, *dbeta;
  int64_t P;
};

__device__ __forceinline__ bf16x8 tr_frag(const char* p0, int stride) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * stride));
  const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, c);
}

template <bool BN>
__global__ __launch_bounds__(256) void conv3_wgrad_kernel(W3Args g) {
  constexpr int ROWB = 80, CPYB = 704;  // 80-B rows (conflict-free staging writes), copies 704 B apart (48 banks: conflict-free reads)
  __shared__ __attribute__((aligned(16))) char strip[4][4 * CPYB];
  __shared__ __attribute__((aligned(16))) char dyt[4][32 * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
  const int items = g.n * g.oh * g.nseg;
  char* sg = strip[wv];
  char* dt = dyt[wv];
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; }

  // staging: lane l (l - 40 for l >= 40) loads input row l / 5, samples 8q .. 8q+11 (q = l % 5) as three 8-byte
  // loads (past the row end -> 0); every lane loads two 16-B dY chunks (px = q >> 2, 8 channels)
  struct Raw { u32x2 v[3]; u32x4 d[2]; u32x4 y[BN ? 2 : 1]; uint32_t ok; };
  // BN: per-channel constants as bn_bwd_apply_kernel<true> forms them (in LDS: registers would cost the
  // kernel its occupancy), [scale, shift, gamma*invstd, mean, invstd, dbeta/P, dgamma/P][channel]
  __shared__ __attribute__((aligned(16))) float bnp[7][32];
  float bs1[8];
  if constexpr (BN) {
    if (threadIdx.x < 32) {
      const int c = threadIdx.x;
      const float invP = 1.f / (float)g.P;
      const float is = g.invstd[c];
      bnp[0][c] = g.scale[c];
      bnp[1][c] = g.shift[c];
      bnp[2][c] = (g.gamma ? g.gamma[c] : 1.f) * is;
      bnp[3][c] = g.mean[c];
      bnp[4][c] = is;
      bnp[5][c] = g.dbeta[c] * invP;
      bnp[6][c] = g.dgamma[c] * invP;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) bs1[i] = 0.f;
    __syncthreads();
  }
  auto load = [&](int it) __attribute__((always_inline)) {
    Raw R;
    it = it < items ? it : items - 1;
    const int seg = it % g.nseg, rest = it / g.nseg;
    const int oy = rest % g.oh, b = rest / g.oh;
    const int l = lane < 40 ? lane : lane - 40;  // lanes 40..63 load lanes 0..23's bytes (not staged)
    const int r = l / 5, q = l % 5;
    const int col = seg * 32 + 8 * q;
    const bf16* src = g.x + ((int64_t)b * g.h + oy + r) * g.wd;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int c = col + 4 * k;
      R.v[k] = c + 4 <= g.wd ? *reinterpret_cast<const u32x2*>(src + c) : u32x2{0u, 0u};
    }
    const int64_t drow = ((int64_t)b * g.oh + oy) * g.ow * 32;
    R.ok = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int qq = lane + 64 * s;
      const int px = seg * 32 + (qq >> 2);
      const int64_t off = drow + (int64_t)px * 32 + (qq & 3) * 8;
      R.d[s] = px < g.ow ? *reinterpret_cast<const u32x4*>(g.dy + off) : u32x4{0u, 0u, 0u, 0u};
      if constexpr (BN) R.y[s] = px < g.ow ? *reinterpret_cast<const u32x4*>(g.ya + off) : u32x4{0u, 0u, 0u, 0u};
      R.ok |= (uint32_t)(px < g.ow) << s;
    }
    (void)drow;
    return R;
  };
  const int i16 = lane & 15, gq = lane >> 4, h = lane >> 5;
  const int n = lane & 31;  // tap within an N tile: ky = 4*nt + (n >> 3), kx = n & 7
  // BN: dY chunk s of item `it` from dA and ya (zero past the row end), stored to dyo and summed
  auto bn_chunk = [&](const Raw& R, int s, int it) __attribute__((always_inline)) -> u32x4 {
    if (!((R.ok >> s) & 1u)) return u32x4{0u, 0u, 0u, 0u};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t dw = R.d[s][k], yw = R.y[s][k];
      float gv[2] = {__uint_as_float(dw << 16), __uint_as_float(dw & 0xffff0000u)};
      const float xv[2] = {__uint_as_float(yw << 16), __uint_as_float(yw & 0xffff0000u)};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = 2 * k + j, c = (lane & 3) * 8 + i;
        gv[j] = fmaf(xv[j], bnp[0][c], bnp[1][c]) > 0.f ? gv[j] : 0.f;
        gv[j] = bnp[2][c] * (gv[j] - bnp[5][c] - (xv[j] - bnp[3][c]) * bnp[4][c] * bnp[6][c]);
        bs1[i] += gv[j];
      }
      o[k] = pk_bf16(gv[0], gv[1]);
    }
    const int seg = it % g.nseg, rest = it / g.nseg;
    const int oy = rest % g.oh, b = rest / g.oh;
    const int qq = lane + 64 * s;
    const int px = seg * 32 + (qq >> 2);
    const u32x4 v = {o[0], o[1], o[2], o[3]};
    *reinterpret_cast<u32x4*>(g.dyo + (((int64_t)b * g.oh + oy) * g.ow + px) * 32 + (qq & 3) * 8) = v;
    return v;
  };
  auto run = [&](const Raw& R, int it) __attribute__((always_inline)) {
    u32x4 dv[2] = {R.d[0], R.d[1]};
    if constexpr (BN) {
      dv[0] = bn_chunk(R, 0, it);
      dv[1] = bn_chunk(R, 1, it);
    }
    wave_sync();  // the previous item's fragment reads are done (common.h)
    if (lane < 40) {  // lanes 40..63 hold duplicates: writing them too cost LDS cycles (0.355 -> 0.292 ms)
      const int l = lane;
      const int r = l / 5, q = l % 5;
      const uint32_t d[6] = {R.v[0][0], R.v[0][1], R.v[1][0], R.v[1][1], R.v[2][0], R.v[2][1]};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        // copy c dword i = samples (8q + c + 2i, +1)
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = c + 2 * i;
          o[i] = (e & 1) ? ((d[e >> 1] >> 16) | (d[(e >> 1) + 1] << 16)) : d[e >> 1];
        }
        *reinterpret_cast<u32x4*>(sg + c * CPYB + r * ROWB + 16 * q) = u32x4{o[0], o[1], o[2], o[3]};
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int qq = lane + 64 * s;
      *reinterpret_cast<u32x4*>(dt + (qq >> 2) * 64 + (qq & 3) * 16) = dv[s];
    }
    wave_sync();
    const int kx = n & 7, cp = kx & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
      const int c4 = 16 * (gq & 1) + 4 * (i16 & 3);
      const bf16x8 fa = tr_frag(dt + kr * 64 + c4 * 2, 64);  // dY^T[co][px = 16ks + 8h + j]
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int ky = 4 * nt + (n >> 3);
        // x[oy+ky][16ks + 8h + kx + j], j = 0..7: copy kx&3 at sample 16ks + 8h + (kx&4)
        const char* src = sg + cp * CPYB + ky * ROWB + 2 * (16 * ks + 8 * h + (kx & 4));
        const u32x2 p0 = *reinterpret_cast<const u32x2*>(src);
        const u32x2 p1 = *reinterpret_cast<const u32x2*>(src + 8);
        const u32x4 f = {p0[0], p0[1], p1[0], p1[1]};
        acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, __builtin_bit_cast(bf16x8, f), acc[nt], 0, 0, 0);
      }
    }
  };

  int it = gw;
  if (it < items) {
    Raw ra = load(it), rb;
    for (;;) {
      rb = load(it + nw);
      run(ra, it);
      it += nw;
      if (it >= items) break;
      ra = load(it + nw);
      run(rb, it);
      it += nw;
      if (it >= items) break;
    }
  }
  // slab [co][tap]: accumulator row = co, column = tap
  float* dst = g.part + (int64_t)gw * 2048;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
      dst[co * 64 + nt * 32 + n] = acc[nt][r];
    }
  if constexpr (BN) {
    // lanes with equal lane & 3 hold the same channels
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int m = 4; m < 64; m <<= 1) bs1[i] += __shfl_xor(bs1[i], m, 64);
    if (lane < 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g.bpart[(int64_t)gw * 32 + lane * 8 + i] = bs1[i];
    }
  }
}

// dbias[c] = sum over the waves' partials (f64, fixed order)
__global__ void conv3_bias_final_kernel(const float* __restrict__ bpart, int nw, float* __restrict__ dbias) {
  const double s = block_sum_strided(bpart + blockIdx.x, nw, 32);
  if (threadIdx.x == 0) dbias[blockIdx.x] = (float)s;
}

// dw[e] = sum of the slabs (fixed order, bit-reproducible), e = co*64 + tap, in two coalesced stages:
// stage 1: group g of C3_G sums its slabs in order into tmp[g][e] (double); stage 2: tmp summed in g order
constexpr int C3_G = 64;
__global__ __launch_bounds__(256) void conv3_wgrad_reduce1_kernel(const float* __restrict__ part, int nslab,
                                                                  double* __restrict__ tmp) {
  const int e = blockIdx.x * 256 + threadIdx.x, gi = blockIdx.y;
  const int per = (nslab + C3_G - 1) / C3_G;
  const int w0 = gi * per, w1 = min(nslab, w0 + per);
  double s = 0.0;
  for (int w = w0; w < w1; ++w) s += (double)part[(int64_t)w * 2048 + e];
  tmp[gi * 2048 + e] = s;
}
__global__ __launch_bounds__(256) void conv3_wgrad_reduce2_kernel(const double* __restrict__ tmp, float* __restrict__ dw) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < C3_G; ++g) s += tmp[g * 2048 + e];
  dw[e] = (float)s;
}

}  // namespace

extern "C" int mia_conv3_wgrad(const void* x, const void* dy, float* dw, float* part, int32_t nwaves, int32_t n,
                               int32_t h, int32_t wd, mia_stream_t stream) {
  MIA_CHECK_ARG(x && dy && dw && part && n > 0 && h >= 8 && wd >= 8, "conv3_wgrad: bad arguments");
  MIA_CHECK_ARG(nwaves > 0 && nwaves % 4 == 0, "conv3_wgrad: nwaves must be a positive multiple of 4");
  MIA_CHECK_ARG(wd % 4 == 0, "conv3_wgrad: image width must be a multiple of 4 (8-byte row alignment)");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(dy) & 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0,
                "conv3_wgrad: dy must be 16-byte and x 8-byte aligned");
  W3Args a{reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(dy), part, n, h, wd, h - 7, wd - 7,
           (int)cdiv(wd - 7, 32)};
  MIA_CHECK_ARG((int64_t)n * a.oh * a.nseg < (1ll << 31), "conv3_wgrad: too many items");
  hipStream_t s = as_stream(stream);
  conv3_wgrad_kernel<false><<<nwaves / 4, 256, 0, s>>>(a);
  MIA_LAUNCH_CHECK("conv3_wgrad");
  double* tmp = reinterpret_cast<double*>(part + (int64_t)nwaves * 2048);
  conv3_wgrad_reduce1_kernel<<<dim3(8, C3_G), 256, 0, s>>>(part, nwaves, tmp);
  conv3_wgrad_reduce2_kernel<<<8, 256, 0, s>>>(tmp, dw);
  MIA_LAUNCH_CHECK("conv3_wgrad_reduce");
  return 0;
}

extern "C" int64_t mia_conv3_wgrad_workspace_bytes(int32_t nwaves) {
  return (int64_t)nwaves * 2048 * 4 + (int64_t)C3_G * 2048 * 8 + (int64_t)nwaves * 32 * 4;
}

extern "C" int mia_conv3_wgrad_bn(const void* x, const void* da, const void* ya, void* dy, float* dw, float* dbias,
                                  float* part, int32_t nwaves, int32_t n, int32_t h, int32_t wd, const float* gamma,
                                  const float* scale, const float* shift, const float* mean, const float* invstd,
                                  const float* dgamma, const float* dbeta, mia_stream_t stream) {
  MIA_CHECK_ARG(x && da && ya && dy && dw && dbias && part && n > 0 && h >= 8 && wd >= 8,
                "conv3_wgrad_bn: bad arguments");
  MIA_CHECK_ARG(scale && shift && mean && invstd && dgamma && dbeta, "conv3_wgrad_bn: null BN statistics");
  MIA_CHECK_ARG(nwaves > 0 && nwaves % 4 == 0, "conv3_wgrad_bn: nwaves must be a positive multiple of 4");
  MIA_CHECK_ARG(wd % 4 == 0, "conv3_wgrad_bn: image width must be a multiple of 4 (8-byte row alignment)");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(da) | reinterpret_cast<uintptr_t>(ya) | reinterpret_cast<uintptr_t>(dy)) &
                 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0,
                "conv3_wgrad_bn: da / ya / dy must be 16-byte and x 8-byte aligned");
  W3Args a{reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(da), part, n, h, wd, h - 7, wd - 7,
           (int)cdiv(wd - 7, 32), reinterpret_cast<const bf16*>(ya), reinterpret_cast<bf16*>(dy), nullptr,
           gamma, scale, shift, mean, invstd, dgamma, dbeta, (int64_t)n * (h - 7) * (wd - 7)};
  MIA_CHECK_ARG((int64_t)n * a.oh * a.nseg < (1ll << 31), "conv3_wgrad_bn: too many items");
  double* tmp = reinterpret_cast<double*>(part + (int64_t)nwaves * 2048);
  a.bpart = reinterpret_cast<float*>(tmp + (int64_t)C3_G * 2048);
  hipStream_t s = as_stream(stream);
  conv3_wgrad_kernel<true><<<nwaves / 4, 256, 0, s>>>(a);
  MIA_LAUNCH_CHECK("conv3_wgrad_bn");
  conv3_wgrad_reduce1_kernel<<<dim3(8, C3_G), 256, 0, s>>>(part, nwaves, tmp);
  conv3_wgrad_reduce2_kernel<<<8, 256, 0, s>>>(tmp, dw);
  conv3_bias_final_kernel<<<32, 256, 0, s>>>(a.bpart, nwaves, dbias);
  MIA_LAUNCH_CHECK("conv3_wgrad_bn reduce");
  return 0;
}
