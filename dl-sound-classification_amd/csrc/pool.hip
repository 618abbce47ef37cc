// Max-pool fused with the preceding BatchNorm-apply + ReLU, and its backward (gfx950).
// nn.MaxPool2d(kernel == stride, floor) after BN+ReLU (envnet_v2.py:16-23, 32-37).
// The pooled layers never materialise relu(bn(x)): the forward reads the raw conv output once and
// writes only the pooled map (+ a u8 argmax per output), the backward scatters the pooled
// gradient through the argmax, masks it with the recomputed ReLU and produces the BN backward
// reductions in the same pass.  Ties keep the first maximum in row-major window order, like the
// PyTorch CPU kernel.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int NT = 256;

// n / d for 0 <= n < 2^31 without an integer division (Granlund-Montgomery: one mul_hi, add, shift)
struct FastDiv {
  uint32_t d, m, l;
};
static FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1u << l) < d) ++l;
  const uint32_t m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
  return FastDiv{d, m, l};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.l; }

__device__ __forceinline__ int64_t out_index(int layout, int b, int oy, int ox, int c, int OH, int OW, int C) {
  if (layout == 0) return (((int64_t)b * OH + oy) * OW + ox) * C + c;
  if (layout == 1) return ((int64_t)b * C + c) * OW + ox;                 // (n, c, ow), OH == 1
  return (((int64_t)b * C + c) * OH + oy) * OW + ox;                       // NCHW flat
}

// one thread = one (output pixel, 8-channel group)
__global__ __launch_bounds__(NT) void pool_fwd_kernel(const void* __restrict__ x, int dtype, int n, int H, int W,
                                                      int C, int kh, int kw, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, void* out, int layout,
                                                      uint8_t* __restrict__ argmax, void* __restrict__ win) {
  const int OH = H / kh, OW = W / kw, G = C / 8;
  const int total = n * OH * OW * G;  // < 2^31 (checked by the launcher): 32-bit index math
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < total; idx += gridDim.x * NT) {
    const int cg = idx % G;
    int p = idx / G;
    const int ox = p % OW;
    p /= OW;
    const int oy = p % OH;
    const int b = p / OH;
    float sc[8], sh[8], best[8], raw[8];
    int arg[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = scale ? scale[cg * 8 + i] : 1.f;
      sh[i] = shift ? shift[cg * 8 + i] : 0.f;
      best[i] = -INFINITY;
      raw[i] = 0.f;
      arg[i] = 0;
    }
    for (int dy = 0; dy < kh; ++dy) {
      const int iy = oy * kh + dy;
      for (int dx = 0; dx < kw; ++dx) {
        const int ix = ox * kw + dx;
        const int64_t off = (((int64_t)b * H + iy) * W + ix) * C + cg * 8;
        float f[8];
        if (dtype == MIA_BF16) {
          uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(x) + off);
          uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(w4[i] << 16); f[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u); }
        } else {
          const float4* q = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x) + off);
          float4 a = q[0], c4 = q[1];
          f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = c4.x; f[5] = c4.y; f[6] = c4.z; f[7] = c4.w;
        }
        const int pos = dy * kw + dx;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float v = fmaxf(fmaf(f[i], sc[i], sh[i]), 0.f);
          if (v > best[i]) { best[i] = v; raw[i] = f[i]; arg[i] = pos; }
        }
      }
    }
    const int64_t aoff = (((int64_t)b * OH + oy) * OW + ox) * C + cg * 8;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a0 |= (uint32_t)arg[i] << (8 * i); a1 |= (uint32_t)arg[i + 4] << (8 * i); }
    *reinterpret_cast<uint2*>(argmax + aoff) = make_uint2(a0, a1);
    if (win) store8(win, dtype, aoff, raw);  // the winner's raw x (exact: x's own dtype) for the backward
    if (layout == 0) {
      store8(out, dtype, aoff, best);  // NHWC: the 8 channels are one 16-B (bf16) / 32-B (f32) run
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) st_elem(out, dtype, out_index(layout, b, oy, ox, cg * 8 + i, OH, OW, C), best[i]);
    }
  }
}

// maxpool(relu(bn(x))) before the BN statistics exist (bf16 x, training): relu(s*x + t) is monotone in
// x with the sign of s = gamma*invstd, i.e. of gamma, so the window's winner is the raw maximum
// (gamma > 0), the raw minimum (gamma < 0) or, gamma == 0, the first position (every z ties), always
// the first occurrence -- torch's max_pool2d routing (when relu clamps the whole window the routed
// position differs from torch's first-position pick, but its gradient relu'(z) * g is 0 at either).
// One pass over x: the winner's raw value (bf16) + argmax, and the BN shifted sums about kshift[c]
// (the conv bias) of every pixel -> partial[block][C][2] for mia_bn_finalize_shifted; the pooled
// relu(s*x_win + t) is written by pool_apply_kernel once the statistics are final.
__global__ __launch_bounds__(NT) void pool_raw_stats_kernel(const bf16* __restrict__ x, int n, int H, int W, int C,
                                                            int kh, int kw, const float* __restrict__ gamma,
                                                            const float* __restrict__ kshift, bf16* __restrict__ win,
                                                            uint8_t* __restrict__ argmax, float* __restrict__ partial) {
  const int OH = H / kh, OW = W / kw, G = C / 8;
  const int total = n * OH * OW * G;
  const int cg = threadIdx.x % G;  // constant per thread (G | NT, gridDim*NT a multiple of G)
  float dir[8], ks[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float gv = gamma[cg * 8 + i];
    dir[i] = gv > 0.f ? 1.f : (gv < 0.f ? -1.f : 0.f);
    ks[i] = kshift[cg * 8 + i];
    s1[i] = 0.f; s2[i] = 0.f;
  }
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < total; idx += gridDim.x * NT) {
    int p = idx / G;
    const int ox = p % OW;
    p /= OW;
    const int oy = p % OH;
    const int b = p / OH;
    float best[8], bestraw[8];
    int arg[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { best[i] = -INFINITY; bestraw[i] = 0.f; arg[i] = 0; }
    for (int dy = 0; dy < kh; ++dy) {
      const int iy = oy * kh + dy;
      const bf16* row = x + (((int64_t)b * H + iy) * W + (int64_t)ox * kw) * C + cg * 8;
#pragma unroll 4
      for (int dx = 0; dx < kw; ++dx) {
        const uint4 u = *reinterpret_cast<const uint4*>(row + (int64_t)dx * C);
        const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
        float f[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(w4[i] << 16); f[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u); }
        const int pos = dy * kw + dx;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = f[i] - ks[i];
          s1[i] += d;
          s2[i] = fmaf(d, d, s2[i]);
          const float key = dir[i] * f[i];  // gamma == 0: key 0 everywhere -> first position wins
          if (key > best[i]) { best[i] = key; bestraw[i] = f[i]; arg[i] = pos; }
        }
      }
    }
    const int64_t aoff = (((int64_t)b * OH + oy) * OW + ox) * C + cg * 8;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a0 |= (uint32_t)arg[i] << (8 * i); a1 |= (uint32_t)arg[i + 4] << (8 * i); }
    *reinterpret_cast<uint2*>(argmax + aoff) = make_uint2(a0, a1);
    uint32_t o4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o4[i] = pk_bf16(bestraw[2 * i], bestraw[2 * i + 1]);  // exact: bf16 inputs
    }
    *reinterpret_cast<uint4*>(win + aoff) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
  }
  // pixels right of the last full window (W % kw of them per row) enter the statistics only
  const int tailw = W - OW * kw;
  const int ttotal = n * H * tailw * G;
  for (int idx = blockIdx.x * NT + threadIdx.x; idx < ttotal; idx += gridDim.x * NT) {
    int p = idx / G;
    const int tx = p % tailw;
    const int r = p / tailw;  // b * H + iy
    const uint4 u = *reinterpret_cast<const uint4*>(x + ((int64_t)r * W + OW * kw + tx) * C + cg * 8);
    const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = __uint_as_float(w4[i] << 16) - ks[2 * i], hi = __uint_as_float(w4[i] & 0xffff0000u) - ks[2 * i + 1];
      s1[2 * i] += lo; s2[2 * i] = fmaf(lo, lo, s2[2 * i]);
      s1[2 * i + 1] += hi; s2[2 * i + 1] = fmaf(hi, hi, s2[2 * i + 1]);
    }
  }
  // block reduction of the shifted sums per channel (threads with equal cg), fixed order
  __shared__ float red[NT][17];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[threadIdx.x][i] = s1[i]; red[threadIdx.x][8 + i] = s2[i]; }
  __syncthreads();
  if ((int)threadIdx.x < C * 2) {
    const int c = threadIdx.x >> 1, which = threadIdx.x & 1, g = c >> 3, i = c & 7;
    float a = 0.f;
    for (int t = g; t < NT; t += G) a += red[t][which * 8 + i];
    partial[((int64_t)blockIdx.x * C + c) * 2 + which] = a;
  }
}

// pooled output relu(scale*x_win + shift) in the requested layout (see pool_fwd_kernel)
__global__ __launch_bounds__(NT) void pool_apply_kernel(const bf16* __restrict__ win, int n, int OH, int OW, int C,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        void* out, int dtype, int layout) {
  const int64_t total = (int64_t)n * OH * OW * C;
  for (int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x; e < total; e += (int64_t)gridDim.x * NT) {
    const int c = (int)(e % C);
    int64_t p = e / C;
    const int ox = (int)(p % OW);
    p /= OW;
    const int oy = (int)(p % OH), b = (int)(p / OH);
    const float v = fmaxf(fmaf((float)win[e], scale[c], shift[c]), 0.f);
    st_elem(out, dtype, out_index(layout, b, oy, ox, c, OH, OW, C), v);
  }
}

// pool_apply into the transposed trunk image (layout 1: (n, 64, ow), oh == 1, bf16): a 64-pixel x 64-channel
// tile per block, read as 16-B channel runs, relu(s x + t) rounded to bf16 into a padded LDS tile, written back
// as 8-B runs of 4 pixels per channel row (the per-element form scattered 2-B stores 2 * ow bytes apart:
// 0.107 ms at 1.4 TB/s for the frontend pool of a B = 256 step).  Same arithmetic, same bits.
__global__ __launch_bounds__(256) void pool_apply_t64_kernel(const bf16* __restrict__ win, int OW,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, bf16* __restrict__ out) {
  __shared__ bf16 tile[64][64 + 4];  // [channel][pixel]
  const int tiles = (OW + 63) / 64;
  const int b = blockIdx.x / tiles, p0 = (blockIdx.x - b * tiles) * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = t + 256 * k, r = q >> 3, ch = q & 7;  // pixel p0 + r, channels 8 ch .. 8 ch + 7
    bf16x8 v = {};
    if (p0 + r < OW) v = *reinterpret_cast<const bf16x8*>(win + ((int64_t)b * OW + p0 + r) * 64 + ch * 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = ch * 8 + i;
      tile[c][r] = (bf16)fmaxf(fmaf((float)v[i], scale[c], shift[c]), 0.f);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int q = t + 256 * k, c = q >> 4, g = q & 15;  // channel c, pixels p0 + 4 g .. + 3
    const int p = p0 + 4 * g;
    bf16* dst = out + ((int64_t)b * 64 + c) * OW + p;
    const bf16x4 w4 = *reinterpret_cast<const bf16x4*>(&tile[c][4 * g]);
    if (p + 4 <= OW && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
      *reinterpret_cast<bf16x4*>(dst) = w4;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (p + i < OW) dst[i] = w4[i];
    }
  }
}

// one thread = one (input pixel, 8-channel group); block partial reductions like norm.hip
__global__ __launch_bounds__(NT) void pool_bwd_kernel(const void* __restrict__ dout, int layout,
                                                      const uint8_t* __restrict__ argmax, const void* __restrict__ x,
                                                      int dtype, int n, int H, int W, int C, int kh, int kw,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ invstd, void* dz,
                                                      float* __restrict__ partial) {
  const int OH = H / kh, OW = W / kw, G = C / 8;
  const int t = threadIdx.x;
  const int cg = t % G, rs = t / G, rslots = NT / G;
  float sc[8], sh[8], mu[8], is[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[cg * 8 + i]; sh[i] = shift[cg * 8 + i]; mu[i] = mean[cg * 8 + i]; is[i] = invstd[cg * 8 + i];
  }
  float s1[8] = {0}, s2[8] = {0};
  const int P = n * H * W;  // < 2^31 (checked by the launcher): 32-bit index math
  for (int r = blockIdx.x * rslots + rs; r < P; r += gridDim.x * rslots) {
    const int ix = r % W;
    const int q = r / W;
    const int iy = q % H;
    const int b = q / H;
    const int64_t off = (int64_t)r * C + cg * 8;
    float g[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = 0.f;
    const int oy = iy / kh, ox = ix / kw;
    if (oy < OH && ox < OW) {
      const int pos = (iy - oy * kh) * kw + (ix - ox * kw);
      const int64_t aoff = (((int64_t)b * OH + oy) * OW + ox) * C + cg * 8;
      const uint2 am = *reinterpret_cast<const uint2*>(argmax + aoff);
      float xv[8];
      if (dtype == MIA_BF16) {
        uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(x) + off);
        uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { xv[2 * i] = __uint_as_float(w4[i] << 16); xv[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u); }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = reinterpret_cast<const float*>(x)[off + i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t word = i < 4 ? am.x : am.y;
        const int a = (int)((word >> (8 * (i & 3))) & 0xffu);
        if (a == pos && fmaf(xv[i], sc[i], sh[i]) > 0.f) {
          g[i] = ld_elem(dout, dtype, out_index(layout, b, oy, ox, cg * 8 + i, OH, OW, C));
          s1[i] += g[i];
          s2[i] = fmaf(g[i], (xv[i] - mu[i]) * is[i], s2[i]);
        }
      }
    }
    store8(dz, dtype, off, g);
  }
  __shared__ float red[NT * 16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[t * 16 + i] = s1[i]; red[t * 16 + 8 + i] = s2[i]; }
  __syncthreads();
  for (int e = t; e < 2 * C; e += NT) {
    const int qq = e / C, c = e % C, g2 = c / 8, ci = c % 8;
    float acc = 0.f;
    for (int r2 = 0; r2 < rslots; ++r2) acc += red[(r2 * G + g2) * 16 + qq * 8 + ci];
    partial[((int64_t)blockIdx.x * C + c) * 2 + qq] = acc;
  }
}

// Sparse BN reductions of the pooled backward: only the argmax position of each pooled cell carries
// a gradient, so dbeta = sum g and dgamma = sum g * xhat are gathered per pooled cell (one thread =
// one (pooled cell, 8-channel group)) without touching the other kh*kw - 1 pixels of the window.
// gm[cell][c] (f32, NHWC cells) keeps the ReLU-masked gradient at the argmax for the dense pass.
// win (optional, NHWC cells, x's dtype): the raw winner value of each cell saved by the forward
// (pool_raw_stats); when given, x is not gathered at all -- a contiguous read replaces kh*kw-strided
// 2-byte gathers that each touch a separate cache line.
__global__ __launch_bounds__(NT) void pool_bwd_sparse_kernel(const void* __restrict__ dout, int layout,
                                                             const uint8_t* __restrict__ argmax,
                                                             const void* __restrict__ x,
                                                             const void* __restrict__ win, int dtype, int n, int H,
                                                             int W, int C, int kh, int kw,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             float* __restrict__ gm,
                                                             float* __restrict__ partial) {
  const int OH = H / kh, OW = W / kw, G = C / 8;
  const int t = threadIdx.x;
  const int cg = t % G, rs = t / G, rslots = NT / G;
  float sc[8], sh[8], mu[8], is[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[cg * 8 + i]; sh[i] = shift[cg * 8 + i]; mu[i] = mean[cg * 8 + i]; is[i] = invstd[cg * 8 + i];
  }
  float s1[8] = {0}, s2[8] = {0};
  const int cells = n * OH * OW;
  for (int cell = blockIdx.x * rslots + rs; cell < cells; cell += gridDim.x * rslots) {
    const int ox = cell % OW;
    const int q = cell / OW;
    const int oy = q % OH;
    const int b = q / OH;
    float xv[8], dv[8];
    if (win) {
      const int64_t off = (int64_t)cell * C + cg * 8;
      load8(win, dtype, off, xv);
#pragma unroll
      for (int i = 0; i < 8; ++i) dv[i] = ld_elem(dout, dtype, out_index(layout, b, oy, ox, cg * 8 + i, OH, OW, C));
    } else {
      const uint2 am = *reinterpret_cast<const uint2*>(argmax + (int64_t)cell * C + cg * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // all loads first, unconditionally
        const uint32_t word = i < 4 ? am.x : am.y;
        const int a = (int)((word >> (8 * (i & 3))) & 0xffu);
        const int iy = oy * kh + a / kw, ix = ox * kw + a % kw;
        xv[i] = ld_elem(x, dtype, (((int64_t)b * H + iy) * W + ix) * C + cg * 8 + i);
        dv[i] = ld_elem(dout, dtype, out_index(layout, b, oy, ox, cg * 8 + i, OH, OW, C));
      }
    }
    float gv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float g = fmaf(xv[i], sc[i], sh[i]) > 0.f ? dv[i] : 0.f;
      gv[i] = g;
      s1[i] += g;
      s2[i] = fmaf(g, (xv[i] - mu[i]) * is[i], s2[i]);
    }
    float4* gq = reinterpret_cast<float4*>(gm + (int64_t)cell * C + cg * 8);
    gq[0] = make_float4(gv[0], gv[1], gv[2], gv[3]);
    gq[1] = make_float4(gv[4], gv[5], gv[6], gv[7]);
  }
  __shared__ float red[NT * 16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[t * 16 + i] = s1[i]; red[t * 16 + 8 + i] = s2[i]; }
  __syncthreads();
  for (int e = t; e < 2 * C; e += NT) {
    const int qq = e / C, c = e % C, g2 = c / 8, ci = c % 8;
    float acc = 0.f;
    for (int r2 = 0; r2 < rslots; ++r2) acc += red[(r2 * G + g2) * 16 + qq * 8 + ci];
    partial[((int64_t)blockIdx.x * C + c) * 2 + qq] = acc;
  }
}

// Dense BN backward of a pooled layer in one pass: dx = gamma*invstd*(g - dbeta/P - xhat*dgamma/P)
// with g = gm[cell] at the argmax position of the pixel's pooled cell, 0 elsewhere (gm already
// carries the ReLU mask).  Reads x once, writes dx once; the masked dense gradient is never
// materialised.  s1 partials = dbias.  All loads are unconditional (a conditional load makes hipcc
// wait vmcnt(0) in the loop); four pixels per thread-iteration.
// Same pass for pool windows kw % 8 == 0 (the frontend (1, 64) pool): a thread owns 8 channels x
// 8 consecutive pixels of one row, which always fall in ONE pooled cell, so the cell's argmax bytes
// and masked gradient (40 B) are read once per 8 pixels instead of once per pixel, and the index
// math runs once per octet.  All 8 pixel loads are issued before any use.
__global__ __launch_bounds__(NT) void pool_bn_bwd_apply_oct_kernel(const float* __restrict__ gm,
                                                                   const uint8_t* __restrict__ argmax,
                                                                   const bf16* __restrict__ x, int n, int H, int W,
                                                                   int C, int kh, int kw, FastDiv dNO, FastDiv dH,
                                                                   FastDiv dG, const float* __restrict__ gamma,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ invstd,
                                                                   const float* __restrict__ dgamma,
                                                                   const float* __restrict__ dbeta, bf16* dx,
                                                                   float* __restrict__ partial) {
  const int OH = H / kh, OW = W / kw, G = C / 8, NO = (W + 7) / 8;
  const int t = threadIdx.x;
  const int cg = t % G;
  const int P = n * H * W;
  float mu[8], is[8], a[8], mb[8], mg[8];
  const float invP = 1.f / (float)P;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i;
    mu[i] = mean[c]; is[i] = invstd[c];
    a[i] = (gamma ? gamma[c] : 1.f) * is[i];
    mb[i] = dbeta[c] * invP;
    mg[i] = dgamma[c] * invP;
  }
  float s1[8] = {0};
  const int64_t units = (int64_t)n * H * NO * G;
  for (int64_t u = (int64_t)blockIdx.x * NT + t; u < units; u += (int64_t)gridDim.x * NT) {
    const int rest = (int)fdiv((uint32_t)(u), dG);       // (b*H + iy)*NO + o8   (units < 2^31 checked)
    const int rowi = (int)fdiv((uint32_t)rest, dNO);     // b*H + iy
    const int o8 = rest - rowi * NO;
    const int iy = rowi - (int)fdiv((uint32_t)rowi, dH) * H;
    const int b = (rowi - iy) / H;
    const int ix0 = o8 * 8;
    const int oy = iy / kh, ox = ix0 / kw;
    const bool cell = oy < OH && ox < OW;
    const int64_t coff = cell ? (((int64_t)b * OH + oy) * OW + ox) * C + cg * 8 : 0;
    const uint2 am = *reinterpret_cast<const uint2*>(argmax + coff);
    const float4 g0 = reinterpret_cast<const float4*>(gm + coff)[0];
    const float4 g1 = reinterpret_cast<const float4*>(gm + coff)[1];
    const int64_t xoff = ((int64_t)rowi * W + ix0) * C + cg * 8;
    uint4 xr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t o = ix0 + j < W ? xoff + (int64_t)j * C : xoff;
      xr[j] = *reinterpret_cast<const uint4*>(x + o);
    }
    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const int pos0 = (iy - oy * kh) * kw + (ix0 - ox * kw);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ix0 + j >= W) break;
      const uint32_t w4[4] = {xr[j].x, xr[j].y, xr[j].z, xr[j].w};
      uint32_t o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float g[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * q + h;
          const float xv = __uint_as_float(h ? (w4[q] & 0xffff0000u) : (w4[q] << 16));
          const uint32_t word = i < 4 ? am.x : am.y;
          const int av = (int)((word >> (8 * (i & 3))) & 0xffu);
          const float gi = cell && av == pos0 + j ? gv[i] : 0.f;
          g[h] = a[i] * (gi - mb[i] - (xv - mu[i]) * is[i] * mg[i]);
          s1[i] += g[h];
        }
        o4[q] = pk_bf16(g[0], g[1]);
      }
      *reinterpret_cast<uint4*>(dx + xoff + (int64_t)j * C) = uint4{o4[0], o4[1], o4[2], o4[3]};
    }
  }
  if (!partial) return;
  __shared__ float red[NT * 8];
#pragma unroll
  for (int i = 0; i < 8; ++i) red[t * 8 + i] = s1[i];
  __syncthreads();
  const int rslots = NT / G;
  for (int c = t; c < C; c += NT) {
    const int g2 = c / 8, ci = c % 8;
    float acc = 0.f;
    for (int r2 = 0; r2 < rslots; ++r2) acc += red[(r2 * G + g2) * 8 + ci];
    partial[((int64_t)blockIdx.x * C + c) * 2] = acc;
  }
}

// Same pass for short pool windows (kw = 2..4, the trunk's (5, 3) and (1, 2) pools): a thread owns 8
// channels x the KW pixels of one row that fall in one pooled cell (a "run"); the cell's argmax bytes
// and masked gradient are read once per run and the index math runs once per run.  Pixels past the
// last whole cell (W % kw, H % kh) form runs with no cell (gradient term 0).  RU runs per
// thread-iteration, all loads issued before any use.  EnvNet block 0 (B = 256, 50 x 846 x 32, (5, 3)):
// 0.447 ms per pixel -> 0.345 ms per run (4.25 TB/s on x + dx + gm); folding the five per-channel
// constants into three (occupancy 4 -> 5) measured no faster.
template <int KW, int RU>
__global__ __launch_bounds__(NT) void pool_bn_bwd_apply_run_kernel(const float* __restrict__ gm,
                                                                   const uint8_t* __restrict__ argmax,
                                                                   const bf16* __restrict__ x, int n, int H, int W,
                                                                   int C, int kh, FastDiv dNR, FastDiv dH, FastDiv dG,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ invstd,
                                                                   const float* __restrict__ dgamma,
                                                                   const float* __restrict__ dbeta, bf16* dx,
                                                                   float* __restrict__ partial) {
  const int OH = H / kh, OW = W / KW, G = C / 8, NR = (W + KW - 1) / KW;
  const int t = threadIdx.x;
  const int cg = t % G;
  const int P = n * H * W;
  float mu[8], is[8], a[8], mb[8], mg[8];
  const float invP = 1.f / (float)P;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i;
    mu[i] = mean[c]; is[i] = invstd[c];
    a[i] = (gamma ? gamma[c] : 1.f) * is[i];
    mb[i] = dbeta[c] * invP;
    mg[i] = dgamma[c] * invP;
  }
  float s1[8] = {0};
  const int units = n * H * NR * G;  // < 2^31 (checked by the launcher)
  const int stride = gridDim.x * NT;
  for (int u0 = blockIdx.x * NT + t; u0 < units; u0 += RU * stride) {
    uint4 xr[RU][KW];
    uint2 am[RU];
    float4 g0[RU], g1[RU];
    int64_t xoff[RU];
    int pos0[RU], ix0[RU];
#pragma unroll
    for (int v = 0; v < RU; ++v) {
      const int u = min(u0 + v * stride, units - 1);
      const int rest = (int)fdiv((uint32_t)u, dG);        // (b*H + iy)*NR + run
      const int rowi = (int)fdiv((uint32_t)rest, dNR);    // b*H + iy
      const int run = rest - rowi * NR;
      const int b = (int)fdiv((uint32_t)rowi, dH);
      const int iy = rowi - b * H;
      ix0[v] = run * KW;
      const int oy = iy / kh;
      const bool cell = oy < OH && run < OW;
      const int64_t coff = cell ? (((int64_t)b * OH + oy) * OW + run) * C + cg * 8 : 0;
      pos0[v] = cell ? (iy - oy * kh) * KW : -256;
      am[v] = *reinterpret_cast<const uint2*>(argmax + coff);
      g0[v] = reinterpret_cast<const float4*>(gm + coff)[0];
      g1[v] = reinterpret_cast<const float4*>(gm + coff)[1];
      xoff[v] = ((int64_t)rowi * W + ix0[v]) * C + cg * 8;
#pragma unroll
      for (int j = 0; j < KW; ++j) {
        const int64_t o = ix0[v] + j < W ? xoff[v] + (int64_t)j * C : xoff[v];
        xr[v][j] = *reinterpret_cast<const uint4*>(x + o);
      }
    }
#pragma unroll
    for (int v = 0; v < RU; ++v) {
      if (u0 + v * stride >= units) break;
      const float gv[8] = {g0[v].x, g0[v].y, g0[v].z, g0[v].w, g1[v].x, g1[v].y, g1[v].z, g1[v].w};
#pragma unroll
      for (int j = 0; j < KW; ++j) {
        if (ix0[v] + j >= W) break;
        const uint32_t w4[4] = {xr[v][j].x, xr[v][j].y, xr[v][j].z, xr[v][j].w};
        uint32_t o4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float g[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * q + h;
            const float xv = __uint_as_float(h ? (w4[q] & 0xffff0000u) : (w4[q] << 16));
            const uint32_t word = i < 4 ? am[v].x : am[v].y;
            const int av = (int)((word >> (8 * (i & 3))) & 0xffu);
            const float gi = av == pos0[v] + j ? gv[i] : 0.f;
            g[h] = a[i] * (gi - mb[i] - (xv - mu[i]) * is[i] * mg[i]);
            s1[i] += g[h];
          }
          o4[q] = pk_bf16(g[0], g[1]);
        }
        *reinterpret_cast<uint4*>(dx + xoff[v] + (int64_t)j * C) = uint4{o4[0], o4[1], o4[2], o4[3]};
      }
    }
  }
  if (!partial) return;
  __shared__ float red[NT * 8];
#pragma unroll
  for (int i = 0; i < 8; ++i) red[t * 8 + i] = s1[i];
  __syncthreads();
  const int rslots = NT / G;
  for (int c = t; c < C; c += NT) {
    const int g2 = c / 8, ci = c % 8;
    float acc = 0.f;
    for (int r2 = 0; r2 < rslots; ++r2) acc += red[(r2 * G + g2) * 8 + ci];
    partial[((int64_t)blockIdx.x * C + c) * 2] = acc;
  }
}

#ifndef PB_UNROLL
#define PB_UNROLL 4
#endif
#ifndef PB_NB
#define PB_NB 1024
#endif
#ifndef PB_RUNS
#define PB_RUNS 1  // runs per thread-iteration: 1, 2, 3 measured equal within 5% (block 0: 0.34-0.36 ms)
#endif
__global__ __launch_bounds__(NT) void pool_bn_bwd_apply_kernel(const float* __restrict__ gm,
                                                               const uint8_t* __restrict__ argmax,
                                                               const void* __restrict__ x, int dtype, int n, int H,
                                                               int W, int C, int kh, int kw, FastDiv dW, FastDiv dH,
                                                               FastDiv dkw, FastDiv dkh,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ dgamma,
                                                               const float* __restrict__ dbeta, void* dx,
                                                               float* __restrict__ partial) {
  const int OH = H / kh, OW = W / kw, G = C / 8;
  const int t = threadIdx.x;
  const int cg = t % G, rs = t / G, rslots = NT / G;
  const int P = n * H * W;
  float mu[8], is[8], a[8], mb[8], mg[8];
  const float invP = 1.f / (float)P;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i;
    mu[i] = mean[c]; is[i] = invstd[c];
    a[i] = (gamma ? gamma[c] : 1.f) * is[i];
    mb[i] = dbeta[c] * invP;
    mg[i] = dgamma[c] * invP;
  }
  float s1[8] = {0};
  const int stride = gridDim.x * rslots;
  for (int r0 = blockIdx.x * rslots + rs; r0 < P; r0 += PB_UNROLL * stride) {
    float xv[PB_UNROLL][8];
    uint2 am[PB_UNROLL];
    float4 g0[PB_UNROLL], g1[PB_UNROLL];
#pragma unroll
    for (int u = 0; u < PB_UNROLL; ++u) {
      const int r = min(r0 + u * stride, P - 1);
      load8(x, dtype, (int64_t)r * C + cg * 8, xv[u]);
      const int q = (int)fdiv(r, dW), ix = r - q * W;
      const int b = (int)fdiv(q, dH), iy = q - b * H;
      const int oy = min((int)fdiv(iy, dkh), OH - 1), ox = min((int)fdiv(ix, dkw), OW - 1);
      const int64_t coff = (((int64_t)b * OH + oy) * OW + ox) * C + cg * 8;
      am[u] = *reinterpret_cast<const uint2*>(argmax + coff);
      g0[u] = reinterpret_cast<const float4*>(gm + coff)[0];
      g1[u] = reinterpret_cast<const float4*>(gm + coff)[1];
    }
#pragma unroll
    for (int u = 0; u < PB_UNROLL; ++u) {
      const int r = r0 + u * stride;
      if (r >= P) break;
      const int q = (int)fdiv(r, dW), ix = r - q * W;
      const int iy = q - (int)fdiv(q, dH) * H;
      const int oy = (int)fdiv(iy, dkh), ox = (int)fdiv(ix, dkw);
      const int pos = oy < OH && ox < OW ? (iy - oy * kh) * kw + (ix - ox * kw) : -1;
      const float gv[8] = {g0[u].x, g0[u].y, g0[u].z, g0[u].w, g1[u].x, g1[u].y, g1[u].z, g1[u].w};
      float g[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t word = i < 4 ? am[u].x : am[u].y;
        const int av = (int)((word >> (8 * (i & 3))) & 0xffu);
        const float gi = av == pos ? gv[i] : 0.f;
        g[i] = a[i] * (gi - mb[i] - (xv[u][i] - mu[i]) * is[i] * mg[i]);
        s1[i] += g[i];
      }
      store8(dx, dtype, (int64_t)r * C + cg * 8, g);
    }
  }
  if (!partial) return;
  __shared__ float red[NT * 8];
#pragma unroll
  for (int i = 0; i < 8; ++i) red[t * 8 + i] = s1[i];
  __syncthreads();
  for (int c = t; c < C; c += NT) {
    const int g2 = c / 8, ci = c % 8;
    float acc = 0.f;
    for (int r2 = 0; r2 < rslots; ++r2) acc += red[(r2 * G + g2) * 8 + ci];
    partial[((int64_t)blockIdx.x * C + c) * 2] = acc;
  }
}

__global__ void partial_final_kernel(const float* __restrict__ partial, int nblk, int C, float* dgamma, float* dbeta) {
  const int c = blockIdx.x;  // one block per channel
  const double a = block_sum_strided(partial + (int64_t)c * 2, nblk, (int64_t)C * 2);
  const double b = block_sum_strided(partial + (int64_t)c * 2 + 1, nblk, (int64_t)C * 2);
  if (threadIdx.x != 0) return;
  if (dbeta) dbeta[c] = (float)a;
  if (dgamma) dgamma[c] = (float)b;
}

// out[b][ih][iw] = sum_ky p[b][ih-ky][iw][ky]
__global__ void col2im_rows_kernel(const float* __restrict__ p, int n, int ph, int w, int kh, void* out, int dtype) {
  const int H = ph + kh - 1;
  const int total = n * H * w;  // < 2^31 (checked by the launcher)
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int iw = idx % w;
    const int q = idx / w;
    const int ih = q % H;
    const int b = q / H;
    float s = 0.f;
    for (int ky = 0; ky < kh; ++ky) {
      const int r = ih - ky;
      if (r >= 0 && r < ph) s += p[(((int64_t)b * ph + r) * w + iw) * kh + ky];
    }
    st_elem(out, dtype, idx, s);
  }
}

}  // namespace

extern "C" int mia_pool_fwd(const void* x, int32_t dtype, int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh,
                            int32_t kw, const float* scale, const float* shift, void* out, int32_t out_layout,
                            uint8_t* argmax, void* win, mia_stream_t stream) {
  MIA_CHECK_ARG(x && out && argmax, "pool_fwd: null pointer");
  MIA_CHECK_ARG(!win || (reinterpret_cast<uintptr_t>(win) & 15) == 0, "pool_fwd: win alignment");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(x) | (out_layout == 0 ? reinterpret_cast<uintptr_t>(out) : 0)) & 15) == 0,
                "pool_fwd: x (and an NHWC out) must be 16-byte aligned");
  MIA_CHECK_ARG(c % 8 == 0 && kh > 0 && kw > 0 && kh * kw <= 256 && h >= kh && w >= kw, "pool_fwd: bad geometry");
  MIA_CHECK_ARG(out_layout >= 0 && out_layout <= 2 && (out_layout != 1 || h / kh == 1), "pool_fwd: bad layout");
  MIA_CHECK_ARG((int64_t)n * h * w * (c / 8) < (1ll << 31), "pool_fwd: too many elements for 32-bit indexing");
  const int64_t total = (int64_t)n * (h / kh) * (w / kw) * (c / 8);
  const int nb = (int)std::min<int64_t>(cdiv(total, NT), 16384);
  pool_fwd_kernel<<<nb, NT, 0, as_stream(stream)>>>(x, dtype, n, h, w, c, kh, kw, scale, shift, out, out_layout, argmax,
                                                    win);
  MIA_LAUNCH_CHECK("pool_fwd");
  return 0;
}

extern "C" int mia_pool_raw_stats(const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh, int32_t kw,
                                  const float* gamma, const float* kshift, void* win, uint8_t* argmax, float* partial,
                                  int32_t nblocks, mia_stream_t stream) {
  MIA_CHECK_ARG(x && gamma && kshift && win && argmax && partial && nblocks > 0, "pool_raw_stats: null pointer");
  MIA_CHECK_ARG(c % 8 == 0 && c >= 8 && c * 2 <= NT && (NT % (c / 8)) == 0, "pool_raw_stats: channels");
  MIA_CHECK_ARG(h % kh == 0 && w >= kw && kh * kw <= 256, "pool_raw_stats: window geometry");
  MIA_CHECK_ARG((int64_t)n * h * w * (c / 8) < (1ll << 31), "pool_raw_stats: too many elements for 32-bit indexing");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(win)) % 16 == 0 &&
                reinterpret_cast<uintptr_t>(argmax) % 8 == 0, "pool_raw_stats: alignment");
  pool_raw_stats_kernel<<<nblocks, NT, 0, as_stream(stream)>>>(reinterpret_cast<const bf16*>(x), n, h, w, c, kh, kw,
                                                               gamma, kshift, reinterpret_cast<bf16*>(win), argmax,
                                                               partial);
  MIA_LAUNCH_CHECK("pool_raw_stats");
  return 0;
}

extern "C" int mia_pool_apply(const void* win, int32_t n, int32_t oh, int32_t ow, int32_t c, const float* scale,
                              const float* shift, void* out, int32_t dtype, int32_t out_layout, mia_stream_t stream) {
  MIA_CHECK_ARG(win && scale && shift && out && n > 0 && oh > 0 && ow > 0 && c > 0, "pool_apply: bad arguments");
  if (out_layout == 1 && oh == 1 && c == 64 && dtype == MIA_BF16 && (reinterpret_cast<uintptr_t>(win) & 15) == 0 &&
      (int64_t)n * cdiv(ow, 64) < (1ll << 31)) {
    pool_apply_t64_kernel<<<(unsigned)(n * cdiv(ow, 64)), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const bf16*>(win), ow, scale, shift, reinterpret_cast<bf16*>(out));
    MIA_LAUNCH_CHECK("pool_apply_t64");
    return 0;
  }
  const int64_t total = (int64_t)n * oh * ow * c;
  const int nb = (int)std::min<int64_t>(cdiv(total, NT), 16384);
  pool_apply_kernel<<<nb, NT, 0, as_stream(stream)>>>(reinterpret_cast<const bf16*>(win), n, oh, ow, c, scale, shift,
                                                      out, dtype, out_layout);
  MIA_LAUNCH_CHECK("pool_apply");
  return 0;
}

extern "C" int mia_pool_bwd_bn_relu_reduce(const void* dout, int32_t out_layout, const uint8_t* argmax, const void* x,
                                           int32_t dtype, int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh,
                                           int32_t kw, const float* scale, const float* shift, const float* mean,
                                           const float* invstd, void* dz, float* dgamma, float* dbeta, void* partial,
                                           mia_stream_t stream) {
  MIA_CHECK_ARG(dout && argmax && x && scale && shift && mean && invstd && dz && dgamma && dbeta && partial,
                "pool_bwd: null pointer");
  MIA_CHECK_ARG(c % 8 == 0 && c >= 8 && (NT % (c / 8)) == 0, "pool_bwd: channels");
  MIA_CHECK_ARG((int64_t)n * h * w < (1ll << 31), "pool_bwd: too many pixels for 32-bit indexing");
  const int rslots = NT / (c / 8);
  const int64_t P = (int64_t)n * h * w;
  hipStream_t s = as_stream(stream);
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(P, (int64_t)rslots * 8), 1024));
  pool_bwd_kernel<<<nb, NT, 0, s>>>(dout, out_layout, argmax, x, dtype, n, h, w, c, kh, kw, scale, shift, mean,
                                    invstd, dz, (float*)partial);
  MIA_LAUNCH_CHECK("pool_bwd");
  partial_final_kernel<<<(unsigned)c, 256, 0, s>>>((const float*)partial, nb, c, dgamma, dbeta);
  MIA_LAUNCH_CHECK("pool_bwd_final");
  return 0;
}

extern "C" int mia_pool_bwd_gather(const void* dout, int32_t out_layout, const uint8_t* argmax, const void* x,
                                   const void* win, int32_t dtype, int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh, int32_t kw,
                                   const float* scale, const float* shift, const float* mean, const float* invstd,
                                   float* gm, float* dgamma, float* dbeta, void* partial, mia_stream_t stream) {
  MIA_CHECK_ARG(dout && argmax && x && scale && shift && mean && invstd && gm && dgamma && dbeta && partial,
                "pool_bwd_gather: null pointer");
  MIA_CHECK_ARG(c % 8 == 0 && c >= 8 && (NT % (c / 8)) == 0, "pool_bwd_gather: channels");
  MIA_CHECK_ARG((int64_t)n * h * w < (1ll << 31), "pool_bwd_gather: too many pixels for 32-bit indexing");
  MIA_CHECK_ARG(h >= kh && w >= kw && kh * kw <= 256 && (reinterpret_cast<uintptr_t>(gm) & 15) == 0,
                "pool_bwd_gather: bad geometry / alignment");
  const int rslots = NT / (c / 8);
  const int64_t cells = (int64_t)n * (h / kh) * (w / kw);
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(cells, (int64_t)rslots * 2), 1024));
  hipStream_t s = as_stream(stream);
  MIA_CHECK_ARG(!win || (reinterpret_cast<uintptr_t>(win) & 15) == 0, "pool_bwd_gather: win alignment");
  pool_bwd_sparse_kernel<<<nb, NT, 0, s>>>(dout, out_layout, argmax, x, win, dtype, n, h, w, c, kh, kw, scale, shift, mean,
                                           invstd, gm, (float*)partial);
  MIA_LAUNCH_CHECK("pool_bwd_gather");
  partial_final_kernel<<<(unsigned)c, 256, 0, s>>>((const float*)partial, nb, c, dgamma, dbeta);
  MIA_LAUNCH_CHECK("pool_bwd_gather_final");
  return 0;
}

extern "C" int mia_pool_bn_relu_bwd_apply(const float* gm, const uint8_t* argmax, const void* x, int32_t dtype,
                                          int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh, int32_t kw,
                                          const float* gamma, const float* mean, const float* invstd,
                                          const float* dgamma, const float* dbeta, void* dx, float* dbias,
                                          void* partial, mia_stream_t stream) {
  MIA_CHECK_ARG(gm && argmax && x && mean && invstd && dgamma && dbeta && dx, "pool_bn_bwd_apply: null pointer");
  MIA_CHECK_ARG(!dbias || partial, "pool_bn_bwd_apply: dbias needs the partial workspace");
  MIA_CHECK_ARG(c % 8 == 0 && c >= 8 && (NT % (c / 8)) == 0, "pool_bn_bwd_apply: channels");
  MIA_CHECK_ARG((int64_t)n * h * w < (1ll << 31), "pool_bn_bwd_apply: too many pixels for 32-bit indexing");
  MIA_CHECK_ARG(h >= kh && w >= kw && kh * kw <= 256, "pool_bn_bwd_apply: bad geometry");
  const int rslots = NT / (c / 8);
  const int64_t P = (int64_t)n * h * w;
  hipStream_t s = as_stream(stream);
  const int64_t units = (int64_t)n * h * ((w + 7) / 8) * (c / 8);
  if (kw % 8 == 0 && dtype == MIA_BF16 && units < (1ll << 31) &&
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dx)) & 15) == 0) {
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(units, NT), 1024));  // partial slab: <= 1024 blocks
    pool_bn_bwd_apply_oct_kernel<<<nb, NT, 0, s>>>(gm, argmax, reinterpret_cast<const bf16*>(x), n, h, w, c, kh, kw,
                                                   make_fastdiv((w + 7) / 8), make_fastdiv(h), make_fastdiv(c / 8),
                                                   gamma, mean, invstd, dgamma, dbeta, reinterpret_cast<bf16*>(dx),
                                                   dbias ? (float*)partial : nullptr);
    MIA_LAUNCH_CHECK("pool_bn_bwd_apply");
    if (dbias) {
      partial_final_kernel<<<(unsigned)c, 256, 0, s>>>((const float*)partial, nb, c, nullptr, dbias);
      MIA_LAUNCH_CHECK("pool_bn_bwd_apply_final");
    }
    return 0;
  }
  const int64_t runs = (int64_t)n * h * cdiv(w, kw) * (c / 8);
  static const bool per_pixel = getenv("MIA_POOL_BWD_PIXEL") != nullptr;  // A/B switch: the per-pixel form
  if (kw >= 2 && kw <= 4 && dtype == MIA_BF16 && runs < (1ll << 31) && !per_pixel &&
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dx)) & 15) == 0) {
    constexpr int RU = PB_RUNS;
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(runs, (int64_t)NT * RU), PB_NB));
    const FastDiv dNR = make_fastdiv((int)cdiv(w, kw)), dH = make_fastdiv(h), dG = make_fastdiv(c / 8);
    float* part = dbias ? (float*)partial : nullptr;
    const bf16* xb = reinterpret_cast<const bf16*>(x);
    bf16* dxb = reinterpret_cast<bf16*>(dx);
    if (kw == 2)
      pool_bn_bwd_apply_run_kernel<2, RU><<<nb, NT, 0, s>>>(gm, argmax, xb, n, h, w, c, kh, dNR, dH, dG, gamma, mean,
                                                            invstd, dgamma, dbeta, dxb, part);
    else if (kw == 3)
      pool_bn_bwd_apply_run_kernel<3, RU><<<nb, NT, 0, s>>>(gm, argmax, xb, n, h, w, c, kh, dNR, dH, dG, gamma, mean,
                                                            invstd, dgamma, dbeta, dxb, part);
    else
      pool_bn_bwd_apply_run_kernel<4, RU><<<nb, NT, 0, s>>>(gm, argmax, xb, n, h, w, c, kh, dNR, dH, dG, gamma, mean,
                                                            invstd, dgamma, dbeta, dxb, part);
    MIA_LAUNCH_CHECK("pool_bn_bwd_apply_run");
    if (dbias) {
      partial_final_kernel<<<(unsigned)c, 256, 0, s>>>((const float*)partial, nb, c, nullptr, dbias);
      MIA_LAUNCH_CHECK("pool_bn_bwd_apply_final");
    }
    return 0;
  }
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(P, (int64_t)rslots * 8), 1024));
  pool_bn_bwd_apply_kernel<<<nb, NT, 0, s>>>(gm, argmax, x, dtype, n, h, w, c, kh, kw, make_fastdiv(w), make_fastdiv(h),
                                             make_fastdiv(kw), make_fastdiv(kh), gamma, mean, invstd, dgamma,
                                             dbeta, dx, dbias ? (float*)partial : nullptr);
  MIA_LAUNCH_CHECK("pool_bn_bwd_apply");
  if (dbias) {
    partial_final_kernel<<<(unsigned)c, 256, 0, s>>>((const float*)partial, nb, c, nullptr, dbias);
    MIA_LAUNCH_CHECK("pool_bn_bwd_apply_final");
  }
  return 0;
}

extern "C" int mia_col2im_rows(const float* p, int32_t n, int32_t ph, int32_t w, int32_t kh, void* out, int32_t dtype,
                               mia_stream_t stream) {
  MIA_CHECK_ARG(p && out && n > 0 && ph > 0 && w > 0 && kh > 0, "col2im_rows: bad arguments");
  MIA_CHECK_ARG((int64_t)n * (ph + kh - 1) * w < (1ll << 31), "col2im_rows: too many elements");
  const int64_t total = (int64_t)n * (ph + kh - 1) * w;
  const int nb = (int)std::min<int64_t>(cdiv(total, 256), 16384);
  col2im_rows_kernel<<<nb, 256, 0, as_stream(stream)>>>(p, n, ph, w, kh, out, dtype);
  MIA_LAUNCH_CHECK("col2im_rows");
  return 0;
}
