// BatchNorm2d (train-mode batch statistics) forward/backward and LayerNorm for gfx950.
//
// BN runs over channels-last (P, C) activations (P = N*H*W).  Every pass reads 16 B per lane
// (8 channels of one pixel) and reduces per channel in two deterministic stages:
// per-block partial sums in LDS -> f32 [nblk][C][2] slab -> one finalize kernel in double.
// The BN *apply* never takes its own pass in the forward: the consumer GEMM applies
// scale/shift (+ReLU) while staging its operand (MIA_PRE_AFFINE_RELU), and the pool kernel does
// the same for the pooled layers.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int MAXBLK = 1024;

// Reduce per-thread channel partials s1[8], s2[8] (thread owns channel group cg, row slot rs)
// across row slots through LDS, then write the block's [C][2] partial.
__device__ __forceinline__ void block_channel_reduce(float (&s1)[8], float (&s2)[8], int C, float* partial) {
  __shared__ float red[NT * 16];
  const int t = threadIdx.x;
  const int G = C / 8;
  const int rslots = NT / G;
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[t * 16 + i] = s1[i]; red[t * 16 + 8 + i] = s2[i]; }
  __syncthreads();
  // entry e < 2C sums quantity q=(e/C) of channel c=(e%C) over the row slots
  for (int e = t; e < 2 * C; e += NT) {
    const int q = e / C, c = e % C, cg = c / 8, ci = c % 8;
    float acc = 0.f;
    for (int r = 0; r < rslots; ++r) acc += red[(r * G + cg) * 16 + q * 8 + ci];
    partial[((int64_t)blockIdx.x * C + c) * 2 + q] = acc;
  }
}

// ---- BN forward statistics: shifted sums about K[c] = x[0][c]
__global__ __launch_bounds__(NT) void bn_stats_kernel(const void* __restrict__ x, int dtype, int64_t P, int C,
                                                      float* __restrict__ partial) {
  const int t = threadIdx.x;
  const int G = C / 8, cg = t % G, rs = t / G, rslots = NT / G;
  float K[8];
  load8(x, dtype, (int64_t)cg * 8, K);
  float s1[8] = {0}, s2[8] = {0};
  for (int64_t r = (int64_t)blockIdx.x * rslots + rs; r < P; r += (int64_t)gridDim.x * rslots) {
    float f[8];
    load8(x, dtype, r * C + cg * 8, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = f[i] - K[i];
      s1[i] += d;
      s2[i] = fmaf(d, d, s2[i]);
    }
  }
  block_channel_reduce(s1, s2, C, partial);
}

__global__ void bn_finalize_kernel(const void* __restrict__ x, int dtype, const float* __restrict__ partial,
                                   int nblk, int64_t P, int C, const float* gamma, const float* beta,
                                   float* running_mean, float* running_var, float momentum, float eps,
                                   float* mean_o, float* invstd_o, float* scale_o, float* shift_o,
                                   const float* __restrict__ kshift = nullptr) {
  const int c = blockIdx.x;  // one block per channel
  const double s1 = block_sum_strided(partial + (int64_t)c * 2, nblk, (int64_t)C * 2);
  const double s2 = block_sum_strided(partial + (int64_t)c * 2 + 1, nblk, (int64_t)C * 2);
  if (threadIdx.x != 0) return;
  const double n = (double)P;
  const double K = kshift ? (double)kshift[c] : (double)ld_elem(x, dtype, c);
  const double dm = s1 / n;
  const double mean = K + dm;
  double var = s2 / n - dm * dm;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_o[c] = (float)mean;
  invstd_o[c] = invstd;
  const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
  scale_o[c] = g * invstd;
  shift_o[c] = bb - (float)mean * g * invstd;
  if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
  if (running_var) {
    const double unb = P > 1 ? var * n / (n - 1.0) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
}

__global__ void bn_eval_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                               float eps, float* mean_o, float* invstd_o, float* scale_o, float* shift_o) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, bb = beta ? beta[c] : 0.f;
  mean_o[c] = rm[c];
  invstd_o[c] = invstd;
  scale_o[c] = g * invstd;
  shift_o[c] = bb - rm[c] * g * invstd;
}

// ---- ReLU+BN backward reductions
__global__ __launch_bounds__(NT) void bn_relu_bwd_reduce_kernel(const void* __restrict__ dact, void* dz,
                                                                const void* __restrict__ x, int dtype, int64_t P,
                                                                int C, const float* __restrict__ scale,
                                                                const float* __restrict__ shift,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                float* __restrict__ partial) {
  const int t = threadIdx.x;
  const int G = C / 8, cg = t % G, rs = t / G, rslots = NT / G;
  float sc[8], sh[8], mu[8], is[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[cg * 8 + i]; sh[i] = shift[cg * 8 + i]; mu[i] = mean[cg * 8 + i]; is[i] = invstd[cg * 8 + i];
  }
  float s1[8] = {0}, s2[8] = {0};
  for (int64_t r = (int64_t)blockIdx.x * rslots + rs; r < P; r += (int64_t)gridDim.x * rslots) {
    float g[8], xv[8];
    const int64_t off = r * C + cg * 8;
    load8(dact, dtype, off, g);
    load8(x, dtype, off, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float z = fmaf(xv[i], sc[i], sh[i]);
      g[i] = z > 0.f ? g[i] : 0.f;
      s1[i] += g[i];
      s2[i] = fmaf(g[i], (xv[i] - mu[i]) * is[i], s2[i]);
    }
    if (dz) store8(dz, dtype, off, g);
  }
  block_channel_reduce(s1, s2, C, partial);
}

// partial [nblk][C][2] -> out0[c] = sum q0, out1[c] = sum q1
__global__ void channel_partial_sum_kernel(const float* __restrict__ partial, int nblk, int C,
                                           float* out_q1, float* out_q0) {
  const int c = blockIdx.x;  // one block per channel
  const double a = block_sum_strided(partial + (int64_t)c * 2, nblk, (int64_t)C * 2);
  const double b = block_sum_strided(partial + (int64_t)c * 2 + 1, nblk, (int64_t)C * 2);
  if (threadIdx.x != 0) return;
  if (out_q0) out_q0[c] = (float)a;
  if (out_q1) out_q1[c] = (float)b;
}

// MASK: dz is the gradient of relu(bn(x)) and the ReLU mask is recomputed from x (scale/shift),
// so the reduce pass never has to write the masked gradient out.
template <bool MASK>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(const void* __restrict__ dz, const void* __restrict__ x,
                                                          void* dx, int dtype, int64_t P, int C,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ dgamma,
                                                          const float* __restrict__ dbeta,
                                                          float* __restrict__ partial,
                                                          const float* __restrict__ scale = nullptr,
                                                          const float* __restrict__ shift = nullptr) {
  const int t = threadIdx.x;
  const int G = C / 8, cg = t % G, rs = t / G, rslots = NT / G;
  float a[8], mu[8], is[8], mb[8], mg[8], sc[8], sh[8];
  if constexpr (MASK) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { sc[i] = scale[cg * 8 + i]; sh[i] = shift[cg * 8 + i]; }
  }
  float s1[8] = {0}, s2[8] = {0};
  const float invP = 1.f / (float)P;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = cg * 8 + i;
    is[i] = invstd[c];
    a[i] = (gamma ? gamma[c] : 1.f) * is[i];
    mu[i] = mean[c];
    mb[i] = dbeta[c] * invP;
    mg[i] = dgamma[c] * invP;
  }
  for (int64_t r = (int64_t)blockIdx.x * rslots + rs; r < P; r += (int64_t)gridDim.x * rslots) {
    float g[8], xv[8];
    const int64_t off = r * C + cg * 8;
    load8(dz, dtype, off, g);
    load8(x, dtype, off, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (MASK) g[i] = fmaf(xv[i], sc[i], sh[i]) > 0.f ? g[i] : 0.f;
      g[i] = a[i] * (g[i] - mb[i] - (xv[i] - mu[i]) * is[i] * mg[i]);
      s1[i] += g[i];
    }
    store8(dx, dtype, off, g);
  }
  if (partial) block_channel_reduce(s1, s2, C, partial);
}

// ---- generic column sum over a (P, C) matrix with row stride ld (any C, scalar loads)
__global__ __launch_bounds__(NT) void colsum_kernel(const void* __restrict__ x, int dtype, int64_t P, int C,
                                                    int64_t ld, float* __restrict__ partial) {
  const int c = blockIdx.y * NT + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int64_t r = blockIdx.x; r < P; r += gridDim.x) s += ld_elem(x, dtype, r * ld + c);
  partial[(int64_t)blockIdx.x * C + c] = s;
}
// vectorised column sum (C % 8 == 0, 16-B aligned rows): thread = 8 columns x a row slot
__global__ __launch_bounds__(NT) void colsum8_kernel(const void* __restrict__ x, int dtype, int64_t P, int C, int64_t ld,
                                                     float* __restrict__ partial) {
  __shared__ float red[NT * 8];
  const int t = threadIdx.x;
  const int G = C / 8, Gb = G < NT ? G : NT, rslots = NT / Gb;
  const int cg = blockIdx.y * NT + t % Gb, rs = t / Gb;
  float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rs < rslots && cg < G) {
    for (int64_t r = (int64_t)blockIdx.x * rslots + rs; r < P; r += (int64_t)gridDim.x * rslots) {
      float f[8];
      load8(x, dtype, r * ld + cg * 8, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) s8[i] += f[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[t * 8 + i] = s8[i];
  __syncthreads();
  for (int e = t; e < Gb * 8; e += NT) {
    const int g = e / 8, i = e % 8;
    float acc = 0.f;
    for (int r2 = 0; r2 < rslots; ++r2) acc += red[(r2 * Gb + g) * 8 + i];
    const int c = (blockIdx.y * NT + g) * 8 + i;
    if (c < C) partial[(int64_t)blockIdx.x * C + c] = acc;
  }
}

__global__ void colsum_final_kernel(const float* __restrict__ partial, int nblk, int C, float* out) {
  const int c = blockIdx.x;  // one block per column
  const double s = block_sum_strided(partial + c, nblk, C);
  if (threadIdx.x == 0) out[c] = (float)s;
}

int nblocks_for(int64_t P, int C) {
  const int rslots = NT / (C / 8);
  int64_t nb = cdiv(P, (int64_t)rslots * 8);
  if (nb > MAXBLK) nb = MAXBLK;
  if (nb < 1) nb = 1;
  return (int)nb;
}

int check_bn(const void* x, int dtype, int64_t P, int C) {
  MIA_CHECK_ARG(x != nullptr, "bn: null input");
  MIA_CHECK_ARG(dtype == MIA_F32 || dtype == MIA_BF16, "bn: dtype");
  MIA_CHECK_ARG(C % 8 == 0 && C >= 8 && C <= 2048 && (NT % (C / 8)) == 0,
                "bn: C must be a multiple of 8 dividing 2048 (got %d)", C);
  MIA_CHECK_ARG(P > 0, "bn: empty input");
  return 0;
}

// ---------------------------------------------------------------- LayerNorm (rows x D), one wave per row
// MX (fp8-mixed): the bf16 output row is also written as OCP MX-fp8 (e4m3 bytes q [rows][D], E8M0
// scales [rows][D / 32]) -- the qkv / fc1 MX GEMM's A operand without a quantisation pass.  Lane l holds
// d = l + 64 i, so lanes 0-31 / 32-63 hold 32-blocks 2i / 2i + 1: the block amax is a 32-lane max.
template <int PER, bool MX = false>
__global__ __launch_bounds__(NT) void ln_fwd_kernel(const void* __restrict__ x, int xdt, const float* __restrict__ g,
                                                    const float* __restrict__ b, void* y, int ydt,
                                                    float* __restrict__ mean_o, float* __restrict__ rstd_o,
                                                    int64_t rows, int D, float eps, uint8_t* __restrict__ q = nullptr,
                                                    uint8_t* __restrict__ qs = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int d = lane + 64 * i;
    v[i] = d < D ? ld_elem(x, xdt, row * D + d) : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int d = lane + 64 * i;
    const float dd = d < D ? v[i] - mean : 0.f;
    ss = fmaf(dd, dd, ss);
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int d = lane + 64 * i;
    if constexpr (MX) {  // D % 64 == 0 (d < D is wave-uniform), bf16 output: quantise the stored value
      if (64 * i >= D) break;
      const float yb = (float)(bf16)((v[i] - mean) * rstd * g[d] + b[d]);
      reinterpret_cast<bf16*>(y)[row * D + d] = (bf16)yb;
      float am = fabsf(yb);
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
      const int e = mx_exponent(am);
      const float t = __builtin_amdgcn_fmed3f(__builtin_amdgcn_ldexpf(yb, -e), -448.f, 448.f);
      q[row * D + d] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(t, 0.f, 0, false) & 0xff);
      if ((lane & 31) == 0) qs[row * (D >> 5) + (d >> 5)] = (uint8_t)(e + 127);
    } else {
      if (d < D) st_elem(y, ydt, row * D + d, (v[i] - mean) * rstd * g[d] + b[d]);
    }
  }
  if (lane == 0) { mean_o[row] = mean; rstd_o[row] = rstd; }
}

// The same LayerNorm for D a multiple of 256 (AST: 768), vectorised: lane l holds the G groups of 4
// consecutive elements d = 4l + 256i, so every load is 16 B (f32) / 8 B (bf16) per lane and every store
// 8 B (bf16) / 16 B (f32) / 4 B (MX bytes): a quarter of the per-element form's memory instructions.
// MX: a 32-block is 8 lanes, its amax a 3-step shuffle; lane 8k writes the block's scale byte.
template <int G, bool MX = false>
__global__ __launch_bounds__(NT) void ln_fwd_vec_kernel(const void* __restrict__ x, int xdt, const float* __restrict__ g,
                                                        const float* __restrict__ b, void* y, int ydt,
                                                        float* __restrict__ mean_o, float* __restrict__ rstd_o,
                                                        int64_t rows, int D, float eps, uint8_t* __restrict__ q = nullptr,
                                                        uint8_t* __restrict__ qs = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[G][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int64_t e = row * D + 4 * lane + 256 * i;
    if (xdt == MIA_F32) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(x) + e);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] = a[k];
    } else {
      const bf16x4 a = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(x) + e);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] = (float)a[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s += v[i][k];
  }
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float dd = v[i][k] - mean;
      ss = fmaf(dd, dd, ss);
    }
  const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int d0 = 4 * lane + 256 * i;
    const int64_t e = row * D + d0;
    const f32x4 gg = *reinterpret_cast<const f32x4*>(g + d0), bb = *reinterpret_cast<const f32x4*>(b + d0);
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (v[i][k] - mean) * rstd * gg[k] + bb[k];
    if (MX || ydt == MIA_BF16) {
      const bf16x4 ob = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(y) + e) = ob;
      if constexpr (MX) {  // quantise the stored (bf16) values
        float am = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) { o[k] = (float)ob[k]; am = fmaxf(am, fabsf(o[k])); }
#pragma unroll
        for (int m = 1; m < 8; m <<= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
        const int ex = mx_exponent(am);
        float tq[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) tq[k] = __builtin_amdgcn_fmed3f(__builtin_amdgcn_ldexpf(o[k], -ex), -448.f, 448.f);
        const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(tq[0], tq[1], 0, false);
        const int w = __builtin_amdgcn_cvt_pk_fp8_f32(tq[2], tq[3], lo, true);
        *reinterpret_cast<uint32_t*>(q + e) = (uint32_t)w;
        if ((lane & 7) == 0) qs[row * (D >> 5) + (d0 >> 5)] = (uint8_t)(ex + 127);
      }
    } else {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(y) + e) = f32x4{o[0], o[1], o[2], o[3]};
    }
  }
  if (lane == 0) { mean_o[row] = mean; rstd_o[row] = rstd; }
}

template <int PER>
__global__ __launch_bounds__(NT) void ln_bwd_kernel(const void* __restrict__ dy, int dydt, const void* __restrict__ x,
                                                    int xdt, const float* __restrict__ g,
                                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                                    void* dx, int dxdt, int accumulate, float* __restrict__ partial,
                                                    int64_t rows, int D, int rows_per_block) {
  // partial layout: [gridDim.x][2][D] (dgamma, dbeta): each wave's sums staged in LDS, added in wave order
  // (fixed order: an LDS atomicAdd of the four waves' sums made dgamma / dbeta differ from run to run)
  __shared__ float pw[NT / 64][2][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ag[PER], ab[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) { ag[i] = 0.f; ab[i] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  for (int64_t row = r0 + wave; row < r0 + rows_per_block && row < rows; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[PER], gy[PER];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int d = lane + 64 * i;
      if (d < D) {
        const float dv = ld_elem(dy, dydt, row * D + d);
        xh[i] = (ld_elem(x, xdt, row * D + d) - mu) * rs;
        gy[i] = dv * g[d];
        ag[i] = fmaf(dv, xh[i], ag[i]);
        ab[i] += dv;
      } else {
        xh[i] = 0.f; gy[i] = 0.f;
      }
      s1 += gy[i];
      s2 = fmaf(gy[i], xh[i], s2);
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int d = lane + 64 * i;
      if (d < D) {
        float v = rs * (gy[i] - s1 - xh[i] * s2);
        const int64_t idx = row * D + d;
        if (accumulate) v += ld_elem(dx, dxdt, idx);
        st_elem(dx, dxdt, idx, v);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int d = lane + 64 * i;
    if (d < D) { pw[wave][0][d] = ag[i]; pw[wave][1][d] = ab[i]; }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * D; i += NT) {
    const int q = i / D, d = i % D;
    float a = pw[0][q][d];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) a += pw[w][q][d];
    partial[(int64_t)blockIdx.x * 2 * D + i] = a;
  }
}

// Vectorised LayerNorm backward for D = 64*PER (PER % 4 == 0): lane owns PER contiguous features
// (16-B / 8-B accesses), one wave per row, LN_VEC_ROWS rows per block; dgamma/dbeta partials are
// summed per lane in registers, then across the 4 waves through LDS (fixed order, no atomics).
constexpr int LN_VEC_ROWS = 64;

// lane l holds the PER / 4 groups of 4 consecutive elements d = 4l + 256i (D = 64 * PER, a multiple of
// 256): every load / store instruction of the wave covers one contiguous 1 KB (f32) / 512 B (bf16) run
template <int PER>
__device__ __forceinline__ void ldv4(const void* p, int dt, int64_t rowoff, int lane, float* f) {
#pragma unroll
  for (int q = 0; q < PER / 4; ++q) {
    const int64_t off = rowoff + 4 * lane + 256 * q;
    if (dt == MIA_BF16) {
      const bf16x4 v = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(p) + off);
#pragma unroll
      for (int k = 0; k < 4; ++k) f[4 * q + k] = (float)v[k];
    } else {
      const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + off);
      f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
    }
  }
}
template <int PER>
__device__ __forceinline__ void stv4(void* p, int dt, int64_t rowoff, int lane, const float* f) {
#pragma unroll
  for (int q = 0; q < PER / 4; ++q) {
    const int64_t off = rowoff + 4 * lane + 256 * q;
    if (dt == MIA_BF16) {
      const bf16x4 v = {(bf16)f[4 * q], (bf16)f[4 * q + 1], (bf16)f[4 * q + 2], (bf16)f[4 * q + 3]};
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p) + off) = v;
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + off) =
          make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
    }
  }
}

// MX (fp8-mixed backward): the bf16 dx2 row is also written as OCP MX-fp8 (q [rows][D], scales [rows][D / 32],
// of the stored bf16 values, as ln_fwd_vec_kernel<MX>) -- the A operand of the next MX backward-data GEMM.
template <int PER, bool CS, bool MX = false>
__global__ __launch_bounds__(NT) void ln_bwd_vec_kernel(const void* __restrict__ dy, int dydt, const void* __restrict__ x,
                                                        int xdt, const float* __restrict__ g,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        void* dx, int dxdt, int accumulate, void* dx2, int dx2dt,
                                                        float* __restrict__ partial, int64_t rows,
                                                        uint8_t* __restrict__ mq = nullptr,
                                                        uint8_t* __restrict__ ms = nullptr) {
  // CS: also the column sums of the stored dx2 values (the next linear's bias gradient); partial
  // rows are then [blk][3][D] instead of [blk][2][D] (and the LDS plane for them exists only then)
  constexpr int D = 64 * PER;
  static_assert(D % 256 == 0, "ln_bwd_vec: D must be a multiple of 256");
  constexpr int nq = CS ? 3 : 2;
  __shared__ float red[4][nq][D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gg[PER];
  ldv4<PER>(g, MIA_F32, 0, lane, gg);
  float ag[PER], ab[PER], ac[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) { ag[i] = 0.f; ab[i] = 0.f; ac[i] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * LN_VEC_ROWS;
  for (int64_t row = r0 + wave; row < r0 + LN_VEC_ROWS && row < rows; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float dv[PER], xh[PER];
    ldv4<PER>(dy, dydt, row * D, lane, dv);
    ldv4<PER>(x, xdt, row * D, lane, xh);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      xh[i] = (xh[i] - mu) * rs;
      ag[i] = fmaf(dv[i], xh[i], ag[i]);
      ab[i] += dv[i];
      dv[i] *= gg[i];
      s1 += dv[i];
      s2 = fmaf(dv[i], xh[i], s2);
    }
    s1 = wave_sum(s1) * (1.f / (float)D);
    s2 = wave_sum(s2) * (1.f / (float)D);
    float o[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) o[i] = rs * (dv[i] - s1 - xh[i] * s2);
    if (accumulate) {
      float old[PER];
      ldv4<PER>(dx, dxdt, row * D, lane, old);
#pragma unroll
      for (int i = 0; i < PER; ++i) o[i] += old[i];
    }
    stv4<PER>(dx, dxdt, row * D, lane, o);
    if (dx2) stv4<PER>(dx2, dx2dt, row * D, lane, o);
    if constexpr (MX) {  // dx2 is bf16 here: quantise the stored values, a 32-block = 8 lanes
#pragma unroll
      for (int q4 = 0; q4 < PER / 4; ++q4) {
        float w[4], am = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) { w[k] = (float)(bf16)o[4 * q4 + k]; am = fmaxf(am, fabsf(w[k])); }
#pragma unroll
        for (int m = 1; m < 8; m <<= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
        const int ex = mx_exponent(am);
        float tq[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) tq[k] = __builtin_amdgcn_fmed3f(__builtin_amdgcn_ldexpf(w[k], -ex), -448.f, 448.f);
        const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(tq[0], tq[1], 0, false);
        const int wd = __builtin_amdgcn_cvt_pk_fp8_f32(tq[2], tq[3], lo, true);
        const int d0 = 4 * lane + 256 * q4;
        *reinterpret_cast<uint32_t*>(mq + row * D + d0) = (uint32_t)wd;
        if ((lane & 7) == 0) ms[row * (D >> 5) + (d0 >> 5)] = (uint8_t)(ex + 127);
      }
    }
    if constexpr (CS) {
#pragma unroll
      for (int i = 0; i < PER; ++i) ac[i] += dx2dt == MIA_BF16 ? (float)(bf16)o[i] : o[i];
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int d = 4 * lane + 256 * (i >> 2) + (i & 3);
    red[wave][0][d] = ag[i];
    red[wave][1][d] = ab[i];
    if constexpr (CS) red[wave][nq - 1][d] = ac[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nq * D; i += NT) {
    const int q = i / D, d = i % D;
    partial[(int64_t)blockIdx.x * nq * D + i] = ((red[0][q][d] + red[1][q][d]) + red[2][q][d]) + red[3][q][d];
  }
}

// partial rows [blk][nq][D] -> (colsum_pass1) slice sums [COLSUM_SLICES][nq * D] -> dgamma, dbeta
// (and, nq == 3, the dx2 column sums), in double; one thread per (q, d)
__global__ void ln_partial_final_kernel(const double* __restrict__ part2, int D, int nq, float* dgamma,
                                        float* dbeta, float* colsum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq * D) return;
  const int q = i / D, d = i - q * D;
  const float v = (float)colsum_slices(part2, nq * D, i);
  float* dst = q == 0 ? dgamma : q == 1 ? dbeta : colsum;
  if (dst) dst[d] = v;
}

constexpr int LN_ROWS_PER_BLOCK = 256;

}  // namespace

extern "C" int64_t mia_bn_partial_bytes(int64_t P, int32_t C) {
  if (C < 8 || C % 8) return 0;
  return (int64_t)MAXBLK * C * 2 * 4;
}

extern "C" int mia_bn_fwd_stats(const void* x, int32_t dtype, int64_t P, int32_t C, const float* gamma,
                                const float* beta, float* running_mean, float* running_var, float momentum,
                                float eps, int32_t training, float* mean, float* invstd, float* scale,
                                float* shift, void* partial, mia_stream_t stream) {
  MIA_CHECK_ARG(mean && invstd && scale && shift, "bn_fwd_stats: null output");
  hipStream_t s = as_stream(stream);
  if (!training) {
    MIA_CHECK_ARG(running_mean && running_var, "bn_fwd_stats: eval needs running stats");
    bn_eval_kernel<<<(unsigned)cdiv(C, 256), 256, 0, s>>>(C, gamma, beta, running_mean, running_var, eps, mean, invstd,
                                                          scale, shift);
    MIA_LAUNCH_CHECK("bn_eval");
    return 0;
  }
  if (int r = check_bn(x, dtype, P, C)) return r;
  MIA_CHECK_ARG(partial != nullptr, "bn_fwd_stats: null partial workspace");
  const int nb = nblocks_for(P, C);
  bn_stats_kernel<<<nb, NT, 0, s>>>(x, dtype, P, C, (float*)partial);
  MIA_LAUNCH_CHECK("bn_stats");
  bn_finalize_kernel<<<(unsigned)C, 256, 0, s>>>(x, dtype, (const float*)partial, nb, P, C, gamma, beta,
                                                            running_mean, running_var, momentum, eps, mean, invstd,
                                                            scale, shift);
  MIA_LAUNCH_CHECK("bn_finalize");
  return 0;
}

extern "C" int mia_bn_finalize_shifted(const float* partial, int32_t nblk, int64_t P, int32_t C, const float* kshift,
                                       const float* gamma, const float* beta, float* running_mean,
                                       float* running_var, float momentum, float eps, int32_t training, float* mean,
                                       float* invstd, float* scale, float* shift, mia_stream_t stream) {
  MIA_CHECK_ARG(partial && kshift && mean && invstd && scale && shift && nblk > 0 && P > 0 && C > 0,
                "bn_finalize_shifted: bad arguments");
  MIA_CHECK_ARG(training, "bn_finalize_shifted: batch statistics are a training-mode path");
  bn_finalize_kernel<<<(unsigned)C, 256, 0, as_stream(stream)>>>(nullptr, MIA_F32, partial, nblk, P, C, gamma, beta,
                                                                running_mean, running_var, momentum, eps, mean,
                                                                invstd, scale, shift, kshift);
  MIA_LAUNCH_CHECK("bn_finalize_shifted");
  return 0;
}

extern "C" int mia_bn_relu_bwd_reduce(const void* dact, void* dz, const void* x, int32_t dtype, int64_t P,
                                      int32_t C, const float* scale, const float* shift, const float* mean,
                                      const float* invstd, float* dgamma, float* dbeta, void* partial,
                                      mia_stream_t stream) {
  if (int r = check_bn(x, dtype, P, C)) return r;
  MIA_CHECK_ARG(dact && scale && shift && mean && invstd && dgamma && dbeta && partial,
                "bn_relu_bwd_reduce: null pointer");
  hipStream_t s = as_stream(stream);
  const int nb = nblocks_for(P, C);
  bn_relu_bwd_reduce_kernel<<<nb, NT, 0, s>>>(dact, dz, x, dtype, P, C, scale, shift, mean, invstd, (float*)partial);
  MIA_LAUNCH_CHECK("bn_relu_bwd_reduce");
  channel_partial_sum_kernel<<<(unsigned)C, 256, 0, s>>>((const float*)partial, nb, C, dgamma, dbeta);
  MIA_LAUNCH_CHECK("channel_partial_sum");
  return 0;
}

extern "C" int mia_bn_bwd_apply(const void* dz, const void* x, void* dx, int32_t dtype, int64_t P, int32_t C,
                                const float* gamma, const float* mean, const float* invstd, const float* dgamma,
                                const float* dbeta, float* dbias, void* partial, mia_stream_t stream) {
  if (int r = check_bn(x, dtype, P, C)) return r;
  MIA_CHECK_ARG(dz && dx && mean && invstd && dgamma && dbeta, "bn_bwd_apply: null pointer");
  MIA_CHECK_ARG(!dbias || partial, "bn_bwd_apply: dbias needs the partial workspace");
  const int nb = nblocks_for(P, C);
  hipStream_t s = as_stream(stream);
  bn_bwd_apply_kernel<false><<<nb, NT, 0, s>>>(dz, x, dx, dtype, P, C, gamma, mean, invstd, dgamma, dbeta,
                                               dbias ? (float*)partial : nullptr);
  MIA_LAUNCH_CHECK("bn_bwd_apply");
  if (dbias) {
    channel_partial_sum_kernel<<<(unsigned)C, 256, 0, s>>>((const float*)partial, nb, C, nullptr, dbias);
    MIA_LAUNCH_CHECK("channel_partial_sum");
  }
  return 0;
}

extern "C" int mia_bn_relu_bwd_apply(const void* dact, const void* x, void* dx, int32_t dtype, int64_t P, int32_t C,
                                     const float* gamma, const float* scale, const float* shift, const float* mean,
                                     const float* invstd, const float* dgamma, const float* dbeta, float* dbias,
                                     void* partial, mia_stream_t stream) {
  if (int r = check_bn(x, dtype, P, C)) return r;
  MIA_CHECK_ARG(dact && dx && scale && shift && mean && invstd && dgamma && dbeta, "bn_relu_bwd_apply: null pointer");
  MIA_CHECK_ARG(!dbias || partial, "bn_relu_bwd_apply: dbias needs the partial workspace");
  const int nb = nblocks_for(P, C);
  hipStream_t s = as_stream(stream);
  bn_bwd_apply_kernel<true><<<nb, NT, 0, s>>>(dact, x, dx, dtype, P, C, gamma, mean, invstd, dgamma, dbeta,
                                              dbias ? (float*)partial : nullptr, scale, shift);
  MIA_LAUNCH_CHECK("bn_relu_bwd_apply");
  if (dbias) {
    channel_partial_sum_kernel<<<(unsigned)C, 256, 0, s>>>((const float*)partial, nb, C, nullptr, dbias);
    MIA_LAUNCH_CHECK("channel_partial_sum");
  }
  return 0;
}

extern "C" int mia_colsum(const void* x, int32_t dtype, int64_t P, int32_t C, int64_t ld, float* out, void* partial,
                          mia_stream_t stream) {
  MIA_CHECK_ARG(x && out && partial && C > 0 && P > 0 && ld >= C, "colsum: bad arguments");
  int nb = (int)std::min<int64_t>(cdiv(P, 64), MIA_COLSUM_MAXBLK);  // workspace: MIA_COLSUM_MAXBLK * C floats
  hipStream_t s = as_stream(stream);
  const int es = dtype == MIA_BF16 ? 2 : 4;
  if (C % 8 == 0 && ld % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (int64_t)es * 8 >= 16) {
    colsum8_kernel<<<dim3(nb, (unsigned)cdiv(C / 8, NT)), NT, 0, s>>>(x, dtype, P, C, ld, (float*)partial);
  } else {
    colsum_kernel<<<dim3(nb, (unsigned)cdiv(C, NT)), NT, 0, s>>>(x, dtype, P, C, ld, (float*)partial);
  }
  MIA_LAUNCH_CHECK("colsum");
  colsum_final_kernel<<<(unsigned)C, 256, 0, s>>>((const float*)partial, nb, C, out);
  MIA_LAUNCH_CHECK("colsum_final");
  return 0;
}

extern "C" int mia_layernorm_fwd(const void* x, int32_t xdtype, const float* gamma, const float* beta, void* y,
                                 int32_t ydtype, float* mean, float* rstd, int64_t rows, int32_t D, float eps,
                                 mia_stream_t stream) {
  MIA_CHECK_ARG(x && gamma && beta && y && mean && rstd, "layernorm_fwd: null pointer");
  MIA_CHECK_ARG(D > 0 && D <= 1024, "layernorm_fwd: D must be <= 1024");
  const unsigned nb = (unsigned)cdiv(rows, 4);
  hipStream_t s = as_stream(stream);
  const bool vec = D % 256 == 0 && (xdtype == MIA_F32 || xdtype == MIA_BF16) && (ydtype == MIA_F32 || ydtype == MIA_BF16) &&
                   ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(gamma) |
                     reinterpret_cast<uintptr_t>(beta)) & 15) == 0;
  if (vec && D == 768) ln_fwd_vec_kernel<3><<<nb, NT, 0, s>>>(x, xdtype, gamma, beta, y, ydtype, mean, rstd, rows, D, eps);
  else if (vec && D == 512) ln_fwd_vec_kernel<2><<<nb, NT, 0, s>>>(x, xdtype, gamma, beta, y, ydtype, mean, rstd, rows, D, eps);
  else if (vec && D == 256) ln_fwd_vec_kernel<1><<<nb, NT, 0, s>>>(x, xdtype, gamma, beta, y, ydtype, mean, rstd, rows, D, eps);
  else if (vec && D == 1024) ln_fwd_vec_kernel<4><<<nb, NT, 0, s>>>(x, xdtype, gamma, beta, y, ydtype, mean, rstd, rows, D, eps);
  else if (D <= 768) ln_fwd_kernel<12><<<nb, NT, 0, s>>>(x, xdtype, gamma, beta, y, ydtype, mean, rstd, rows, D, eps);
  else ln_fwd_kernel<16><<<nb, NT, 0, s>>>(x, xdtype, gamma, beta, y, ydtype, mean, rstd, rows, D, eps);
  MIA_LAUNCH_CHECK("layernorm_fwd");
  return 0;
}

extern "C" int mia_layernorm_fwd_mx(const void* x, int32_t xdtype, const float* gamma, const float* beta, void* y,
                                    void* q, void* scales, float* mean, float* rstd, int64_t rows, int32_t D, float eps,
                                    mia_stream_t stream) {
  MIA_CHECK_ARG(x && gamma && beta && y && q && scales && mean && rstd, "layernorm_fwd_mx: null pointer");
  MIA_CHECK_ARG(D > 0 && D <= 768 && D % 64 == 0, "layernorm_fwd_mx: D must be a multiple of 64, <= 768");
  const unsigned nb = (unsigned)cdiv(rows, 4);
  const bool vec = D == 768 && (xdtype == MIA_F32 || xdtype == MIA_BF16) &&
                   ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(gamma) |
                     reinterpret_cast<uintptr_t>(beta) | reinterpret_cast<uintptr_t>(q)) & 15) == 0;
  if (vec)
    ln_fwd_vec_kernel<3, true><<<nb, NT, 0, as_stream(stream)>>>(x, xdtype, gamma, beta, y, MIA_BF16, mean, rstd, rows, D,
                                                                 eps, reinterpret_cast<uint8_t*>(q),
                                                                 reinterpret_cast<uint8_t*>(scales));
  else
    ln_fwd_kernel<12, true><<<nb, NT, 0, as_stream(stream)>>>(x, xdtype, gamma, beta, y, MIA_BF16, mean, rstd, rows, D, eps,
                                                               reinterpret_cast<uint8_t*>(q), reinterpret_cast<uint8_t*>(scales));
  MIA_LAUNCH_CHECK("layernorm_fwd_mx");
  return 0;
}

// partial rows of the widest form, then (256-B aligned) the slice sums of colsum_pass1
static int64_t ln_rows_bytes(int64_t rows, int32_t D) {
  const int64_t a = cdiv(rows, LN_VEC_ROWS) * 3 * D * 4, b = cdiv(rows, 256) * 2 * D * 4;
  return cdiv(a > b ? a : b, 256) * 256;
}
extern "C" int64_t mia_layernorm_partial_bytes(int64_t rows, int32_t D) {
  return ln_rows_bytes(rows, D) + colsum_part2_bytes(3 * D);
}

static int layernorm_bwd_impl(const void* dy, int32_t dydtype, const void* x, int32_t xdtype, const float* gamma,
                              const float* mean, const float* rstd, void* dx, int32_t dxdtype, int32_t accumulate,
                              void* dx2, int32_t dx2dtype, float* dgamma, float* dbeta, float* dx2_colsum,
                              void* partial, int64_t rows, int32_t D, mia_stream_t stream, void* mq = nullptr,
                              void* ms = nullptr) {
  MIA_CHECK_ARG(dy && x && gamma && mean && rstd && dx && partial, "layernorm_bwd: null pointer");
  MIA_CHECK_ARG(!dx2_colsum || dx2, "layernorm_bwd: the column sums are of dx2");
  MIA_CHECK_ARG(D > 0 && D <= 1024, "layernorm_bwd: D must be <= 1024");
  hipStream_t s = as_stream(stream);
  unsigned nb;
  const bool al = ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dx) |
                    reinterpret_cast<uintptr_t>(dx2) | reinterpret_cast<uintptr_t>(gamma)) & 15) == 0;
  if (D == 768 && al) {
    nb = (unsigned)cdiv(rows, LN_VEC_ROWS);
    if (mq)
      ln_bwd_vec_kernel<12, true, true><<<nb, NT, 0, s>>>(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype,
                                                          accumulate, dx2, dx2dtype, (float*)partial, rows,
                                                          (uint8_t*)mq, (uint8_t*)ms);
    else if (dx2_colsum)
      ln_bwd_vec_kernel<12, true><<<nb, NT, 0, s>>>(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype, accumulate,
                                                    dx2, dx2dtype, (float*)partial, rows);
    else
      ln_bwd_vec_kernel<12, false><<<nb, NT, 0, s>>>(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype,
                                                     accumulate, dx2, dx2dtype, (float*)partial, rows);
  } else {
    MIA_CHECK_ARG(dx2 == nullptr, "layernorm_bwd: the bf16 copy needs D == 768 and aligned rows");
    MIA_CHECK_ARG(mq == nullptr, "layernorm_bwd: the MX copy needs D == 768 and aligned rows");
    nb = (unsigned)cdiv(rows, LN_ROWS_PER_BLOCK);
    if (D <= 768)
      ln_bwd_kernel<12><<<nb, NT, 0, s>>>(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype, accumulate,
                                          (float*)partial, rows, D, LN_ROWS_PER_BLOCK);
    else
      ln_bwd_kernel<16><<<nb, NT, 0, s>>>(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype, accumulate,
                                          (float*)partial, rows, D, LN_ROWS_PER_BLOCK);
  }
  MIA_LAUNCH_CHECK("layernorm_bwd");
  const int nq = dx2_colsum ? 3 : 2;
  double* part2 = reinterpret_cast<double*>(static_cast<char*>(partial) + ln_rows_bytes(rows, D));
  colsum_pass1((const float*)partial, (int64_t)nb, nq * D, (int64_t)nq * D, part2, s);
  ln_partial_final_kernel<<<(unsigned)cdiv(nq * D, 256), 256, 0, s>>>(part2, D, nq, dgamma, dbeta, dx2_colsum);
  MIA_LAUNCH_CHECK("layernorm_partial_final");
  return 0;
}

extern "C" int mia_layernorm_bwd(const void* dy, int32_t dydtype, const void* x, int32_t xdtype, const float* gamma,
                                 const float* mean, const float* rstd, void* dx, int32_t dxdtype, int32_t accumulate,
                                 void* dx2, int32_t dx2dtype, float* dgamma, float* dbeta, void* partial, int64_t rows,
                                 int32_t D, mia_stream_t stream) {
  return layernorm_bwd_impl(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype, accumulate, dx2, dx2dtype, dgamma,
                            dbeta, nullptr, partial, rows, D, stream);
}

extern "C" int mia_layernorm_bwd_colsum_mx(const void* dy, int32_t dydtype, const void* x, int32_t xdtype,
                                           const float* gamma, const float* mean, const float* rstd, void* dx,
                                           int32_t dxdtype, int32_t accumulate, void* dx2, float* dgamma,
                                           float* dbeta, float* dx2_colsum, void* q, void* scales, void* partial,
                                           int64_t rows, int32_t D, mia_stream_t stream) {
  MIA_CHECK_ARG(dx2_colsum && dx2 && q && scales && D == 768, "layernorm_bwd_colsum_mx: needs dx2 (bf16), its column "
                "sums, the MX q / scales and D == 768");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(q) & 3) == 0, "layernorm_bwd_colsum_mx: q must be 4-B aligned");
  return layernorm_bwd_impl(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype, accumulate, dx2, MIA_BF16, dgamma,
                            dbeta, dx2_colsum, partial, rows, D, stream, q, scales);
}

extern "C" int mia_layernorm_bwd_colsum(const void* dy, int32_t dydtype, const void* x, int32_t xdtype,
                                        const float* gamma, const float* mean, const float* rstd, void* dx,
                                        int32_t dxdtype, int32_t accumulate, void* dx2, int32_t dx2dtype,
                                        float* dgamma, float* dbeta, float* dx2_colsum, void* partial, int64_t rows,
                                        int32_t D, mia_stream_t stream) {
  MIA_CHECK_ARG(dx2_colsum && dx2 && D == 768, "layernorm_bwd_colsum: needs dx2, dx2_colsum and D == 768");
  return layernorm_bwd_impl(dy, dydtype, x, xdtype, gamma, mean, rstd, dx, dxdtype, accumulate, dx2, dx2dtype, dgamma,
                            dbeta, dx2_colsum, partial, rows, D, stream);
}
