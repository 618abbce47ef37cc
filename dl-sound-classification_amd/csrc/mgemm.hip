// Dense bf16 GEMM for the AST block linears (timm Block qkv / proj / fc1 / fc2, reference
// src/models/ast.py:38,60-61): forward (x W^T), backward-data (dy W) and weight gradient (dy^T x)
// with their epilogues fused -- bias, exact-erf GELU (+ the pre-activation saved for the backward),
// the f32 residual add, gelu'(u) applied to the fc2 backward-data output together with the column
// sums of what it stores (fc1's bias gradient), and deterministic split-K slabs for the weight
// gradients.  Hand-written for gfx950; no vendor library, no run-time tuning, no host sync.
//
// * one 512-thread workgroup (8 waves, 2 per SIMD) per CU owns a 256 x 256 output tile; wave w keeps
//   the 128 x 64 sub-tile (rows 128 * (w >> 2), columns 64 * (w & 3)) in 32 accumulators of
//   v_mfma_f32_16x16x32_bf16 (128 VGPRs), computed TRANSPOSED (C^T = B^T A^T) so each lane holds four
//   consecutive columns of one row: f32 outputs are stored as 16 B per lane straight from the
//   accumulators; bf16 outputs are rounded (as autocast rounds a Linear's output before the GELU /
//   its backward), staged through LDS and stored as 16-B pieces of whole 128-B rows (a wave's
//   128 x 64 bf16 image is 16 KB: the eight fill the two operand stages);
// * operand tiles travel HBM/L2 -> LDS by buffer-load LDS-DMA (16 B per lane, 1 KB per wave
//   instruction) into two 64 KB stages; rows/k-rows outside the operand read as zeros (descriptor
//   range), the XOR swizzle rides the per-lane SOURCE offset so every fragment read is conflict-free
//   (ds_read_b128 for k-contiguous operands, ds_read_b64_tr_b16 for k-by-m operands);
// * each K-tile is two phases of 32 MFMAs; waves 4-7 run one barrier behind waves 0-3, so on every
//   SIMD one wave issues its MFMAs while its partner reads its fragments and issues the next
//   LDS-DMA (MI355X_MICROARCH.md, "Two waves per SIMD"); every LDS-DMA is retired by a counted
//   vmcnt one phase after its issue and read one barrier later;
#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int MG_NT = 512;
constexpr int MG_BM = 256, MG_BN = 256, MG_BK = 64;
constexpr int MG_HALF = 16384;                 // bytes of one half-tile (128 x 64 bf16)
constexpr int MG_STAGE = 4 * MG_HALF;          // A0 A1 B0 B1
constexpr int MG_LDS = 2 * MG_STAGE;

enum { MG_KC = MIA_LAYOUT_KC, MG_RC = MIA_LAYOUT_RC };
enum { EPI_PLAIN = 0, EPI_GELU = 1, EPI_GELU_SAVE = 2, EPI_ADD_AUX = 3, EPI_DGELU = 4, EPI_SLAB = 5, EPI_GELU_SAVE_D = 6,
       EPI_DMUL = 7 };

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_vp;

struct MArgs {
  const bf16* a;
  const bf16* b;
  int64_t lda, ldb, M, N, K, kper;
  int nbm, nbn, split;
  void* out;
  int64_t ldc;
  int out_f32;
  const float* bias;
  const void* aux;
  int64_t ldaux;
  float* ws;          // EPI_SLAB: [split][M][N] f32
  float* colsum_part; // EPI_DGELU with colsum: [nbm][N] f32
  float* acs_part;    // A-operand column sums (RC A only): [split][M] f32, written by the bn == 0 tiles
  uint8_t* mxq;       // optional MX-fp8 copy of a bf16 output: e4m3 [M][N] (row stride N) ...
  uint8_t* mxs;       // ... and its scales [M][N / 32]
  int64_t drop_w;     // EPI_PLAIN with a drop-mode row map (MIA_RM_DROP): row m -> m - m / drop_w, rows with
                      // m % drop_w == drop_w - 1 not stored (0: off)
  int group_m;        // tile order (mg_tile_of): 0 = column block fastest, > 0 = groups of group_m row blocks
};

typedef unsigned mg_u32x4 __attribute__((ext_vector_type(4)));
// The bf16 epilogue's 16-B stores (8 lanes = one whole 128-B line), non-temporal: the outputs (0.65-2.6 GB
// at the AST shapes) are far larger than the Infinity Cache.  A/B at B = 256 (tools/gemm_ab.sh): qkv.fwd
// 1.635 -> 1.57 ms, fc1.fwd (GELU_SAVE) 2.765 -> 2.60 ms, fc2.dgrad 3.11 -> 3.08 ms; AST step +1 %.  (The
// f32 residual outputs leave the accumulators as 64-B halves of lines: non-temporal partial lines are
// twice as slow, they stay default-policy.)
__device__ __forceinline__ void mg_st16(void* p, uint4 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(mg_u32x4, v), reinterpret_cast<mg_u32x4*>(p));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, int64_t bytes) {
  const uint32_t n = bytes <= 0 ? 0u : (bytes >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)n, 0x00020000);
}

// 32-byte chunk swizzle of the k-by-m images (RC): the 8 k-rows one 32-lane half of a transposed
// fragment read touches ({k0..k0+3} and {k0+8..k0+11}) land on 8 different chunks
__device__ __forceinline__ int rc_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// One operand (A or B) of the tile: its buffer descriptor, the four per-lane source offsets of this
// wave's DMA instructions (2 per half-tile) and the byte step per K-tile.
template <int L>
struct Loader {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff[4];
  uint32_t kstep;
  // KC: rows [r0, r0 + 256) of a row-major [rows][K] operand, k from kbeg; RC: k-rows [kbeg, kend)
  // of a row-major [K][cols] operand, columns [r0, r0 + 256)
  __device__ __forceinline__ void init(const bf16* p, int64_t ld, int64_t rows, int64_t r0, int64_t kbeg,
                                       int64_t kend, int wave, int lane) {
    if constexpr (L == MG_KC) {
      const bf16* base = p + r0 * ld + kbeg;
      const int64_t nrows = rows - r0 < 256 ? rows - r0 : 256;
      rsrc = rsrc_of(base, ((nrows - 1) * ld + (kend - kbeg)) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hh = i >> 1, j = 2 * wave + (i & 1);
        const int r = hh * 128 + 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        voff[i] = (uint32_t)(((int64_t)r * ld + c * 8) * 2);
      }
      kstep = 128;
    } else {
      const bf16* base = p + kbeg * ld + r0;
      const int64_t ncols = rows - r0 < 256 ? rows - r0 : 256;
      rsrc = rsrc_of(base, ((kend - kbeg - 1) * ld + ncols) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hh = i >> 1, j = 2 * wave + (i & 1);
        const int k = 4 * j + (lane >> 4);
        const int s = lane & 15;
        const int c = (s >> 1) ^ rc_swz(k);
        voff[i] = (uint32_t)(((int64_t)k * ld + hh * 128 + c * 16 + (s & 1) * 8) * 2);
      }
      kstep = (uint32_t)(64 * ld * 2);
    }
  }
  // both half-tiles of K-tile kt into the stage at `tile` (this wave's 4 instructions)
  __device__ __forceinline__ void issue(char* tile, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_vp)(tile + (i >> 1) * MG_HALF + (2 * wave + (i & 1)) * 1024),
                                               16, voff[i], kt * kstep, 0, 0);
  }
};

// fragment of 16 rows (KC: operand rows; RC: operand columns) at `r0` inside a half-tile image, k-step ks
template <int L>
__device__ __forceinline__ bf16x8 frag(const char* half, int r0, int ks, int lane) {
  if constexpr (L == MG_KC) {
    const int r = r0 + (lane & 15);
    const int c = 4 * ks + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(half + r * 128 + ((c ^ (r & 7)) << 4));
  } else {
    const int i = lane & 15, g = lane >> 4;
    const int k = 32 * ks + 8 * g + (i >> 2);
    const int ch = r0 >> 4;
    const char* p0 = half + k * 256 + ((ch ^ rc_swz(k)) << 5) + (i & 3) * 8;
    const char* p1 = half + (k + 4) * 256 + ((ch ^ rc_swz(k + 4)) << 5) + (i & 3) * 8;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p1));
    const s16x8 cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, cc);
  }
}

// transposed product: lane (l & 15) = row of C, 4 (l >> 4) + r = its columns
__device__ __forceinline__ f32x4 mfma_t(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, 0, 0, 0);
}

// Exact-erf GELU and its derivative at bf16 output precision: Phi(x) = 0.5 erfc(-x / sqrt 2) with
// erfc from the Numerical Recipes rational-exponential form (fractional error < 1.2e-7 for every
// argument: one reciprocal, one exp, nine FMAs -- a third of the instructions of libm's erff, which
// dominated the fc1 / fc2-backward epilogues), no cancellation on either side of 0.
__device__ __forceinline__ float gelu_cdf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float half_erfc = 0.5f * t * __expf(fmaf(-z, z, p));  // 0.5 erfc(|x| / sqrt 2)
  return x >= 0.f ? 1.f - half_erfc : half_erfc;
}
__device__ __forceinline__ float gelu_f(float x) { return x * gelu_cdf(x); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return fmaf(x * 0.39894228040143268f, __expf(-0.5f * x * x), gelu_cdf(x));
}

// The same two functions on element pairs for the epilogues, which are VALU-bound: the polynomial and
// the products run as packed f32 (v_pk_fma_f32 / v_pk_mul_f32, two lanes' worth per instruction), log2 e
// is folded into the polynomial so the exponential is a bare v_exp_f32.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
constexpr float L2E = 1.4426950408889634f;
// Phi(x) of a pair and z^2 = x^2 / 2
__device__ __forceinline__ f2 gelu_cdf2(f2 x, f2& zz) {
  const f2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f2 d = pfma(z, f2{0.5f, 0.5f}, f2{1.f, 1.f});
  const f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f2 p = f2{0.17087277f * L2E, 0.17087277f * L2E};
  p = pfma(p, t, f2{-0.82215223f * L2E, -0.82215223f * L2E});
  p = pfma(p, t, f2{1.48851587f * L2E, 1.48851587f * L2E});
  p = pfma(p, t, f2{-1.13520398f * L2E, -1.13520398f * L2E});
  p = pfma(p, t, f2{0.27886807f * L2E, 0.27886807f * L2E});
  p = pfma(p, t, f2{-0.18628806f * L2E, -0.18628806f * L2E});
  p = pfma(p, t, f2{0.09678418f * L2E, 0.09678418f * L2E});
  p = pfma(p, t, f2{0.37409196f * L2E, 0.37409196f * L2E});
  p = pfma(p, t, f2{1.00002368f * L2E, 1.00002368f * L2E});
  p = pfma(p, t, f2{-1.26551223f * L2E, -1.26551223f * L2E});
  zz = z * z;
  const f2 a = pfma(-zz, f2{L2E, L2E}, p);
  const f2 he = t * f2{0.5f * __builtin_amdgcn_exp2f(a.x), 0.5f * __builtin_amdgcn_exp2f(a.y)};
  return f2{x.x >= 0.f ? 1.f - he.x : he.x, x.y >= 0.f ? 1.f - he.y : he.y};
}
__device__ __forceinline__ f2 gelu2(f2 x) {
  f2 zz;
  return x * gelu_cdf2(x, zz);
}
// gelu'(x) = Phi(x) + x phi(x) for the dGELU epilogue, with erfc from Abramowitz-Stegun 7.1.26:
// erfc(z) = t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) exp(-z^2), t = 1 / (1 + p z), |error| <= 1.5e-7
// absolute (gelu'(x) within 5.6e-5 relative wherever |gelu'| > 1e-3: 0.03 bf16 ulp).  Its exp(-z^2), z = |x| / sqrt 2, is
// phi's, so a pair costs one reciprocal and one exp per element (the erfc form above: two exps).
__device__ __forceinline__ f2 gelu_grad2(f2 x) {
  const f2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f2 d = pfma(z, f2{0.3275911f, 0.3275911f}, f2{1.f, 1.f});
  const f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f2 p = f2{0.5f * 1.061405429f, 0.5f * 1.061405429f};
  p = pfma(p, t, f2{0.5f * -1.453152027f, 0.5f * -1.453152027f});
  p = pfma(p, t, f2{0.5f * 1.421413741f, 0.5f * 1.421413741f});
  p = pfma(p, t, f2{0.5f * -0.284496736f, 0.5f * -0.284496736f});
  p = pfma(p, t, f2{0.5f * 0.254829592f, 0.5f * 0.254829592f});
  const f2 a = -(z * z) * L2E;
  const f2 e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};  // exp(-x^2 / 2)
  const f2 he = p * t * e;                                                  // 0.5 erfc(|x| / sqrt 2)
  const f2 c = {x.x >= 0.f ? 1.f - he.x : he.x, x.y >= 0.f ? 1.f - he.y : he.y};  // Phi(x)
  return pfma(x * 0.39894228040143268f, e, c);
}
// gelu(x) of a pair and, into d, gelu'(x) = Phi(x) + x phi(x), both from gelu_grad2's Abramowitz-Stegun
// erfc, whose exp(-x^2 / 2) is phi's: one reciprocal and one exp per element for the pair of outputs
// (|error| <= 7.5e-8 absolute in Phi: relative to gelu(x) that is < 1e-4 for x > -3.4, where gelu
// has |values| > 1e-3; the erfc form above keeps the tails relative for the GELU-only epilogues)
__device__ __forceinline__ f2 gelu_and_grad2(f2 x, f2& d) {
  const f2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f2 dd = pfma(z, f2{0.3275911f, 0.3275911f}, f2{1.f, 1.f});
  const f2 t = {__builtin_amdgcn_rcpf(dd.x), __builtin_amdgcn_rcpf(dd.y)};
  f2 p = f2{0.5f * 1.061405429f, 0.5f * 1.061405429f};
  p = pfma(p, t, f2{0.5f * -1.453152027f, 0.5f * -1.453152027f});
  p = pfma(p, t, f2{0.5f * 1.421413741f, 0.5f * 1.421413741f});
  p = pfma(p, t, f2{0.5f * -0.284496736f, 0.5f * -0.284496736f});
  p = pfma(p, t, f2{0.5f * 0.254829592f, 0.5f * 0.254829592f});
  const f2 a = -(z * z) * L2E;
  const f2 e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};  // exp(-x^2 / 2)
  const f2 he = p * t * e;                                                  // 0.5 erfc(|x| / sqrt 2)
  const f2 c = {x.x >= 0.f ? 1.f - he.x : he.x, x.y >= 0.f ? 1.f - he.y : he.y};  // Phi(x)
  d = pfma(x * 0.39894228040143268f, e, c);
  return x * c;
}
// v * gelu'(u) / gelu(v) on 4 values in place
__device__ __forceinline__ void gelu4(f32x4& v) {
  const f2 a = gelu2(f2{v[0], v[1]}), b = gelu2(f2{v[2], v[3]});
  v = f32x4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ void gelu_d4(f32x4& v, f32x4& d) {
  f2 da, db;
  const f2 a = gelu_and_grad2(f2{v[0], v[1]}, da), b = gelu_and_grad2(f2{v[2], v[3]}, db);
  v = f32x4{a.x, a.y, b.x, b.y};
  d = f32x4{da.x, da.y, db.x, db.y};
}
__device__ __forceinline__ void dgelu4(f32x4& v, f32x4 u) {
  const f2 a = gelu_grad2(f2{u[0], u[1]}), b = gelu_grad2(f2{u[2], u[3]});
  v = f32x4{v[0] * a.x, v[1] * a.y, v[2] * b.x, v[3] * b.y};
}

__device__ __forceinline__ uint2 pack4(f32x4 v) {
  return make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
}
__device__ __forceinline__ f32x4 unpack4(uint2 u) {
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

// Epilogue shared by the bf16 and the MX-fp8 kernels: lane holds C[m][n .. n+3] of fragment (i, j):
// m = m0 + 128 wr + 16 i + (lane & 15), n = n0 + 64 wc + 16 j + 4 (lane >> 4).  f32 outputs (residual
// stream, slabs) are stored from the registers (16 B per lane); bf16 outputs are rounded, staged in a
// per-wave [128][64] bf16 image and stored as 16-B pieces of whole 128-B rows, with the aux tensors read
// the same way.
template <int EPI>
__device__ __forceinline__ void mg_epilogue(const MArgs& g, f32x4 (&acc)[8][4], char* smem, int wave, int lane,
                                            int bm, int z, int64_t m0, int64_t n0) {
  const int wr = wave >> 2, wc = wave & 3;
  f32x4 bias4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wc * 64 + 16 * j + 4 * (lane >> 4);
    if (EPI != EPI_SLAB && EPI != EPI_DGELU && EPI != EPI_DMUL && g.bias && n < g.N)
      bias4[j] = *reinterpret_cast<const f32x4*>(g.bias + n);
    else
      bias4[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr bool DG = EPI == EPI_DGELU || EPI == EPI_DMUL;  // backward epilogues (aux read, column sums)
  const bool bf_out = EPI == EPI_GELU || EPI == EPI_GELU_SAVE || EPI == EPI_GELU_SAVE_D || DG ||
                      (EPI == EPI_PLAIN && !g.out_f32);
  if (!bf_out) {
    // ADD_AUX: the residual rows of fragment row i + 2 are requested while row i is added and stored (a
    // rolling three-row window of loads in flight instead of a wait at every fragment)
    f32x4 ax[8][4];
    auto ld_row = [&](int i) __attribute__((always_inline)) {
      const int64_t m = m0 + wr * 128 + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = n0 + wc * 64 + 16 * j + 4 * (lane >> 4);
        ax[i][j] = (m < g.M && n < g.N)
                       ? *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(g.aux) + m * g.ldaux + n)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };
    if constexpr (EPI == EPI_ADD_AUX) {
      ld_row(0);
      ld_row(1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (EPI == EPI_ADD_AUX) {
        if (i + 2 < 8) ld_row(i + 2);
      }
      const int64_t m = m0 + wr * 128 + 16 * i + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = n0 + wc * 64 + 16 * j + 4 * (lane >> 4);
        if (n >= g.N) continue;
        f32x4 v = acc[i][j] + bias4[j];
        if constexpr (EPI == EPI_ADD_AUX) v += ax[i][j];
        float* dst = EPI == EPI_SLAB ? g.ws + ((int64_t)z * g.M + m) * g.N + n
                                     : reinterpret_cast<float*>(g.out) + m * g.ldc + n;
        *reinterpret_cast<f32x4*>(dst) = v;
      }
    }
    return;
  }
  if constexpr (EPI != EPI_SLAB && EPI != EPI_ADD_AUX) {
    // all waves are past their last fragment read and every DMA has landed (vmcnt(0) in the last
    // step): the ring is free.  Image row r, 16-B chunk c at chunk c ^ (r & 7) ^ ((r >> 3) & 1):
    // conflict-free 8-B writes (16 rows of one column group) and 16-B row reads.
    __syncthreads();
    char* img = smem + wave * 16384;
    // the backward epilogues' aux rows (saved gelu'(u) / u) requested before the image pass, so their
    // latency runs under it instead of under the store loop (fc2.dgrad 1.99 -> 1.73 ms at B = 256,
    // tools/gemm_epi_ab.sh, gpurun_out r5o / r5p); non-temporal: read once, kept out of the operands' L2
    // (fc2.dgrad DMUL 2.44 -> 2.41 ms, r6nt; the f32 residual reads of ADD_AUX measured 2-3 % slower that way)
    uint4 ua[16];
    if constexpr (DG) {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int r = 8 * it + (lane >> 3);
        const int64_t m = m0 + wr * 128 + r, n = n0 + wc * 64 + 8 * (lane & 7);
        ua[it] = (m < g.M && n < g.N)
                     ? __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const mg_u32x4*>(
                           reinterpret_cast<const bf16*>(g.aux) + m * g.ldaux + n)))
                     : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * i + (lane & 15), g4 = lane >> 4;
        const int c = 2 * j + (g4 >> 1);
        *reinterpret_cast<uint2*>(img + r * 128 + ((c ^ (r & 7) ^ ((r >> 3) & 1)) << 4) + (g4 & 1) * 8) =
            pack4(acc[i][j] + bias4[j]);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    float cs[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) cs[c] = 0.f;
    const int cc = lane & 7;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int r = 8 * it + (lane >> 3);
      const uint4 q = *reinterpret_cast<const uint4*>(img + r * 128 + ((cc ^ (r & 7) ^ ((r >> 3) & 1)) << 4));
      const int64_t m = m0 + wr * 128 + r, n = n0 + wc * 64 + 8 * cc;
      const bool ok = m < g.M && n < g.N;  // no early exit: the MX block exponent is a 4-lane exchange
      uint4 o = q;
      if constexpr (EPI == EPI_GELU_SAVE) {
        if (ok) mg_st16(reinterpret_cast<bf16*>(const_cast<void*>(g.aux)) + m * g.ldaux + n, q);
      }
      if constexpr (EPI == EPI_GELU || EPI == EPI_GELU_SAVE || EPI == EPI_GELU_SAVE_D || DG) {
        f32x4 v0 = unpack4(make_uint2(q.x, q.y)), v1 = unpack4(make_uint2(q.z, q.w));
        if constexpr (DG) {
          const uint4 u = ua[it];
          const f32x4 u0 = unpack4(make_uint2(u.x, u.y)), u1 = unpack4(make_uint2(u.z, u.w));
          if constexpr (EPI == EPI_DGELU) {
            dgelu4(v0, u0);
            dgelu4(v1, u1);
          } else {  // the saved gelu'(u)
            v0 *= u0;
            v1 *= u1;
          }
        } else if constexpr (EPI == EPI_GELU_SAVE_D) {
          f32x4 d0, d1;
          gelu_d4(v0, d0);
          gelu_d4(v1, d1);
          const uint2 e0 = pack4(d0), e1 = pack4(d1);
          if (ok) mg_st16(reinterpret_cast<bf16*>(const_cast<void*>(g.aux)) + m * g.ldaux + n, make_uint4(e0.x, e0.y, e1.x, e1.y));
        } else {
          gelu4(v0);
          gelu4(v1);
        }
        const uint2 p0 = pack4(v0), p1 = pack4(v1);
        o = make_uint4(p0.x, p0.y, p1.x, p1.y);
        if constexpr (DG) {
          if (ok) {
            const f32x4 w0 = unpack4(p0), w1 = unpack4(p1);
#pragma unroll
            for (int k = 0; k < 4; ++k) { cs[k] += w0[k]; cs[4 + k] += w1[k]; }
          }
        }
      }
      {
        if (g.mxq) {  // MX-fp8 copy of the stored bf16 values (the next MX GEMM's A operand)
          const f32x4 w0 = unpack4(make_uint2(o.x, o.y)), w1 = unpack4(make_uint2(o.z, o.w));
          const float v8[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
          const int e = mx_exponent_4lanes(v8);
          const uint2 p = mx_pack8(v8, e);
          if (ok) {
            *reinterpret_cast<uint2*>(g.mxq + m * g.N + n) = p;
            if ((cc & 3) == 0) g.mxs[m * (g.N >> 5) + (n >> 5)] = (uint8_t)(e + 127);
          }
        }
      }
      if constexpr (EPI == EPI_PLAIN) {
        if (g.drop_w) {
          const int64_t x = m % g.drop_w;
          if (ok && x != g.drop_w - 1) mg_st16(reinterpret_cast<bf16*>(g.out) + (m - m / g.drop_w) * g.ldc + n, o);
          continue;
        }
      }
      if (ok) mg_st16(reinterpret_cast<bf16*>(g.out) + m * g.ldc + n, o);
    }
    if constexpr (DG) {
      if (g.colsum_part) {
        // column sums of the stored values: lanes with equal (lane & 7) hold the same 8 columns
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float v = cs[c];
          v += __shfl_xor(v, 8, 64);
          v += __shfl_xor(v, 16, 64);
          v += __shfl_xor(v, 32, 64);
          cs[c] = v;
        }
        __syncthreads();  // every wave is done with its image
        float* red = reinterpret_cast<float*>(smem);  // [2 row halves][256 columns]
        if (lane < 8) {
#pragma unroll
          for (int c = 0; c < 8; ++c) red[wr * 256 + wc * 64 + 8 * lane + c] = cs[c];
        }
        __syncthreads();
        if (threadIdx.x < 256) {
          const int64_t n = n0 + threadIdx.x;
          if (n < g.N) g.colsum_part[(int64_t)bm * g.N + n] = red[threadIdx.x] + red[256 + threadIdx.x];
        }
      }
    }
  }
}

// sum of the 8 bf16 of a fragment added to c (v_dot2_f32_bf16 against ones: exact products, f32 adds)
__device__ __forceinline__ float frag_sum(bf16x8 f, float c) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 one2 = {(__bf16)1.f, (__bf16)1.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_fdot2_f32_bf16(bf2{f[2 * j], f[2 * j + 1]}, one2, c, false);
  return c;
}

// ACS (RC A operand, the split-K weight gradients): also the column sums over k of A -- the bias gradient of
// the linear -- from the K-tiles in LDS: wave (wr, wc) sums rows 16 wc .. 16 wc + 15 and 64 + 16 wc .. of its
// 128-row half (the four wc waves read the same A rows), two extra transposed fragment reads per k-step
// Logical tile -> (row block, column block).  Default: column block fastest (a row block of A is read by all its
// column tiles at about the same time, from the XCD's L2).  group_m > 0 (mg_group_m): groups of group_m row
// blocks with the row block fastest inside a group, so the XCD's concurrent tiles share fewer B column blocks
// (gpurun_out r6gm / r6gm2: fc2.dgrad -2.3 %; the N = 768 shapes are 1-4 % slower with it).  Either order runs
// every tile's own K loop unchanged: the output is bit-identical.
__device__ __forceinline__ void mg_tile_of(const MArgs& g, int rem, int& bm, int& bn) {
  if (g.group_m > 0) {
    const int gsz = g.group_m * g.nbn;
    const int grp = rem / gsz, off = rem - grp * gsz;
    const int rows = min(g.group_m, g.nbm - grp * g.group_m);
    bn = off / rows;
    bm = grp * g.group_m + (off - bn * rows);
  } else {
    bm = rem / g.nbn;
    bn = rem - bm * g.nbn;
  }
}

template <int LA, int LB, int EPI, bool ACS = false>
__global__ __launch_bounds__(MG_NT, 2) void mgemm_kernel(MArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[MG_LDS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // XCD-aware tile order: the blocks one XCD runs (b, b + 8, ...) take consecutive logical tiles,
  // N fastest, so a row block of A is read by all its column tiles from that XCD's L2
  const int nwg = (int)gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_z = g.nbm * g.nbn;
  const int z = lid / per_z;
  const int rem = lid - z * per_z;
  int bm, bn;
  mg_tile_of(g, rem, bm, bn);
  const int64_t m0 = (int64_t)bm * MG_BM, n0 = (int64_t)bn * MG_BN;
  const int64_t kbeg = (int64_t)z * g.kper;
  const int64_t kend = kbeg + g.kper < g.K ? kbeg + g.kper : g.K;
  const int nk = kend > kbeg ? (int)((kend - kbeg + 63) >> 6) : 0;

  Loader<LA> la;
  Loader<LB> lb;
  la.init(g.a, g.lda, g.M, m0, kbeg, kend, wave, lane);
  lb.init(g.b, g.ldb, g.N, n0, kbeg, kend, wave, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* const st0 = smem;
  char* const st1 = smem + MG_STAGE;
  // prologue: K-tile 0 (A and B) -> stage 0, K-tile 1's B -> stage 1
  if (nk > 0) {
    la.issue(st0, 0, wave);
    lb.issue(st0 + 2 * MG_HALF, 0, wave);
  }
  if (nk > 1) {
    lb.issue(st1 + 2 * MG_HALF, 1, wave);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  const int bhalf = wc >> 1;  // B half-tile holding this wave's 64 columns, at column 64 * (wc & 1)
  const int bcol = 64 * (wc & 1);
  bf16x8 af[2][4], bfr[2][4];
  float acs0 = 0.f, acs1 = 0.f;  // ACS: this lane's partial column sums (8 k of rows 16 wc + (lane & 15), +64)
  for (int t = 0; t < nk; ++t) {
    const char* cur = (t & 1) ? st1 : st0;
    const char* ah = cur + wr * MG_HALF;  // the wave's 128 rows are A half-tile wr
    const char* bh = cur + (2 + bhalf) * MG_HALF;
    // ---------------- phase 0: rows 0..63 of the wave's 128, all 64 columns
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag<LA>(ah, 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[ks][j] = frag<LB>(bh, bcol + 16 * j, ks, lane);
    }
    if constexpr (ACS) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        acs0 = frag_sum(frag<LA>(ah, 16 * wc, ks, lane), acs0);
        acs1 = frag_sum(frag<LA>(ah, 64 + 16 * wc, ks, lane), acs1);
      }
    }
    if (t + 1 < nk) {  // K-tile t+1's A -> the other stage (its previous contents, K-tile t-1, are read)
      la.issue((t & 1) ? st0 : st1, t + 1, wave);
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_t(af[ks][i], bfr[ks][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---------------- phase 1: rows 64..127, the same B fragments
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = frag<LA>(ah, 64 + 16 * i, ks, lane);
    if (t + 2 < nk) {  // K-tile t+2's B -> this stage (K-tile t's B fragments are all in registers)
      lb.issue(const_cast<char*>(cur) + 2 * MG_HALF, t + 2, wave);
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[4 + i][j] = mfma_t(af[ks][i], bfr[ks][j], acc[4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the two halves
  if constexpr (ACS) {
    // the four lane groups (lane >> 4) hold different k of the same rows: fixed-order butterfly
    acs0 += __shfl_xor(acs0, 16, 64);
    acs0 += __shfl_xor(acs0, 32, 64);
    acs1 += __shfl_xor(acs1, 16, 64);
    acs1 += __shfl_xor(acs1, 32, 64);
    if (bn == 0 && lane < 16) {
      const int64_t m = m0 + wr * 128 + 16 * wc + lane;
      if (m < g.M) g.acs_part[(int64_t)z * g.M + m] = acs0;
      if (m + 64 < g.M) g.acs_part[(int64_t)z * g.M + m + 64] = acs1;
    }
  }
  mg_epilogue<EPI>(g, acc, smem, wave, lane, bm, z, m0, n0);
}

// Every instantiation explicitly: with implicit instantiation from launch_epi, hipcc (ROCm 7.2)
// emitted the host-side launch stub of the first instantiation only (the others stayed undefined
// symbols of the shared library).
template __global__ void mgemm_kernel<0, 0, 0>(MArgs);
template __global__ void mgemm_kernel<0, 0, 1>(MArgs);
template __global__ void mgemm_kernel<0, 0, 2>(MArgs);
template __global__ void mgemm_kernel<0, 0, 3>(MArgs);
template __global__ void mgemm_kernel<0, 0, 4>(MArgs);
template __global__ void mgemm_kernel<0, 0, 5>(MArgs);
template __global__ void mgemm_kernel<0, 1, 0>(MArgs);
template __global__ void mgemm_kernel<0, 1, 1>(MArgs);
template __global__ void mgemm_kernel<0, 1, 2>(MArgs);
template __global__ void mgemm_kernel<0, 1, 3>(MArgs);
template __global__ void mgemm_kernel<0, 1, 4>(MArgs);
template __global__ void mgemm_kernel<0, 1, 5>(MArgs);
template __global__ void mgemm_kernel<1, 0, 0>(MArgs);
template __global__ void mgemm_kernel<1, 0, 1>(MArgs);
template __global__ void mgemm_kernel<1, 0, 2>(MArgs);
template __global__ void mgemm_kernel<1, 0, 3>(MArgs);
template __global__ void mgemm_kernel<1, 0, 4>(MArgs);
template __global__ void mgemm_kernel<1, 0, 5>(MArgs);
template __global__ void mgemm_kernel<1, 1, 0>(MArgs);
template __global__ void mgemm_kernel<1, 1, 1>(MArgs);
template __global__ void mgemm_kernel<1, 1, 2>(MArgs);
template __global__ void mgemm_kernel<1, 1, 3>(MArgs);
template __global__ void mgemm_kernel<1, 1, 4>(MArgs);
template __global__ void mgemm_kernel<1, 1, 5>(MArgs);
template __global__ void mgemm_kernel<1, 1, 5, true>(MArgs);
template __global__ void mgemm_kernel<1, 0, 5, true>(MArgs);
template __global__ void mgemm_kernel<1, 1, 0, true>(MArgs);
template __global__ void mgemm_kernel<1, 0, 0, true>(MArgs);

// ---------------------------------------------------------------- MX-fp8 (OCP e4m3fn, E8M0 per 32 K)
// Forward block linears under trainer.precision=fp8-mixed (north_star config 5; the reference has no fp8
// path).  A [M][K] and B [N][K] are e4m3 bytes, K contiguous, with one E8M0 scale byte per 32 K-elements
// ([rows][K / 32]).  The tile, LDS ring, phase structure and epilogue are the bf16 kernel's: a K-tile is
// 128 e4m3 = 128 B per row (the bf16 kernel's 64 elements), so the loaders move the same bytes, and each
// phase is 16 v_mfma_scale_f32_16x16x128_f8f6f4 (twice the cycles of a 16x16x32 bf16 MFMA for four
// times the K: 2x the bf16 rate).  Operand lane map (tools/probe/mx16_layout.cpp, measured): lane group
// g = lane >> 4 of row (lane & 15) holds k [16g, 16g + 16) and [64 + 16g, 64 + 16g + 16) of the K-tile,
// i.e. 16-B chunks g and 4 + g of the row; the scale of (row, k-block b) comes from lane row + 16 b.
// The per-K-tile scale dwords ([256 rows][4 blocks] for A and for B, 1 KB each) arrive by 4-B-per-lane
// LDS-DMA with the A tile (waves 0-3: A rows 64w.., waves 4-7: B rows), double-buffered after the ring.
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4v __attribute__((ext_vector_type(4)));
constexpr int MX_SC = MG_LDS;  // scale ring: [2 stages][A 1 KB | B 1 KB]

struct MxArgs {
  const uint8_t* sa;  // [M][K / 32]
  const uint8_t* sb;  // [N][K / 32]
};

__device__ __forceinline__ i32x8 mx_frag(const char* half, int r0, int lane) {
  const int r = r0 + (lane & 15), g = lane >> 4;
  const i32x4v lo = *reinterpret_cast<const i32x4v*>(half + r * 128 + ((g ^ (r & 7)) << 4));
  const i32x4v hi = *reinterpret_cast<const i32x4v*>(half + r * 128 + (((4 + g) ^ (r & 7)) << 4));
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ int mx_scale(const char* sbuf, int r0, int lane) {
  return *reinterpret_cast<const uint8_t*>(sbuf + (r0 + (lane & 15)) * 4 + (lane >> 4));
}

template <int EPI>
__global__ __launch_bounds__(MG_NT, 2) void mxgemm_kernel(MArgs g, MxArgs x) {
  __shared__ __attribute__((aligned(1024))) char smem[MG_LDS + 4096];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nwg = (int)gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  int bm, bn;
  mg_tile_of(g, lid, bm, bn);
  const int64_t m0 = (int64_t)bm * MG_BM, n0 = (int64_t)bn * MG_BN;
  const int nk = (int)(g.K >> 7);
  // e4m3 rows seen as bf16 pairs: the bf16 loaders move 128-B K-tiles unchanged
  Loader<MG_KC> la, lb;
  la.init(g.a, g.lda, g.M, m0, 0, g.K >> 1, wave, lane);
  lb.init(g.b, g.ldb, g.N, n0, 0, g.K >> 1, wave, lane);
  // scale DMA: one 4-B-per-lane piece per wave and K-tile (waves 0-3: A rows, 4-7: B rows)
  const int64_t kb32 = g.K >> 5;
  const int srow = 64 * (wave & 3) + lane;
  const uint8_t* sbase = wr == 0 ? x.sa + m0 * kb32 : x.sb + n0 * kb32;
  const int64_t srows = wr == 0 ? g.M - m0 : g.N - n0;
  const __amdgpu_buffer_rsrc_t srsrc = rsrc_of(sbase, (srows < 256 ? srows : 256) * kb32);
  const uint32_t svoff = (uint32_t)(srow * kb32);
  char* const sdst0 = smem + MX_SC + wr * 1024 + (wave & 3) * 256;
  auto sissue = [&](int kt) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(srsrc, (lds_vp)(sdst0 + (kt & 1) * 2048), 4, svoff, kt * 4, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* const st0 = smem;
  char* const st1 = smem + MG_STAGE;
  if (nk > 0) {
    la.issue(st0, 0, wave);
    sissue(0);
    lb.issue(st0 + 2 * MG_HALF, 0, wave);
  }
  if (nk > 1) {
    lb.issue(st1 + 2 * MG_HALF, 1, wave);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  const int bhalf = wc >> 1;
  const int bcol = 64 * (wc & 1);
  i32x8 af[4], bfr[4];
  int sa[4], sb[4];
  for (int t = 0; t < nk; ++t) {
    const char* cur = (t & 1) ? st1 : st0;
    const char* ah = cur + wr * MG_HALF;
    const char* bh = cur + (2 + bhalf) * MG_HALF;
    const char* scur = smem + MX_SC + (t & 1) * 2048;
    // ---------------- phase 0: rows 0..63 of the wave's 128
#pragma unroll
    for (int i = 0; i < 4; ++i) { af[i] = mx_frag(ah, 16 * i, lane); sa[i] = mx_scale(scur, 128 * wr + 16 * i, lane); }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bfr[j] = mx_frag(bh, bcol + 16 * j, lane);
      sb[j] = mx_scale(scur + 1024, 128 * bhalf + bcol + 16 * j, lane);
    }
    if (t + 1 < nk) {
      la.issue((t & 1) ? st0 : st1, t + 1, wave);
      sissue(t + 1);
      asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0, 0, 0, sb[j], 0, sa[i]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---------------- phase 1: rows 64..127, the same B fragments
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i] = mx_frag(ah, 64 + 16 * i, lane);
      sa[i] = mx_scale(scur, 128 * wr + 64 + 16 * i, lane);
    }
    if (t + 2 < nk) {
      lb.issue(const_cast<char*>(cur) + 2 * MG_HALF, t + 2, wave);
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] =
            __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[4 + i][j], 0, 0, 0, sb[j], 0, sa[i]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();
  mg_epilogue<EPI>(g, acc, smem, wave, lane, bm, 0, m0, n0);
}
template __global__ void mxgemm_kernel<0>(MArgs, MxArgs);
template __global__ void mxgemm_kernel<1>(MArgs, MxArgs);
template __global__ void mxgemm_kernel<2>(MArgs, MxArgs);
template __global__ void mxgemm_kernel<3>(MArgs, MxArgs);
template __global__ void mxgemm_kernel<7>(MArgs, MxArgs);  // EPI_DMUL: the fp8 backward-data of fc2

// MX quantiser: 8 values per thread, 4 threads per 32-element block (a block never straddles a row:
// cols % 32 == 0).  OCP MX rule: shared exponent e = floor(log2(amax)) - 8 (e4m3 emax), clamped to
// [-127, 127], scale byte e + 127; elements x * 2^-e saturated to +-448 and rounded to nearest-even
// e4m3fn (v_cvt_pk_fp8_f32, OCP format on gfx950); an all-zero block gets scale byte 0.
template <typename T>
__global__ __launch_bounds__(256) void mx_quant_kernel(const T* __restrict__ x, int64_t rows, int64_t cols, int64_t ldx,
                                                       uint8_t* __restrict__ q, int64_t ldq, uint8_t* __restrict__ sc) {
  const int64_t per_row = cols >> 3;
  const int64_t total = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = (i - r * per_row) * 8;
    float v[8];
    if constexpr (sizeof(T) == 2) {
      const uint4 u = *reinterpret_cast<const uint4*>(x + r * ldx + c);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[2 * k] = __uint_as_float(w[k] << 16); v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u); }
    } else {
      const float4 a = *reinterpret_cast<const float4*>(x + r * ldx + c);
      const float4 b = *reinterpret_cast<const float4*>(x + r * ldx + c + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    const int e = mx_exponent_4lanes(v);
    *reinterpret_cast<uint2*>(q + r * ldq + c) = mx_pack8(v, e);
    if ((c & 31) == 0) sc[r * (cols >> 5) + (c >> 5)] = (uint8_t)(e + 127);
  }
}

// MX quantiser of a transpose: q[c][r] = x[r][c] with one shared exponent per 32 consecutive r (the
// backward-data operand W^T of a weight stored W[out][in]: the contraction runs over `out`).  One thread per
// 32-element block, lanes over c (coalesced 4-B / 2-B column reads), the same OCP rule as mx_quant_kernel.
template <typename T>
__global__ __launch_bounds__(256) void mx_quant_t_kernel(const T* __restrict__ x, int64_t rows, int64_t cols,
                                                         int64_t ldx, uint8_t* __restrict__ q, int64_t ldq,
                                                         uint8_t* __restrict__ sc) {
  const int64_t nb = rows >> 5;  // blocks per output row
  const int64_t total = nb * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t blk = i / cols, c = i - blk * cols;
    float v[32];
    float am = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      v[k] = (float)x[(blk * 32 + k) * ldx + c];
      am = fmaxf(am, fabsf(v[k]));
    }
    const int e = mx_exponent(am);
    uint2* dst = reinterpret_cast<uint2*>(q + c * ldq + blk * 32);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = mx_pack8(v + 8 * k, e);
    sc[c * nb + blk] = (uint8_t)(e + 127);
  }
}

// fixed-order split-K reduction of the f32 slabs into the epilogue's output (f32 or bf16, +bias)
__global__ __launch_bounds__(256) void mg_splitk_reduce_kernel(const float* __restrict__ ws, int split, int64_t M,
                                                               int64_t N, void* out, int64_t ldc, int out_f32,
                                                               const float* __restrict__ bias) {
  const int64_t n4 = N >> 2;
  const int64_t total = M * n4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / n4, n = (i - m * n4) * 4;
    f32x4 s = *reinterpret_cast<const f32x4*>(ws + m * N + n);
    for (int zz = 1; zz < split; ++zz) s += *reinterpret_cast<const f32x4*>(ws + ((int64_t)zz * M + m) * N + n);
    if (bias) {
#pragma unroll
      for (int c = 0; c < 4; ++c) s[c] += bias[n + c];
    }
    if (out_f32) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + m * ldc + n) = s;
    else *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + m * ldc + n) = pack4(s);
  }
}

// A-operand column sums: the split-K partials in slice order (deterministic)
__global__ __launch_bounds__(256) void mg_acs_reduce_kernel(const float* __restrict__ part, int split, int64_t M,
                                                            float* __restrict__ out) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  float acc = 0.f;
  for (int z = 0; z < split; ++z) acc += part[(int64_t)z * M + m];
  out[m] = acc;
}

__global__ __launch_bounds__(256) void mg_colsum_final_kernel(const double* __restrict__ part2, int N, float* out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) out[c] = (float)colsum_slices(part2, N, c);
}

template <int LA, int LB>
hipError_t launch_epi(const MArgs& a, int epi, hipStream_t s) {
  const unsigned grid = (unsigned)((int64_t)a.nbm * a.nbn * a.split);
  if constexpr (LA == MG_RC) {
    if (a.acs_part) {  // A-operand column sums: split-K slabs or an unsplit f32 output
      if (epi == EPI_SLAB) mgemm_kernel<LA, LB, EPI_SLAB, true><<<grid, MG_NT, 0, s>>>(a);
      else mgemm_kernel<LA, LB, EPI_PLAIN, true><<<grid, MG_NT, 0, s>>>(a);
      return hipGetLastError();
    }
  }
  switch (epi) {
    case EPI_PLAIN: mgemm_kernel<LA, LB, EPI_PLAIN><<<grid, MG_NT, 0, s>>>(a); break;
    case EPI_GELU: mgemm_kernel<LA, LB, EPI_GELU><<<grid, MG_NT, 0, s>>>(a); break;
    case EPI_GELU_SAVE: mgemm_kernel<LA, LB, EPI_GELU_SAVE><<<grid, MG_NT, 0, s>>>(a); break;
    case EPI_ADD_AUX: mgemm_kernel<LA, LB, EPI_ADD_AUX><<<grid, MG_NT, 0, s>>>(a); break;
    case EPI_DGELU: mgemm_kernel<LA, LB, EPI_DGELU><<<grid, MG_NT, 0, s>>>(a); break;
    case EPI_GELU_SAVE_D: mgemm_kernel<LA, LB, EPI_GELU_SAVE_D><<<grid, MG_NT, 0, s>>>(a); break;
    case EPI_DMUL: mgemm_kernel<LA, LB, EPI_DMUL><<<grid, MG_NT, 0, s>>>(a); break;
    default: mgemm_kernel<LA, LB, EPI_SLAB><<<grid, MG_NT, 0, s>>>(a); break;
  }
  return hipGetLastError();
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

namespace mgemm {

// Tile order for a launch, a fixed function of the shape and layout: grouped (8 row blocks) for wide unsplit
// outputs of a k-by-n (RC) B operand -- the backward-data GEMMs of the wide linears (fc2.dgrad 2.43 -> 2.38 ms);
// the k-contiguous forward shapes measured mixed (qkv.fwd -0.8 %, fc1.fwd +1.7 %, MX-fp8 unchanged: r6gm2)
int mg_group_m(int nbm, int nbn, int split, int lb) {
  return split == 1 && lb == MIA_LAYOUT_RC && nbn >= 9 && nbm >= 16 ? 8 : 0;
}

// Which epilogue kind the kernel would run for E (-1: not this kernel)
int mg_epi_kind(const MiaEpilogue& E, int64_t N) {
  // a drop-mode row map (MIA_RM_DROP) only on a plain / bias bf16 output without an MX copy
  const bool drop = E.rm_inner && E.rm_offset == MIA_RM_DROP && E.rm_istride == 1 && E.rm_outer == E.rm_inner - 1 &&
                    E.act == MIA_ACT_NONE && E.dtype == MIA_BF16 && !E.mx_q && !E.colsum;
  if (E.accumulate || (E.rm_inner && !drop) || E.sqsum || E.alpha != 1.f || !E.ptr) return -1;
  if (E.mx_q && (!E.mx_scales || E.dtype != MIA_BF16 || E.ldc != N || N % 32 ||
                 (E.colsum && E.act != MIA_DACT_MUL) ||
                 !(E.act == MIA_ACT_NONE || E.act == MIA_ACT_GELU || E.act == MIA_ACT_GELU_SAVE ||
                   E.act == MIA_ACT_GELU_SAVE_D || E.act == MIA_DACT_MUL)))
    return -1;
  const bool bf = E.dtype == MIA_BF16, f32 = E.dtype == MIA_F32;
  if ((E.ldc & 3) || E.ldc < N || (reinterpret_cast<uintptr_t>(E.ptr) & (bf ? 7 : 15)) != 0) return -1;
  // bf16 outputs leave the LDS image as 16-B pieces (8 columns) guarded by n < N only
  if (bf && N % 8) return -1;
  if (E.bias && (reinterpret_cast<uintptr_t>(E.bias) & 15)) return -1;
  const bool aux_ok = E.aux && aligned16(E.aux) && (E.ldaux & 3) == 0 && E.ldaux >= N;
  switch (E.act) {
    case MIA_ACT_NONE: return (bf || f32) && !E.colsum ? EPI_PLAIN : -1;
    case MIA_ACT_GELU: return bf && !E.colsum ? EPI_GELU : -1;
    case MIA_ACT_GELU_SAVE: return bf && aux_ok && E.aux_dtype == MIA_BF16 && !E.colsum ? EPI_GELU_SAVE : -1;
    case MIA_ACT_ADD_AUX: return f32 && aux_ok && E.aux_dtype == MIA_F32 && !E.colsum ? EPI_ADD_AUX : -1;
    case MIA_DACT_GELU: return bf && aux_ok && E.aux_dtype == MIA_BF16 && !E.bias ? EPI_DGELU : -1;
    case MIA_ACT_GELU_SAVE_D: return bf && aux_ok && E.aux_dtype == MIA_BF16 && !E.colsum ? EPI_GELU_SAVE_D : -1;
    case MIA_DACT_MUL: return bf && aux_ok && E.aux_dtype == MIA_BF16 && !E.bias ? EPI_DMUL : -1;
    default: return -1;
  }
}

// This kernel takes dense bf16 GEMMs big enough to fill the chip with 256 x 256 tiles (AST token
// counts, or a weight gradient over them): A/B without pre-op, 16-B aligned, ld % 8 == 0, N % 4 == 0
// (N % 8 == 0 for a bf16 output),
// K % 64 == 0 where K is the contiguous dimension (KC), any K where it is the row index (RC).
bool mg_ok(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
           int compute) {
  if (compute != MIA_BF16 || M < 256 || N < 256 || N % 4 || K < 64) return false;
  if (cdiv(M, MG_BM) * cdiv(N, MG_BN) < 32 && K < 16384) return false;  // small: the 128 x 128 kernel
  if (A.kind != MIA_OP_DENSE || B.kind != MIA_OP_DENSE || A.dtype != MIA_BF16 || B.dtype != MIA_BF16) return false;
  if (A.pre != MIA_PRE_NONE || B.pre != MIA_PRE_NONE || A.ld % 8 || B.ld % 8 || !aligned16(A.ptr) || !aligned16(B.ptr))
    return false;
  if (A.layout == MIA_LAYOUT_KC) { if (A.rows != M || A.cols < K || K % MG_BK) return false; }
  else if (A.rows < K || A.cols != M || M % 8) return false;
  if (B.layout == MIA_LAYOUT_KC) { if (B.rows != N || B.cols < K || K % MG_BK) return false; }
  else if (B.rows < K || B.cols != N || N % 8) return false;
  if (cdiv(M, MG_BM) * cdiv(N, MG_BN) >= (1ll << 24)) return false;
  // A-operand column sums: a k-by-m A and a plain output (the weight gradients)
  if (E.a_colsum && (A.layout != MIA_LAYOUT_RC || mg_epi_kind(E, N) != EPI_PLAIN)) return false;
  return mg_epi_kind(E, N) >= 0;
}

// split-K width for the weight gradients (few output tiles, K = tokens): tiles x split = one round of
// workgroups on the MI355X's 256 CUs (a constant, not the device's count: the split sets the summation order,
// so it stays a fixed function of the shape), K-slices of at least 1024.  Measured against the earlier ~3
// rounds (768) and against 128 / 192 / 384 (tools/gemm_ab.sh, r6sp / r6sp2): fc1.wgrad 1.87 -> 1.78 ms, fc2.wgrad
// 1.97 -> 1.86, proj.wgrad 0.58 -> 0.52, qkv.wgrad 1.39 -> 1.34 (fewer f32 slabs, no partial last round); a
// partial round (192, 384) or fewer workgroups than CUs (128) is slower.
int mg_split(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = cdiv(M, MG_BM) * cdiv(N, MG_BN);
  if (tiles >= 512 || K < 4096) return 1;
  int64_t s = 256 / tiles;  // 27 tiles x 9, 36 x 7, 9 x 28
  const int64_t smax = K / 1024;
  if (s > smax) s = smax;
  return (int)(s < 1 ? 1 : s);
}

static void mg_geometry(int64_t M, int64_t N, int64_t K, int& split, int64_t& kper) {
  split = mg_split(M, N, K);
  kper = cdiv(cdiv(K, split), 64) * 64;
  split = (int)cdiv(K, kper);
}

int64_t mg_workspace_bytes(int64_t M, int64_t N, int64_t K, int colsum, int a_colsum) {
  int split;
  int64_t kper;
  mg_geometry(M, N, K, split, kper);
  int64_t b = split > 1 ? (int64_t)split * M * N * 4 : 0;
  b = cdiv(b, 256) * 256;
  if (colsum) b += cdiv(cdiv(M, MG_BM) * N * 4, 256) * 256 + colsum_part2_bytes((int)N);
  if (a_colsum) b += cdiv((int64_t)split * M * 4, 256) * 256;
  return b;
}

int mg_run(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
           void* workspace, hipStream_t s) {
  const int epi = mg_epi_kind(E, N);
  MArgs a;
  memset(&a, 0, sizeof(a));
  a.a = reinterpret_cast<const bf16*>(A.ptr);
  a.b = reinterpret_cast<const bf16*>(B.ptr);
  a.lda = A.ld; a.ldb = B.ld; a.M = M; a.N = N; a.K = K;
  mg_geometry(M, N, K, a.split, a.kper);
  a.nbm = (int)cdiv(M, MG_BM); a.nbn = (int)cdiv(N, MG_BN);
  a.group_m = mg_group_m(a.nbm, a.nbn, a.split, B.layout);
  a.out = E.ptr; a.ldc = E.ldc; a.out_f32 = E.dtype == MIA_F32;
  a.drop_w = E.rm_inner && E.rm_offset == MIA_RM_DROP ? E.rm_inner : 0;
  a.bias = E.bias; a.aux = E.aux; a.ldaux = E.ldaux;
  a.mxq = reinterpret_cast<uint8_t*>(E.mx_q); a.mxs = reinterpret_cast<uint8_t*>(E.mx_scales);
  const int need_ws = a.split > 1 || E.colsum || E.a_colsum;
  MIA_CHECK_ARG(!need_ws || workspace, "gemm: the 256x128 path needs the workspace of mia_gemm_workspace_bytes_ex");
  char* ws = reinterpret_cast<char*>(workspace);
  int kind = epi;
  if (a.split > 1) {
    MIA_CHECK_ARG(epi == EPI_PLAIN && !E.colsum, "gemm: split-K weight gradients take a plain epilogue");
    a.ws = reinterpret_cast<float*>(ws);
    a.bias = nullptr;  // added by the reduction
    kind = EPI_SLAB;
    ws += cdiv((int64_t)a.split * M * N * 4, 256) * 256;
  }
  if (E.colsum) {
    a.colsum_part = reinterpret_cast<float*>(ws);
    ws += cdiv((int64_t)a.nbm * N * 4, 256) * 256;
  }
  if (E.a_colsum) a.acs_part = reinterpret_cast<float*>(ws);  // after the slabs (plain epilogue: no colsum)
  hipError_t err;
  const int la = A.layout, lb = B.layout;
  if (la == MIA_LAYOUT_KC && lb == MIA_LAYOUT_KC) err = launch_epi<MG_KC, MG_KC>(a, kind, s);
  else if (la == MIA_LAYOUT_KC) err = launch_epi<MG_KC, MG_RC>(a, kind, s);
  else if (lb == MIA_LAYOUT_RC) err = launch_epi<MG_RC, MG_RC>(a, kind, s);
  else err = launch_epi<MG_RC, MG_KC>(a, kind, s);
  if (err != hipSuccess) return mia::fail(-(int)err, "mgemm launch: %s", hipGetErrorString(err));
  if (a.split > 1) {
    const int64_t total = M * (N / 4);
    const int blocks = (int)std::min<int64_t>(cdiv(total, 256), 4096);
    mg_splitk_reduce_kernel<<<blocks, 256, 0, s>>>(a.ws, a.split, M, N, E.ptr, E.ldc, E.dtype == MIA_F32, E.bias);
    MIA_LAUNCH_CHECK("mgemm splitk reduce");
  }
  if (E.a_colsum) {
    mg_acs_reduce_kernel<<<(unsigned)cdiv(M, 256), 256, 0, s>>>(a.acs_part, a.split, M, E.a_colsum);
    MIA_LAUNCH_CHECK("mgemm a_colsum");
  }
  if (E.colsum && (kind == EPI_DGELU || kind == EPI_DMUL)) {
    double* part2 = reinterpret_cast<double*>(ws);
    colsum_pass1(a.colsum_part, a.nbm, (int)N, N, part2, s);
    mg_colsum_final_kernel<<<(unsigned)cdiv(N, 256), 256, 0, s>>>(part2, (int)N, E.colsum);
    MIA_LAUNCH_CHECK("mgemm colsum");
  }
  return 0;
}

}  // namespace mgemm

// ---------------------------------------------------------------- MX-fp8 C ABI
extern "C" int mia_mx_quantize(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ldx, void* q,
                               int64_t ldq, void* scales, mia_stream_t stream) {
  MIA_CHECK_ARG(x_dtype == MIA_BF16 || x_dtype == MIA_F32, "mx_quantize: input must be bf16 or f32");
  MIA_CHECK_ARG(rows >= 0 && cols >= 0 && cols % 32 == 0, "mx_quantize: cols must be a multiple of 32");
  MIA_CHECK_ARG(ldx >= cols && ldq >= cols && ldq % 8 == 0 && ldx % 8 == 0, "mx_quantize: bad leading dimension");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(q) & 7) == 0,
                "mx_quantize: x must be 16-B and q 8-B aligned");
  if (rows == 0 || cols == 0) return 0;
  const int64_t total = rows * (cols / 8);
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(total, 256), 16384);
  hipStream_t s = as_stream(stream);
  if (x_dtype == MIA_BF16)
    mx_quant_kernel<bf16><<<blocks, 256, 0, s>>>(reinterpret_cast<const bf16*>(x), rows, cols, ldx,
                                                 reinterpret_cast<uint8_t*>(q), ldq, reinterpret_cast<uint8_t*>(scales));
  else
    mx_quant_kernel<float><<<blocks, 256, 0, s>>>(reinterpret_cast<const float*>(x), rows, cols, ldx,
                                                  reinterpret_cast<uint8_t*>(q), ldq, reinterpret_cast<uint8_t*>(scales));
  MIA_LAUNCH_CHECK("mx_quantize");
  return 0;
}

extern "C" int mia_mx_quantize_t(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ldx, void* q,
                                 int64_t ldq, void* scales, mia_stream_t stream) {
  MIA_CHECK_ARG(x_dtype == MIA_BF16 || x_dtype == MIA_F32, "mx_quantize_t: input must be bf16 or f32");
  MIA_CHECK_ARG(rows >= 0 && cols >= 0 && rows % 32 == 0, "mx_quantize_t: rows must be a multiple of 32");
  MIA_CHECK_ARG(ldx >= cols && ldq >= rows && ldq % 8 == 0, "mx_quantize_t: bad leading dimension");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(q) & 7) == 0, "mx_quantize_t: q must be 8-B aligned");
  if (rows == 0 || cols == 0) return 0;
  const int64_t total = (rows / 32) * cols;
  const unsigned blocks = (unsigned)std::min<int64_t>(cdiv(total, 256), 16384);
  hipStream_t s = as_stream(stream);
  if (x_dtype == MIA_BF16)
    mx_quant_t_kernel<bf16><<<blocks, 256, 0, s>>>(reinterpret_cast<const bf16*>(x), rows, cols, ldx,
                                                   reinterpret_cast<uint8_t*>(q), ldq, reinterpret_cast<uint8_t*>(scales));
  else
    mx_quant_t_kernel<float><<<blocks, 256, 0, s>>>(reinterpret_cast<const float*>(x), rows, cols, ldx,
                                                    reinterpret_cast<uint8_t*>(q), ldq, reinterpret_cast<uint8_t*>(scales));
  MIA_LAUNCH_CHECK("mx_quantize_t");
  return 0;
}

extern "C" int64_t mia_gemm_mxfp8_workspace_bytes(int64_t M, int64_t N, int32_t colsum) {
  return colsum ? cdiv(cdiv(M, MG_BM) * N * 4, 256) * 256 + colsum_part2_bytes((int)N) : 0;
}

extern "C" int mia_gemm_mxfp8(const void* a, const void* a_scales, int64_t lda, const void* b, const void* b_scales,
                              int64_t ldb, const MiaEpilogue* E, int64_t M, int64_t N, int64_t K, mia_stream_t stream) {
  return mia_gemm_mxfp8_ex(a, a_scales, lda, b, b_scales, ldb, E, M, N, K, nullptr, stream);
}

extern "C" int mia_gemm_mxfp8_ex(const void* a, const void* a_scales, int64_t lda, const void* b, const void* b_scales,
                                 int64_t ldb, const MiaEpilogue* E, int64_t M, int64_t N, int64_t K, void* workspace,
                                 mia_stream_t stream) {
  MIA_CHECK_ARG(a && b && a_scales && b_scales && E && E->ptr, "gemm_mxfp8: null operand");
  MIA_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 128 == 0, "gemm_mxfp8: K must be a positive multiple of 128");
  MIA_CHECK_ARG(lda >= K && ldb >= K && lda % 16 == 0 && ldb % 16 == 0, "gemm_mxfp8: lda / ldb (bytes) must be >= K and 16-B multiples");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(a) & 15) == 0 && (reinterpret_cast<uintptr_t>(b) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(a_scales) & 3) == 0 && (reinterpret_cast<uintptr_t>(b_scales) & 3) == 0,
                "gemm_mxfp8: operands 16-B and scales 4-B aligned");
  MIA_CHECK_ARG(N % 4 == 0 && (E->dtype != MIA_BF16 || N % 8 == 0) && cdiv(M, MG_BM) * cdiv(N, MG_BN) < (1ll << 24),
                "gemm_mxfp8: N must be a multiple of 4 (of 8 for a bf16 output)");
  const int epi = mgemm::mg_epi_kind(*E, N);
  MIA_CHECK_ARG(epi == EPI_PLAIN || epi == EPI_GELU || epi == EPI_GELU_SAVE || epi == EPI_GELU_SAVE_D || epi == EPI_ADD_AUX ||
                    epi == EPI_DMUL,
                "gemm_mxfp8: epilogue must be plain / bias / GELU / GELU_SAVE(_D) / f32 residual / x saved gelu' "
                "(row-major, aligned)");
  MIA_CHECK_ARG(!E->colsum || (epi == EPI_DMUL && workspace),
                "gemm_mxfp8: column sums ride the x-gelu' epilogue and need mia_gemm_mxfp8_workspace_bytes");
  MArgs g;
  memset(&g, 0, sizeof(g));
  g.a = reinterpret_cast<const bf16*>(a);
  g.b = reinterpret_cast<const bf16*>(b);
  g.lda = lda / 2; g.ldb = ldb / 2;  // e4m3 rows seen as bf16 pairs by the loaders
  g.M = M; g.N = N; g.K = K; g.kper = K; g.split = 1;
  g.nbm = (int)cdiv(M, MG_BM); g.nbn = (int)cdiv(N, MG_BN);
  g.group_m = 0;  // MX-fp8 operands are k-contiguous (mg_group_m)
  g.out = E->ptr; g.ldc = E->ldc; g.out_f32 = E->dtype == MIA_F32;
  g.bias = E->bias; g.aux = E->aux; g.ldaux = E->ldaux;
  g.mxq = reinterpret_cast<uint8_t*>(E->mx_q); g.mxs = reinterpret_cast<uint8_t*>(E->mx_scales);
  MxArgs x{reinterpret_cast<const uint8_t*>(a_scales), reinterpret_cast<const uint8_t*>(b_scales)};
  const unsigned grid = (unsigned)((int64_t)g.nbm * g.nbn);
  hipStream_t s = as_stream(stream);
  if (E->colsum) g.colsum_part = reinterpret_cast<float*>(workspace);
  switch (epi) {
    case EPI_PLAIN: mxgemm_kernel<EPI_PLAIN><<<grid, MG_NT, 0, s>>>(g, x); break;
    case EPI_GELU: mxgemm_kernel<EPI_GELU><<<grid, MG_NT, 0, s>>>(g, x); break;
    case EPI_GELU_SAVE: mxgemm_kernel<EPI_GELU_SAVE><<<grid, MG_NT, 0, s>>>(g, x); break;
    case EPI_GELU_SAVE_D: mxgemm_kernel<EPI_GELU_SAVE_D><<<grid, MG_NT, 0, s>>>(g, x); break;
    case EPI_DMUL: mxgemm_kernel<EPI_DMUL><<<grid, MG_NT, 0, s>>>(g, x); break;
    default: mxgemm_kernel<EPI_ADD_AUX><<<grid, MG_NT, 0, s>>>(g, x); break;
  }
  MIA_LAUNCH_CHECK("gemm_mxfp8");
  if (E->colsum) {
    double* part2 = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + cdiv((int64_t)g.nbm * N * 4, 256) * 256);
    colsum_pass1(g.colsum_part, g.nbm, (int)N, N, part2, s);
    mg_colsum_final_kernel<<<(unsigned)cdiv(N, 256), 256, 0, s>>>(part2, (int)N, E->colsum);
    MIA_LAUNCH_CHECK("gemm_mxfp8 colsum");
  }
  return 0;
}
