// Implicit-GEMM on MFMA for gfx950 — the dense contractions of the hot path.
//
// One kernel template serves: every EnvNet-v2 conv (fwd = im2col(x) . W^T, dgrad = conv of the
// padded dY with the flipped kernel, wgrad = dY^T . im2col(x)), the FC layers, the AST linears and
// the AST patch-embed conv.  Operands are gathered straight from NHWC activations (no im2col
// buffer), converted to the compute type while staging into LDS, optionally transformed by the
// previous layer's BatchNorm affine + ReLU (so BN-apply never takes its own HBM pass).
//
//  * compute bf16: v_mfma_f32_32x32x16_bf16, lane holds 8 consecutive k of its row.
//  * compute f32 : v_mfma_f32_32x32x2_f32 x 8 per 16-k step over the SAME 8-consecutive-k lane
//                  fragments (the k order inside a step is permuted identically for A and B,
//                  so the sum is unchanged) — exact-f32 path used for parity.
//  * LDS tile layouts: KC = [row][k] (+16 B row pad: conflict-free ds_read_b128),
//                      RC = [k][row] read with ds_read_b64_tr_b16 (bf16) / ds_read_b32 (f32),
//                      row stride padded to 16 dwords mod 64 (conflict-free transposed reads).
//  * 256 threads = 4 waves, each owning (BM/WM) x (BN/WN) of 32x32 accumulator tiles;
//    register-staged double-buffered K loop (BK = 32), one barrier per K tile.
//  * split-K writes f32 partial slabs; a reduce kernel applies the epilogue.
#include "gemm_common.h"

#include <cstdlib>

namespace {

using namespace mgemm;

constexpr int BK = 32;
constexpr int NT = 256;

struct OpDev {
  const char* ptr;
  int kind, dtype, pre;
  int64_t rows, cols, ld;
  int n, h, w, c, oh, ow, kh, kw, sh, sw, ph, pw;
  int npix, ohw, kwc, jtot;
  const float* ps;
  const float* pt;
};



struct GemmArgs {
  OpDev a, b;
  EpiDev e;
  int64_t M, N, K, kper;
  int split;
  float* ws;
};

template <typename T> struct TT;
template <> struct TT<bf16> { static constexpr int dt = MIA_BF16; static constexpr int CW = 4; };
template <> struct TT<float> { static constexpr int dt = MIA_F32; static constexpr int CW = 8; };

__device__ __forceinline__ float apply_pre(const OpDev& o, float v, int ch) {
  if (o.pre == MIA_PRE_AFFINE || o.pre == MIA_PRE_AFFINE_RELU) {
    v = fmaf(v, o.ps[ch], o.pt[ch]);
    if (o.pre == MIA_PRE_AFFINE_RELU) v = fmaxf(v, 0.f);
  } else if (o.pre == MIA_PRE_GELU) {
    v = gelu_erf(v);
  }
  return v;
}

// Load 8 consecutive source elements starting at element offset `off` (off < 0: zeros),
// apply the pre-op, and pack them as the compute type T into v[].
template <typename T>
__device__ __forceinline__ void load_chunk(const OpDev& o, int64_t off, int nvalid, int ch,
                                           uint32_t (&v)[TT<T>::CW]) {
  constexpr int CW = TT<T>::CW;
  if (off < 0) {
#pragma unroll
    for (int i = 0; i < CW; ++i) v[i] = 0u;
    return;
  }
  float f[8];
  if (o.dtype == MIA_BF16) {
    const bf16* p = reinterpret_cast<const bf16*>(o.ptr) + off;
    if (nvalid == 8 && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
      uint4 u = *reinterpret_cast<const uint4*>(p);
      if constexpr (TT<T>::dt == MIA_BF16) {
        if (o.pre == MIA_PRE_NONE) {
          v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
          return;
        }
      }
      uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w4[i] << 16);
        f[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = i < nvalid ? (float)p[i] : 0.f;
    }
  } else {
    const float* p = reinterpret_cast<const float*>(o.ptr) + off;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if (nvalid == 8 && (a & 15) == 0) {
      float4 x0 = reinterpret_cast<const float4*>(p)[0];
      float4 x1 = reinterpret_cast<const float4*>(p)[1];
      f[0] = x0.x; f[1] = x0.y; f[2] = x0.z; f[3] = x0.w;
      f[4] = x1.x; f[5] = x1.y; f[6] = x1.z; f[7] = x1.w;
    } else if (nvalid == 8 && (a & 7) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float2 x = reinterpret_cast<const float2*>(p)[i];
        f[2 * i] = x.x; f[2 * i + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = i < nvalid ? p[i] : 0.f;
    }
  }
  if (o.pre != MIA_PRE_NONE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = i < nvalid ? apply_pre(o, f[i], ch + i) : 0.f;
  }
  if constexpr (TT<T>::dt == MIA_BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = pk_bf16(f[2 * i], f[2 * i + 1]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = __float_as_uint(f[i]);
  }
}

// -------------------------------------------------------------------------- loaders
// KC: tile rows R, each row = BK k-elements; a thread owns chunk column kq = t%4 and rows t/4+64s.
template <typename T, int R>
struct LoaderKC {
  static constexpr int CHUNKS = R * BK / 8;
  static constexpr int CH = (CHUNKS + NT - 1) / NT;
  static constexpr int CW = TT<T>::CW;
  static constexpr int RS = BK * (int)sizeof(T) + 16;  // LDS row stride (bytes)
  static constexpr int BYTES = R * RS;
  int kq;
  bool active[CH];
  int64_t rowoff[CH];        // DENSE
  int bh[CH], bih[CH], biw[CH];  // CONV: b*h, y*sh-ph, x*sw-pw
  bool rvalid[CH];
  int ky, kx, ci;            // CONV tap state for j
  int64_t j;
  uint32_t v[CH][CW];

  __device__ __forceinline__ void init(const OpDev& o, int64_t r0, int64_t kbeg, int t) {
    kq = t & 3;
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const int chunk = t + NT * s;
      active[s] = chunk < CHUNKS;
      const int64_t row = r0 + (chunk >> 2);
      if (o.kind == MIA_OP_DENSE) {
        rvalid[s] = row < o.rows;
        rowoff[s] = row * o.ld;
      } else {
        rvalid[s] = row < o.npix;
        const int ri = rvalid[s] ? (int)row : 0;
        const int b = ri / o.ohw;
        const int rr = ri - b * o.ohw;
        const int y = rr / o.ow;
        const int x = rr - y * o.ow;
        bh[s] = b * o.h;
        bih[s] = y * o.sh - o.ph;
        biw[s] = x * o.sw - o.pw;
      }
    }
    j = kbeg + kq * 8;
    if (o.kind == MIA_OP_CONV) {
      ci = (int)(j % o.c);
      const int tt = (int)(j / o.c);
      kx = tt % o.kw;
      ky = tt / o.kw;
    } else if (o.kind == MIA_OP_CONVROW) {
      ky = (int)(j / o.kwc);
      ci = (int)(j - (int64_t)ky * o.kwc);
      kx = 0;
    }
  }
  __device__ __forceinline__ void advance(const OpDev& o) {
    j += BK;
    if (o.kind == MIA_OP_CONV) {
      ci += BK;
      while (ci >= o.c) {
        ci -= o.c;
        if (++kx == o.kw) { kx = 0; ++ky; }
      }
    } else if (o.kind == MIA_OP_CONVROW) {
      ci += BK;
      while (ci >= o.kwc) { ci -= o.kwc; ++ky; }
    }
  }
  __device__ __forceinline__ void load(const OpDev& o, int64_t kend) {
    const bool jok = j < kend;
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      if (!active[s]) continue;
      int64_t off = -1;
      int nvalid = 8;
      int ch = 0;
      if (jok && rvalid[s]) {
        if (o.kind == MIA_OP_DENSE) {
          if (j < o.cols) {
            off = rowoff[s] + j;
            const int64_t rem = o.cols - j;
            nvalid = rem < 8 ? (int)rem : 8;
            ch = (int)j;
          }
        } else if (j < o.jtot) {
          const int ih = bih[s] + ky;
          const int iw = biw[s] + kx;
          if (ih >= 0 && ih < o.h && iw >= 0 && iw < o.w) {
            off = ((int64_t)(bh[s] + ih) * o.w + iw) * o.c + ci;
            ch = ci;
          }
        }
      }
      load_chunk<T>(o, off, nvalid, ch, v[s]);
    }
  }
  __device__ __forceinline__ void store(char* lds, int t) const {
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      if (!active[s]) continue;
      const int row = (t + NT * s) >> 2;
      char* p = lds + row * RS + kq * 8 * (int)sizeof(T);
      if constexpr (CW == 4) {
        *reinterpret_cast<uint4*>(p) = make_uint4(v[s][0], v[s][1], v[s][2], v[s][3]);
      } else {
        reinterpret_cast<uint4*>(p)[0] = make_uint4(v[s][0], v[s][1], v[s][2], v[s][3]);
        reinterpret_cast<uint4*>(p)[1] = make_uint4(v[s][4], v[s][5], v[s][6], v[s][7]);
      }
    }
  }
};

// RC: tile = BK k-rows x R contiguous elements; thread owns row-chunk rq = t%RQ, k-rows t/RQ + step*s.
template <typename T, int R>
struct LoaderRC {
  static constexpr int RQ = R / 8;
  static constexpr int STEP = NT / RQ;
  static constexpr int CHUNKS = BK * RQ;
  static constexpr int CH = (CHUNKS + NT - 1) / NT;
  static constexpr int CW = TT<T>::CW;
  static constexpr int PADDW = sizeof(T) == 2 ? ((16 - R / 2) % 64 + 64) % 64 : 4;
  static constexpr int RS = R * (int)sizeof(T) + PADDW * 4;
  static constexpr int BYTES = BK * RS;
  int rq, kr0;
  bool active[CH];
  bool jvalid;
  int64_t j;
  int ky, kx, ci;
  uint32_t v[CH][CW];
  int64_t k0;

  __device__ __forceinline__ void init(const OpDev& o, int64_t r0, int64_t kbeg, int t) {
    rq = t % RQ;
    kr0 = t / RQ;
#pragma unroll
    for (int s = 0; s < CH; ++s) active[s] = (t + NT * s) < CHUNKS;
    j = r0 + rq * 8;
    if (o.kind == MIA_OP_DENSE) {
      jvalid = j < o.cols;
    } else {
      jvalid = j < o.jtot;
      if (o.kind == MIA_OP_CONV) {
        ci = (int)(j % o.c);
        const int tt = (int)(j / o.c);
        kx = tt % o.kw;
        ky = tt / o.kw;
      } else {
        ky = (int)(j / o.kwc);
        ci = (int)(j - (int64_t)ky * o.kwc);
        kx = 0;
      }
    }
    k0 = kbeg;
  }
  __device__ __forceinline__ void advance(const OpDev&) { k0 += BK; }
  __device__ __forceinline__ void load(const OpDev& o, int64_t kend) {
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      if (!active[s]) continue;
      const int64_t k = k0 + kr0 + STEP * s;
      int64_t off = -1;
      int nvalid = 8;
      int ch = 0;
      if (jvalid && k < kend) {
        if (o.kind == MIA_OP_DENSE) {
          if (k < o.rows) {
            off = k * o.ld + j;
            const int64_t rem = o.cols - j;
            nvalid = rem < 8 ? (int)rem : 8;
            ch = (int)j;
          }
        } else if (k < o.npix) {
          const int ki = (int)k;
          const int b = ki / o.ohw;
          const int rr = ki - b * o.ohw;
          const int y = rr / o.ow;
          const int x = rr - y * o.ow;
          const int ih = y * o.sh - o.ph + ky;
          const int iw = x * o.sw - o.pw + kx;
          if (ih >= 0 && ih < o.h && iw >= 0 && iw < o.w) {
            off = ((int64_t)(b * o.h + ih) * o.w + iw) * o.c + ci;
            ch = ci;
          }
        }
      }
      load_chunk<T>(o, off, nvalid, ch, v[s]);
    }
  }
  __device__ __forceinline__ void store(char* lds, int t) const {
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      if (!active[s]) continue;
      const int kr = kr0 + STEP * s;
      char* p = lds + kr * RS + rq * 8 * (int)sizeof(T);
      if constexpr (CW == 4) {
        *reinterpret_cast<uint4*>(p) = make_uint4(v[s][0], v[s][1], v[s][2], v[s][3]);
      } else {
        reinterpret_cast<uint4*>(p)[0] = make_uint4(v[s][0], v[s][1], v[s][2], v[s][3]);
        reinterpret_cast<uint4*>(p)[1] = make_uint4(v[s][4], v[s][5], v[s][6], v[s][7]);
      }
    }
  }
};

template <typename T, int L, int R> struct LoaderSel;
template <typename T, int R> struct LoaderSel<T, MIA_LAYOUT_KC, R> { using type = LoaderKC<T, R>; };
template <typename T, int R> struct LoaderSel<T, MIA_LAYOUT_RC, R> { using type = LoaderRC<T, R>; };

// -------------------------------------------------------------------------- fragments
// Fragment of 8 consecutive k (k = ks*16 + 8*(lane>>5) ..+7) for tile row `row`.
template <typename T> struct Frag;
template <> struct Frag<bf16> { bf16x8 x; };
template <> struct Frag<float> { float x[8]; };

template <typename T, int L, int R>
__device__ __forceinline__ Frag<T> read_frag(const char* lds, int row, int ks, int lane) {
  Frag<T> f;
  if constexpr (L == MIA_LAYOUT_KC) {
    constexpr int RS = LoaderKC<T, R>::RS;
    const int kbyte = (ks * 16 + 8 * (lane >> 5)) * (int)sizeof(T);
    const char* p = lds + row * RS + kbyte;
    if constexpr (sizeof(T) == 2) {
      f.x = *reinterpret_cast<const bf16x8*>(p);
    } else {
      float4 a = reinterpret_cast<const float4*>(p)[0];
      float4 b = reinterpret_cast<const float4*>(p)[1];
      f.x[0] = a.x; f.x[1] = a.y; f.x[2] = a.z; f.x[3] = a.w;
      f.x[4] = b.x; f.x[5] = b.y; f.x[6] = b.z; f.x[7] = b.w;
    }
  } else {
    constexpr int RS = LoaderRC<T, R>::RS;
    if constexpr (sizeof(T) == 2) {
      // row = base + (lane & 31); transposed read: group g = lane>>4 reads rows
      // k0..k0+3 (k0 = ks*16 + 8*(g>>1)) x columns col0..col0+15 (col0 = base + 16*(g&1)).
      const int i16 = lane & 15;
      const int g = lane >> 4;
      const int base = row - (lane & 31);
      const int col = base + 16 * (g & 1) + 4 * (i16 & 3);
      const int kr = ks * 16 + 8 * (g >> 1) + (i16 >> 2);
      const char* p0 = lds + kr * RS + col * 2;
      const char* p1 = p0 + 4 * RS;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p1));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      f.x = __builtin_bit_cast(bf16x8, c);
    } else {
      const int kr = ks * 16 + 8 * (lane >> 5);
#pragma unroll
      for (int t = 0; t < 8; ++t)
        f.x[t] = *reinterpret_cast<const float*>(lds + (kr + t) * RS + row * 4);
    }
  }
  return f;
}

__device__ __forceinline__ void mma(f32x16& acc, const Frag<bf16>& a, const Frag<bf16>& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.x, b.x, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma(f32x16& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int t = 0; t < 8; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x[t], b.x[t], acc, 0, 0, 0);
}

template <typename T, int BM, int BN, int WM, int LA, int LB>
__global__ __launch_bounds__(NT) void igemm_kernel(GemmArgs g) {
  constexpr int WN = 4 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  using LA_t = typename LoaderSel<T, LA, BM>::type;
  using LB_t = typename LoaderSel<T, LB, BN>::type;
  constexpr int ABYTES = LA_t::BYTES, BBYTES = LB_t::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * (ABYTES + BBYTES)];
  static_assert(2 * (ABYTES + BBYTES) >= 4 * 32 * 33 * 4, "epilogue staging needs 16.5 KB of LDS");

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  const int z = blockIdx.z;
  const int64_t kbeg = (int64_t)z * g.kper;
  int64_t kend = kbeg + g.kper;
  if (kend > g.K) kend = g.K;
  const int nk = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;

  LA_t la;
  LB_t lb;
  la.init(g.a, m0, kbeg, t);
  lb.init(g.b, n0, kbeg, t);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jn = 0; jn < TN; ++jn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][jn][r] = 0.f;

  if (nk > 0) {
    la.load(g.a, kend);
    lb.load(g.b, kend);
    la.store(smem, t);
    lb.store(smem + ABYTES, t);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* As = smem + cur * (ABYTES + BBYTES);
    const char* Bs = As + ABYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      la.advance(g.a);
      lb.advance(g.b);
      la.load(g.a, kend);
      lb.load(g.b, kend);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      Frag<T> fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = read_frag<T, LA, BM>(As, wm * WTM + i * 32 + (lane & 31), ks, lane);
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) fb[jn] = read_frag<T, LB, BN>(Bs, wn * WTN + jn * 32 + (lane & 31), ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jn = 0; jn < TN; ++jn) mma(acc[i][jn], fa[i], fb[jn]);
    }
    if (more) {
      char* An = smem + (cur ^ 1) * (ABYTES + BBYTES);
      la.store(An, t);
      lb.store(An + ABYTES, t);
    }
    __syncthreads();
  }

  // Epilogue, staged through LDS per 32x32 accumulator tile so each lane then owns 16
  // contiguous output columns of one row (coalesced stores, static accumulator indexing).
  // C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * 33);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jn = 0; jn < TN; ++jn) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        stage[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = acc[i][jn][r];
      __syncthreads();
      const int row = lane >> 1;
      const int c0 = (lane & 1) * 16;
      const int64_t m = m0 + wm * WTM + i * 32 + row;
      const int64_t nb = n0 + wn * WTN + jn * 32 + c0;
      if (m < g.M) {
        if (g.split > 1) {
          float* dst = g.ws + ((int64_t)z * g.M + m) * g.N;
          for (int c = 0; c < 16; ++c)
            if (nb + c < g.N) dst[nb + c] = stage[row * 33 + c0 + c];
        } else if (nb < g.N) {
          float v[16];
#pragma unroll
          for (int c = 0; c < 16; ++c) v[c] = stage[row * 33 + c0 + c];
          epi_store16(g.e, m, nb, g.N, v);
        }
      }
      __syncthreads();
    }
}

__global__ void splitk_reduce_kernel(const float* ws, int split, int64_t M, int64_t N, EpiDev e) {
  const int64_t total = M * N;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < split; ++z) s += ws[z * total + idx];
    epi_store(e, idx / N, idx % N, s);
  }
}

// -------------------------------------------------------------------------- row-window conv
// Direct convolution for the EnvNet-v2 trunk/frontend shapes (stride (1, S), C in {32, 64},
// N = Cout in {32, 64}): a block owns BM consecutive output pixels of ONE output row and, per
// kernel row ky, stages the input row segment they read — (BM-1)*S + KW pixels x C channels —
// once in LDS (BN affine + ReLU of the producer applied while staging, zero padding after it).
// Every im2col element (KW*C per output pixel) is then a ds_read_b128 of that window: the 8-tap
// x C reuse that a gathered im2col tile re-fetches from L2 stays on chip.  S = 2 windows are
// stored de-interleaved (even | odd pixels) so a fragment read is unit-stride in either case.
// The weight tile (N x 128 of the packed [N][KH][KW][C] matrix) is double-buffered; the window
// is single-buffered and swapped only when ky advances.  MFMA 32x32x16 bf16, 4 waves, each
// owning BM/4 output pixels x all N channels.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Loads are issued unconditionally (out-of-range chunks read the tensor base instead) and kept raw in
// registers; zero padding, the producer's BN affine + ReLU and the bf16 pack are applied when the
// chunk is written to LDS.  A per-load branch or a conversion right after the load would make hipcc
// wait vmcnt(0) at the load and serialise the HBM latency with the MFMA work.
struct RawChunk {
  u32x4 a, b;  // 8 elements: bf16 in a; f32 in a (0..3) and b (4..7)
};
template <typename TS>
__device__ __forceinline__ RawChunk load_raw(const TS* p) {
  RawChunk r;
  r.a = *reinterpret_cast<const u32x4*>(p);
  if constexpr (sizeof(TS) == 4) r.b = *reinterpret_cast<const u32x4*>(p + 4);
  else r.b = u32x4{0u, 0u, 0u, 0u};
  return r;
}
template <typename TS, bool PRE>
__device__ __forceinline__ u32x4 cook_raw(const RawChunk& r, bool ok, const float* sc, const float* sh, bool relu) {
  if (!ok) return u32x4{0u, 0u, 0u, 0u};
  if constexpr (sizeof(TS) == 2 && !PRE) return r.a;
  float f[8];
  if constexpr (sizeof(TS) == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(r.a[i] << 16); f[2 * i + 1] = __uint_as_float(r.a[i] & 0xffff0000u); }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[i] = __uint_as_float(r.a[i]); f[4 + i] = __uint_as_float(r.b[i]); }
  }
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f[i] = fmaf(f[i], sc[i], sh[i]);
      if (relu) f[i] = fmaxf(f[i], 0.f);
    }
  }
  uint32_t w4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w4[i] = pk_bf16(f[2 * i], f[2 * i + 1]);
  }
  return u32x4{w4[0], w4[1], w4[2], w4[3]};
}

struct RowArgs {
  const char* x;
  int xdt, pre;
  int n, h, w, oh, ow, kh, kw, ph, pw;
  const float* ps;
  const float* pt;
  const bf16* wt;
  int64_t ldw, N, M;
  EpiDev e;
};

template <int BM, int NB, int S, int C, int KWMAX>
struct RowCfg {
  static constexpr int CG = C / 8;                       // 16-B chunks per pixel
  static constexpr int WPX = (BM - 1) * S + KWMAX;       // window pixels
  static constexpr int HALF = (WPX + 1) / 2;
  static constexpr int NSLOT = S == 1 ? WPX : 2 * HALF;
  static constexpr int PSB = C * 2 + 16;                 // LDS bytes per pixel (conflict-free b128 reads)
  static constexpr int WBYTES = NSLOT * PSB;
  static constexpr int RSB = 128 * 2 + 16;               // weight tile row stride
  static constexpr int BBYTES = NB * RSB;
  static constexpr int WCH = (WPX * CG + NT - 1) / NT;   // window chunks per thread
  static constexpr int BCH = NB * 16 / NT;               // weight chunks per thread
  static constexpr int LDS = WBYTES + 2 * BBYTES;
};

template <int S, int HALF>
__device__ __forceinline__ int win_slot(int p) {
  if constexpr (S == 1) return p;
  else return (p & 1) * HALF + (p >> 1);
}

template <typename TS, int BM, int NB, int S, int C, int KWMAX, bool PRE>
__global__ __launch_bounds__(NT) void rowconv_kernel(RowArgs g) {
  using Cfg = RowCfg<BM, NB, S, C, KWMAX>;
  constexpr int TM = BM / 128, TN = NB / 32;
  __shared__ __attribute__((aligned(16))) char smem[Cfg::LDS > 4 * 32 * 33 * 4 ? Cfg::LDS : 4 * 32 * 33 * 4];
  char* win = smem;
  char* bbuf = smem + Cfg::WBYTES;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int x0 = blockIdx.x * BM, oy = blockIdx.y, b = blockIdx.z;
  const int KT = g.kw * C / 128;            // k-tiles per kernel row
  const int nk = g.kh * KT;
  const int px0 = x0 * S - g.pw;            // input column of window pixel 0
  const int cg = t % Cfg::CG;               // this thread's channel chunk (constant: CG | NT)

  float sc[8], sh[8];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { sc[i] = g.ps[cg * 8 + i]; sh[i] = g.pt[cg * 8 + i]; }
  }

  RawChunk wraw[Cfg::WCH];
  uint32_t wok = 0;
  u32x4 breg[Cfg::BCH];
  const bool relu = g.pre == MIA_PRE_AFFINE_RELU;

  auto load_window = [&](int ky) __attribute__((always_inline)) {
    const int iy = oy + ky - g.ph;
    const bool rowok = iy >= 0 && iy < g.h;
    const TS* xs = reinterpret_cast<const TS*>(g.x);
    wok = 0;
#pragma unroll
    for (int s = 0; s < Cfg::WCH; ++s) {
      const int q = t + NT * s;
      const int p = q / Cfg::CG;
      const int ix = px0 + p;
      const bool ok = p < Cfg::WPX && rowok && ix >= 0 && ix < g.w;
      const int64_t off = ok ? ((int64_t)(b * g.h + iy) * g.w + ix) * C + cg * 8 : 0;
      wraw[s] = load_raw<TS>(xs + off);
      wok |= (uint32_t)ok << s;
    }
  };
  auto store_window = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < Cfg::WCH; ++s) {
      const int q = t + NT * s;
      const int p = q / Cfg::CG;
      if (p < Cfg::WPX)
        *reinterpret_cast<u32x4*>(win + win_slot<S, Cfg::HALF>(p) * Cfg::PSB + cg * 16) =
            cook_raw<TS, PRE>(wraw[s], (wok >> s) & 1u, sc, sh, relu);
    }
  };
  auto load_b = [&](int kt) __attribute__((always_inline)) {
    const int64_t k0 = (int64_t)kt * 128;
#pragma unroll
    for (int s = 0; s < Cfg::BCH; ++s) {
      const int q = t + NT * s;
      const int row = q >> 4, kc = q & 15;
      breg[s] = *reinterpret_cast<const u32x4*>(g.wt + row * g.ldw + k0 + kc * 8);
    }
  };
  auto store_b = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < Cfg::BCH; ++s) {
      const int q = t + NT * s;
      const int row = q >> 4, kc = q & 15;
      *reinterpret_cast<u32x4*>(bbuf + buf * Cfg::BBYTES + row * Cfg::RSB + kc * 16) = breg[s];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_window(0);
  load_b(0);
  store_window();
  store_b(0);
  __syncthreads();

  const int g2 = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    const bool newwin = more && ((kt + 1) % KT == 0);
    if (more) load_b(kt + 1);
    if (newwin) load_window((kt + 1) / KT);
    const char* bs = bbuf + (kt & 1) * Cfg::BBYTES;
    const int kk0 = (kt % KT) * 128;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int kk = kk0 + ks * 16 + 8 * g2;
      const int kx = kk / C, ci = kk % C;
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wave * (BM / 4) + i * 32 + (lane & 31);
        int slot;
        if constexpr (S == 1) slot = r + kx;
        else slot = (kx & 1) * Cfg::HALF + r + (kx >> 1);
        fa[i] = *reinterpret_cast<const bf16x8*>(win + slot * Cfg::PSB + ci * 2);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(bs + (j * 32 + (lane & 31)) * Cfg::RSB + (ks * 16 + 8 * g2) * 2);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_b((kt + 1) & 1);
    if (newwin) {
      __syncthreads();
      store_window();
    }
    __syncthreads();
  }

  // epilogue through LDS, 16 contiguous output channels per lane
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * 33);
  const int64_t mrow0 = ((int64_t)b * g.oh + oy) * g.ow;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        stage[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = acc[i][j][r];
      __syncthreads();
      const int row = lane >> 1, c0 = (lane & 1) * 16;
      const int ox = x0 + wave * (BM / 4) + i * 32 + row;
      if (ox < g.ow) {
        float v[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] = stage[row * 33 + c0 + c];
        epi_store16(g.e, mrow0 + ox, j * 32 + c0, g.N, v);
      }
      __syncthreads();
    }
}

// -------------------------------------------------------------------------- row-window wgrad
// dW[n][ky][kx][ci] = sum_{b,oy,ox} dY[b,oy,ox,n] * X'[b, oy+ky-ph, ox*S+kx-pw, ci]  (X' = pre-op(X))
// for the same conv shapes.  Block (ky, z) walks output-row chunks of BP pixels (chunk ids
// z, z+Z, ...): it stages the dY chunk [BP px][NOUT] and the input window it touches
// [(BP-1)*S+KW px][C] in LDS, and both MFMA operands are ds_read_b64_tr_b16 transposed reads
// (dY^T rows = output channels; im2col rows = (kx, ci) columns of the window, pixel-strided).
// Accumulators stay in registers across all chunks; each block writes one f32 partial slab
// ws[z][NOUT][KH*KW*C] (its ky columns) and splitk_reduce sums the Z slabs + applies the epilogue.
struct RowWArgs {
  const char* x;
  const char* dy;
  int pre;
  int n, h, w, oh, ow, kh, kw, ph, pw;
  const float* ps;
  const float* pt;
  int Z;
  int64_t Ntot;
  float* ws;
};

template <typename T, int NOUT, int S, int C, int KWMAX, int KYB, bool PRE, bool FULL = false>
__global__ __launch_bounds__(NT) void rowwgrad_kernel(RowWArgs g) {
  constexpr int BP = 128;
  constexpr int CG = C / 8;
  constexpr int WPX = (BP - 1) * S + KWMAX;
  constexpr int HALF = (WPX + 1) / 2;
  constexpr int NSLOT = S == 1 ? WPX : 2 * HALF;
  constexpr int PSB = C == 32 ? 64 : 192;          // 16 / 48 dwords: conflict-free transposed reads
  constexpr int DSB = NOUT == 32 ? 64 : 192;
  constexpr int WBYTES = NSLOT * PSB;
  constexpr int DBYTES = BP * DSB;
  constexpr int WCH = (WPX * CG + NT - 1) / NT;
  constexpr int DCH = BP * NOUT / 8 / NT;           // 2 or 4
  constexpr int MT = NOUT / 32;
  constexpr int TPW = MT * (KWMAX * C / 32) / 4;    // accumulator tiles per wave (upper bound)
  constexpr int ES = sizeof(T);
  __shared__ __attribute__((aligned(16))) char smem[KYB * WBYTES + DBYTES];
  char* win = smem;
  char* dyt = smem + KYB * WBYTES;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ky0 = blockIdx.x * KYB, z = blockIdx.y;
  const int NC = (FULL ? KWMAX : g.kw) * C;  // columns of this ky (FULL: kw == KWMAX, tile loop static)
  const int NCT = NC / 32;
  const int ntiles = MT * NCT;
  const int CPR = (g.ow + BP - 1) / BP;
  const int64_t nchunks = (int64_t)g.n * g.oh * CPR;
  const int cg = t % CG;

  float sc[8], sh[8];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { sc[i] = g.ps[cg * 8 + i]; sh[i] = g.pt[cg * 8 + i]; }
  }

  RawChunk wraw[KYB][WCH];
  RawChunk draw[DCH];
  uint32_t wok = 0, dok = 0;
  const bool relu = g.pre == MIA_PRE_AFFINE_RELU;

  auto load_chunk = [&](int64_t c) __attribute__((always_inline)) {
    const int64_t row = c / CPR;
    const int x0 = (int)(c - row * CPR) * BP;
    const int b = (int)(row / g.oh), oy = (int)(row - (int64_t)b * g.oh);
    const T* dys = reinterpret_cast<const T*>(g.dy);
    const int64_t dbase = ((int64_t)row * g.ow + x0) * NOUT;
    dok = 0;
#pragma unroll
    for (int s = 0; s < DCH; ++s) {
      const int q = t + NT * s;
      const int p = q / (NOUT / 8), cc = q % (NOUT / 8);
      const bool ok = x0 + p < g.ow;
      draw[s] = load_raw<T>(dys + (ok ? dbase + p * NOUT + cc * 8 : 0));
      dok |= (uint32_t)ok << s;
    }
    const int px0 = x0 * S - g.pw;
    const T* xs = reinterpret_cast<const T*>(g.x);
    wok = 0;
#pragma unroll
    for (int kyi = 0; kyi < KYB; ++kyi) {
      const int iy = oy + ky0 + kyi - g.ph;
      const bool rowok = iy >= 0 && iy < g.h;
#pragma unroll
      for (int s = 0; s < WCH; ++s) {
        const int q = t + NT * s;
        const int p = q / CG;
        const int ix = px0 + p;
        const bool ok = p < WPX && rowok && ix >= 0 && ix < g.w;
        wraw[kyi][s] = load_raw<T>(xs + (ok ? ((int64_t)(b * g.h + iy) * g.w + ix) * C + cg * 8 : 0));
        wok |= (uint32_t)ok << (kyi * WCH + s);
      }
    }
  };
  auto store_chunk = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < DCH; ++s) {
      const int q = t + NT * s;
      const int p = q / (NOUT / 8), cc = q % (NOUT / 8);
      *reinterpret_cast<u32x4*>(dyt + p * DSB + cc * 16) = cook_raw<T, false>(draw[s], (dok >> s) & 1u, sc, sh, false);
    }
#pragma unroll
    for (int kyi = 0; kyi < KYB; ++kyi)
#pragma unroll
    for (int s = 0; s < WCH; ++s) {
      const int q = t + NT * s;
      const int p = q / CG;
      if (p < WPX)
        *reinterpret_cast<u32x4*>(win + kyi * WBYTES + win_slot<S, HALF>(p) * PSB + cg * 16) =
            cook_raw<T, PRE>(wraw[kyi][s], (wok >> (kyi * WCH + s)) & 1u, sc, sh, relu);
    }
  };

  f32x16 acc[KYB * TPW];
#pragma unroll
  for (int q = 0; q < KYB * TPW; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;

  const int i16 = lane & 15, gq = lane >> 4;
  int64_t c = z;
  if (c < nchunks) {
    load_chunk(c);
    store_chunk();
  }
  __syncthreads();
  for (; c < nchunks; c += g.Z) {
    const int64_t cn = c + g.Z;
    const bool more = cn < nchunks;
    if (more) load_chunk(cn);
#pragma unroll
    for (int ks = 0; ks < BP / 16; ++ks) {
      const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
      bf16x8 fa[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int col = mt * 32 + 16 * (gq & 1) + 4 * (i16 & 3);
        const char* p0 = dyt + kr * DSB + col * 2;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * DSB));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        fa[mt] = __builtin_bit_cast(bf16x8, cc);
      }
#pragma unroll
      for (int kyi = 0; kyi < KYB; ++kyi)
#pragma unroll
      for (int q = 0; q < TPW; ++q) {
        const int tile = wave + 4 * q;
        if (tile < ntiles) {
          const int mt = tile / NCT, nt = tile - mt * NCT;
          const int col = nt * 32 + 16 * (gq & 1);
          const int kx = col / C, ci = col % C + 4 * (i16 & 3);
          int slot;
          if constexpr (S == 1) slot = kr + kx;
          else slot = (kx & 1) * HALF + kr + (kx >> 1);
          const char* p0 = win + kyi * WBYTES + slot * PSB + ci * 2;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * PSB));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8 fb = __builtin_bit_cast(bf16x8, cc);
          bf16x8 a = fa[0];
          if constexpr (MT > 1) if (mt == 1) a = fa[1];
          acc[kyi * TPW + q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, fb, acc[kyi * TPW + q], 0, 0, 0);
        }
      }
    }
    __syncthreads();
    if (more) {
      store_chunk();
      __syncthreads();
    }
  }

  // partial slab: ws[z][m][ky*NC + n]
#pragma unroll
  for (int kyi = 0; kyi < KYB; ++kyi) {
  float* dst = g.ws + (int64_t)z * NOUT * g.Ntot + (int64_t)(ky0 + kyi) * NC;
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    const int tile = wave + 4 * q;
    if (tile < ntiles) {
      const int mt = tile / NCT, nt = tile - mt * NCT;
      const int n = nt * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        dst[(int64_t)m * g.Ntot + n] = acc[kyi * TPW + q][r];
      }
    }
  }
  }
}

bool rowwgrad_ok(const MiaOperand& A, const MiaOperand& B, int64_t M, int64_t N, int64_t K, int compute, int split) {
  if (compute != MIA_BF16 || split < 2) return false;
  if (A.kind != MIA_OP_DENSE || A.layout != MIA_LAYOUT_RC || A.pre != MIA_PRE_NONE) return false;
  if (B.kind != MIA_OP_CONV || B.layout != MIA_LAYOUT_RC || B.sh != 1 || (B.sw != 1 && B.sw != 2)) return false;
  if (A.dtype != B.dtype || (A.dtype != MIA_BF16 && A.dtype != MIA_F32)) return false;
  if (M != 32 && M != 64) return false;
  if (A.rows != K || A.cols != M || A.ld != M) return false;
  if (B.c != 32 && B.c != 64) return false;
  if (B.c == 64 && B.sw != 1) return false;
  if (B.kw > (B.sw == 1 ? 8 : 16) || (B.kw * B.c) % 128 != 0) return false;
  if (B.pre != MIA_PRE_NONE && B.pre != MIA_PRE_AFFINE && B.pre != MIA_PRE_AFFINE_RELU) return false;
  if (N != (int64_t)B.kh * B.kw * B.c || K != (int64_t)B.n * B.oh * B.ow) return false;
  if (B.kh > 65535 || split > 65535) return false;
  if ((reinterpret_cast<uintptr_t>(A.ptr) | reinterpret_cast<uintptr_t>(B.ptr)) & 15) return false;
  return true;
}

template <typename T, int NOUT, int S, int C, int KWMAX, int KYB = 1>
hipError_t rowwgrad_launch2(const RowWArgs& r, bool pre, hipStream_t s) {
  dim3 grid((unsigned)(r.kh / KYB), (unsigned)r.Z);
  if (r.kw == KWMAX) {
    if (pre) rowwgrad_kernel<T, NOUT, S, C, KWMAX, KYB, true, true><<<grid, NT, 0, s>>>(r);
    else rowwgrad_kernel<T, NOUT, S, C, KWMAX, KYB, false, true><<<grid, NT, 0, s>>>(r);
  } else {
    if (pre) rowwgrad_kernel<T, NOUT, S, C, KWMAX, KYB, true><<<grid, NT, 0, s>>>(r);
    else rowwgrad_kernel<T, NOUT, S, C, KWMAX, KYB, false><<<grid, NT, 0, s>>>(r);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t rowwgrad_launch1(const RowWArgs& r, int NOUT, int S, int C, bool pre, hipStream_t s) {
  if (S == 2) {
    if (NOUT == 64) return rowwgrad_launch2<T, 64, 2, 32, 16>(r, pre, s);
    return rowwgrad_launch2<T, 32, 2, 32, 16>(r, pre, s);
  }
  if (C == 64) {
    if (NOUT == 64) return rowwgrad_launch2<T, 64, 1, 64, 8>(r, pre, s);
    return rowwgrad_launch2<T, 32, 1, 64, 8>(r, pre, s);
  }
  if (NOUT == 64) return rowwgrad_launch2<T, 64, 1, 32, 8>(r, pre, s);
  if (r.kh % 4 == 0) return rowwgrad_launch2<T, 32, 1, 32, 8, 4>(r, pre, s);  // conv4: dY chunk shared by 4 ky
  return rowwgrad_launch2<T, 32, 1, 32, 8>(r, pre, s);
}

// -------------------------------------------------------------------------- single-channel tap wgrad
// dW[n][ky][kx] = sum_{b,oy,ox} dY[b,oy,ox,n] * X[b, oy+ky, S*ox+kx]  for the 1-channel convs of
// EnvNet-v2 (frontend conv1: 1x64 taps, stride 2 over the waveform; trunk conv3: 8x8 taps over the
// 64 x Wp image).  N = 32 output channels, KH*KW = 64 taps.  Per chunk of BP output pixels the
// block stages the dY tile [BP][32] (transposed MFMA reads) and, for every (ky, parity) tap
// sequence seq[i] = X[oy+ky][S*(x0+i)+par], 8 copies shifted by 0..7 elements so that the 8
// consecutive output pixels an MFMA k-group needs (X[..][S*(ox..ox+7)+kx]) are one aligned
// 16-byte LDS read whatever the tap offset.  The 4 waves split the chunk's k-steps; partials are
// summed through LDS into one f32 slab per block (ws[z][32][64]) -> splitk_reduce.
struct TapWArgs {
  const char* x;
  const char* dy;
  int n, h, wx, oh, ow;
  int Z;
  float* ws;
  // BNB (single pass, BN-backward reductions not yet known): dy is the gradient w.r.t. relu(bn(y));
  // the kernel stages dz = mask(y) * dy and y itself as two A operands and accumulates
  //   G1 = sum dz x,  G3 = sum y x   (slabs ws[z][2][32][64])
  // and per channel sum dz, sum dz*xhat, sum y (dbp[z][32][3]).  The BN-input gradient is linear,
  //   g = A dz + B + C y  (A = gamma*invstd, B = -A*dbeta/P + A*invstd*mean*dgamma/P, C = -A*invstd*dgamma/P),
  // so dW = A G1 + B G2 + C G3 with G2[k] = sum x[2p+k] (fe_conv1_lin_final).
  const bf16* by;
  const float *bsc, *bsh, *bmean, *binvstd;
  float* dbp;
  int64_t bP;
};

template <typename TD, typename TX, int S, int KH, int KW, bool BNB = false>
__global__ __launch_bounds__(NT) void tapwgrad_kernel(TapWArgs g) {
  constexpr int BP = 256;
  constexpr int NS = KW / S;                       // taps per parity sequence
  constexpr int LP = (BP + NS + 7) / 8 * 8;        // copy length
  constexpr int LR = LP + 8;                       // raw length (covers shift 7)
  constexpr int NSEQ = KH * S;
  constexpr int CPB = LP * 2;                      // bytes per shifted copy
  constexpr int SQB = 8 * CPB + 16;                // bytes per sequence (+16: parity banks)
  constexpr int DYB = BP * 64;                     // dY tile [BP][32] bf16
  constexpr int RAWB = NSEQ * LR * 2;
  constexpr int CPYB = NSEQ * SQB;
  constexpr int MAINB0 = DYB + RAWB + CPYB;
  constexpr int MAINB = MAINB0 + (BNB ? DYB : 0);
  constexpr int REDB = 4 * 32 * 64 * 4;
  constexpr int RCH = (NSEQ * LR + NT - 1) / NT;
  constexpr int DCH = BP * 32 / 8 / NT;            // 4
  static_assert(KH * KW == 64, "64 taps");
  __shared__ __attribute__((aligned(16))) char smem[MAINB > REDB ? MAINB : REDB];
  char* dyt = smem;
  bf16* raw = reinterpret_cast<bf16*>(smem + DYB);
  char* cpy = smem + DYB + RAWB;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int z = blockIdx.x;
  const int CPR = (g.ow + BP - 1) / BP;
  const int64_t nchunks = (int64_t)g.n * g.oh * CPR;
  const TD* dys = reinterpret_cast<const TD*>(g.dy);
  const TX* xs = reinterpret_cast<const TX*>(g.x);

  u32x4 dreg[DCH];
  float rreg[RCH];
  u32x4 yreg[BNB ? DCH : 1];
  uint32_t dok = 0;
  float bsc[8], bsh[8], bmu[8], bis[8], sdz[8], sdx[8], sy[8];
  if constexpr (BNB) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ch = (t & 3) * 8 + i;
      bsc[i] = g.bsc[ch];
      bsh[i] = g.bsh[ch];
      bis[i] = g.binvstd[ch];
      bmu[i] = g.bmean[ch];
      sdz[i] = 0.f; sdx[i] = 0.f; sy[i] = 0.f;
    }
  }
  char* yt = smem + MAINB0;  // BNB: second A tile (y), [BP][32] bf16

  auto load_chunk = [&](int64_t c) __attribute__((always_inline)) {
    const int64_t row = c / CPR;
    const int x0 = (int)(c - row * CPR) * BP;
    const int b = (int)(row / g.oh), oy = (int)(row - (int64_t)b * g.oh);
    const TD* src = dys + ((int64_t)row * g.ow + x0) * 32;
    dok = 0;
#pragma unroll
    for (int s2 = 0; s2 < DCH; ++s2) {
      const int q = t + NT * s2;
      const int p = q >> 2, cc = q & 3;
      u32x4 v = {0u, 0u, 0u, 0u};
      if constexpr (BNB) {
        const bool ok = x0 + p < g.ow;
        const int64_t off = ok ? ((int64_t)row * g.ow + x0 + p) * 32 + cc * 8 : 0;
        dreg[s2] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16*>(g.dy) + off);
        yreg[s2] = *reinterpret_cast<const u32x4*>(g.by + off);
        dok |= (uint32_t)ok << s2;
        continue;
      }
      if (x0 + p < g.ow) {
        if constexpr (sizeof(TD) == 2) {
          v = *reinterpret_cast<const u32x4*>(src + p * 32 + cc * 8);
        } else {
          const float4 a = reinterpret_cast<const float4*>(src + p * 32 + cc * 8)[0];
          const float4 d = reinterpret_cast<const float4*>(src + p * 32 + cc * 8)[1];
          const float f[8] = {a.x, a.y, a.z, a.w, d.x, d.y, d.z, d.w};
          uint32_t w4[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            w4[i] = pk_bf16(f[2 * i], f[2 * i + 1]);
          }
          v = u32x4{w4[0], w4[1], w4[2], w4[3]};
        }
      }
      dreg[s2] = v;
    }
#pragma unroll
    for (int s2 = 0; s2 < RCH; ++s2) {
      const int e = t + NT * s2;
      float v = 0.f;
      if (e < NSEQ * LR) {
        const int seq = e / LR, i = e - seq * LR;
        const int ky = seq / S, par = seq - ky * S;
        const int iy = oy + ky;
        const int ix = S * (x0 + i) + par;
        if (iy < g.h && ix < g.wx) v = (float)xs[((int64_t)b * g.h + iy) * g.wx + ix];
      }
      rreg[s2] = v;
    }
  };
  auto store_chunk = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s2 = 0; s2 < DCH; ++s2) {
      const int q = t + NT * s2;
      u32x4 v = dreg[s2];
      if constexpr (BNB) {
        uint32_t w4[4] = {0u, 0u, 0u, 0u}, y4[4] = {0u, 0u, 0u, 0u};
        if ((dok >> s2) & 1u) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float gv[2], yv[2];
            gv[0] = __uint_as_float(dreg[s2][i] << 16);
            gv[1] = __uint_as_float(dreg[s2][i] & 0xffff0000u);
            yv[0] = __uint_as_float(yreg[s2][i] << 16);
            yv[1] = __uint_as_float(yreg[s2][i] & 0xffff0000u);
            uint32_t m = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int c = 2 * i + h;
              const bool on = fmaf(yv[h], bsc[c], bsh[c]) > 0.f;
              const float d = on ? gv[h] : 0.f;
              sdz[c] += d;
              sdx[c] = fmaf(d, (yv[h] - bmu[c]) * bis[c], sdx[c]);
              sy[c] += yv[h];
              m |= on ? (0xffffu << (16 * h)) : 0u;
            }
            w4[i] = dreg[s2][i] & m;  // dz = mask * dy exactly (bf16 bits kept or zeroed)
            y4[i] = yreg[s2][i];
          }
        }
        v = u32x4{w4[0], w4[1], w4[2], w4[3]};
        *reinterpret_cast<u32x4*>(yt + (q >> 2) * 64 + (q & 3) * 16) = u32x4{y4[0], y4[1], y4[2], y4[3]};
      }
      *reinterpret_cast<u32x4*>(dyt + (q >> 2) * 64 + (q & 3) * 16) = v;
    }
#pragma unroll
    for (int s2 = 0; s2 < RCH; ++s2) {
      const int e = t + NT * s2;
      if (e < NSEQ * LR) raw[e] = (bf16)rreg[s2];
    }
  };
  auto build_copies = [&]() __attribute__((always_inline)) {
    constexpr int PIECES = NSEQ * 8 * (LP / 8);
    for (int pc = t; pc < PIECES; pc += NT) {
      const int seq = pc / (8 * (LP / 8));
      const int rem = pc - seq * 8 * (LP / 8);
      const int sh = rem / (LP / 8), blk = rem - sh * (LP / 8);
      const unsigned short* r = reinterpret_cast<const unsigned short*>(raw) + seq * LR + blk * 8 + sh;
      uint32_t w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) w4[i] = (uint32_t)r[2 * i] | ((uint32_t)r[2 * i + 1] << 16);
      *reinterpret_cast<u32x4*>(cpy + seq * SQB + sh * CPB + blk * 16) = u32x4{w4[0], w4[1], w4[2], w4[3]};
    }
  };

  f32x16 acc[2], acc3[BNB ? 2 : 1];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  if constexpr (BNB) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc3[j][r] = 0.f;
  }

  const int i16 = lane & 15, gq = lane >> 4, g2 = lane >> 5;
  // this lane's tap per n-tile: n = nt*32 + (lane&31) -> (ky, kx) -> (seq, j)
  int bseq[2], bj[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = nt * 32 + (lane & 31);
    const int ky = n / KW, kx = n - ky * KW;
    bseq[nt] = ky * S + kx % S;
    bj[nt] = kx / S;
  }

  int64_t c = z;
  if (c < nchunks) {
    load_chunk(c);
    store_chunk();
  }
  __syncthreads();
  if (c < nchunks) build_copies();
  __syncthreads();
  for (; c < nchunks; c += g.Z) {
    const int64_t cn = c + g.Z;
    const bool more = cn < nchunks;
    if (more) load_chunk(cn);
#pragma unroll
    for (int kk = 0; kk < BP / 16 / 4; ++kk) {
      const int ks = wave + 4 * kk;
      const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
      const int col = 16 * (gq & 1) + 4 * (i16 & 3);
      const char* p0 = dyt + kr * 64 + col * 2;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * 64));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const bf16x8 fa = __builtin_bit_cast(bf16x8, cc);
      bf16x8 fy;
      if constexpr (BNB) {
        const char* py = yt + kr * 64 + col * 2;
        const s16x4 ylo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(py));
        const s16x4 yhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(py + 4 * 64));
        const s16x8 yc = {ylo[0], ylo[1], ylo[2], ylo[3], yhi[0], yhi[1], yhi[2], yhi[3]};
        fy = __builtin_bit_cast(bf16x8, yc);
      }
      const int ox0 = ks * 16 + 8 * g2;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int q = ox0 + bj[nt];
        const int sh = q & 7;
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(cpy + bseq[nt] * SQB + sh * CPB + (q - sh) * 2);
        acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[nt], 0, 0, 0);
        if constexpr (BNB) acc3[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fy, fb, acc3[nt], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      store_chunk();
      __syncthreads();
      build_copies();
      __syncthreads();
    }
  }

  // sum the 4 waves' partials, write the block's slab ws[z][32][64] (BNB: ws[z][2][32][64], G1 then G3)
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int which = 0; which < (BNB ? 2 : 1); ++which) {
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (r & 3) + 8 * (r >> 2) + 4 * g2;
        float v = acc[nt][r];
        if constexpr (BNB) if (which) v = acc3[nt][r];
        red[(wave * 32 + m) * 64 + nt * 32 + (lane & 31)] = v;
      }
    __syncthreads();
    float* dst = g.ws + ((int64_t)z * (BNB ? 2 : 1) + which) * 32 * 64;
    for (int e = t; e < 32 * 64; e += NT)
      dst[e] = red[e] + red[2048 + e] + red[4096 + e] + red[6144 + e];
  }
  if constexpr (BNB) {
    // per-channel sums of this block: channel c = (t&3)*8 + i summed over the 64 threads of its
    // group in thread order (deterministic) -> dbp[z][c][0..2] = (sum dz, sum dz*xhat, sum y)
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[t * 8 + i] = sdz[i];
      red[2048 + t * 8 + i] = sdx[i];
      red[4096 + t * 8 + i] = sy[i];
    }
    __syncthreads();
    if (t < 96) {
      const int q = t / 32, ch = t % 32, cg = ch >> 3, i = ch & 7;
      float a = 0.f;
      for (int k = 0; k < NT / 4; ++k) a += red[q * 2048 + (k * 4 + cg) * 8 + i];
      g.dbp[((int64_t)z * 32 + ch) * 3 + q] = a;
    }
  }
}

// 1-channel conv wgrad (path 3): A = dY [P][32] as RC, B = CONVROW/RC with c == 1 (any stride
// (1,1), kh*kw == 64) or the c == 2 stride-1 pair view of a stride-2 1-D conv (kw*2 == 64).
bool tapwgrad_ok(const MiaOperand& A, const MiaOperand& B, int64_t M, int64_t N, int64_t K, int compute, int split) {
  if (compute != MIA_BF16 || split < 2 || M != 32 || N != 64) return false;
  if (A.kind != MIA_OP_DENSE || A.layout != MIA_LAYOUT_RC || A.pre != MIA_PRE_NONE) return false;
  if (A.dtype != MIA_BF16 && A.dtype != MIA_F32) return false;
  if (A.rows != K || A.cols != 32 || A.ld != 32) return false;
  if (B.kind != MIA_OP_CONVROW || B.layout != MIA_LAYOUT_RC || B.pre != MIA_PRE_NONE) return false;
  if (B.dtype != MIA_BF16 && B.dtype != MIA_F32) return false;
  if (B.sh != 1 || B.sw != 1 || B.ph != 0 || B.pw != 0) return false;
  if (K != (int64_t)B.n * B.oh * B.ow) return false;
  const bool conv1 = B.c == 2 && B.kh == 1 && B.kw == 32 && B.h == 1;
  const bool conv3 = B.c == 1 && B.kh == 8 && B.kw == 8;
  if (!conv1 && !conv3) return false;
  if (conv1 && B.dtype != MIA_F32) return false;
  if ((reinterpret_cast<uintptr_t>(A.ptr) & 15)) return false;
  return true;
}

template <typename TD, typename TX, int S, int KH, int KW, bool BNB = false>
hipError_t tapwgrad_launch(const TapWArgs& r, hipStream_t s) {
  tapwgrad_kernel<TD, TX, S, KH, KW, BNB><<<(unsigned)r.Z, NT, 0, s>>>(r);
  return hipGetLastError();
}

// -------------------------------------------------------------------------- single-channel tap conv (fwd)
// y[b,oy,ox,n] = sum_{ky,kx} W[n][ky][kx] * X[b, oy+ky, S*ox+kx]  (+ epilogue) for conv1 (1x64,
// stride 2 over the f32 waveform) and conv3 (8x8 over the 1-channel trunk image): K = 64 taps,
// N = 32.  A block owns BP output pixels of one row; it stages the KH input row segments it reads
// and 8 copies of each shifted by 0..7 samples, so that every MFMA A fragment (8 consecutive taps
// = 8 consecutive samples at any offset) is one aligned ds_read_b128.  Weight fragments are read
// once per wave straight from global memory (4 KB, L2-resident).  Output is HBM-write-bound.
struct TapArgs {
  const char* x;
  int n, h, wx, oh, ow;
  const bf16* wt;
  EpiDev e;
};

template <typename TX, int S, int KH, int KW>
__global__ __launch_bounds__(NT) void tapconv_kernel(TapArgs g) {
  constexpr int BP = 256;
  constexpr int RAWL = S * (BP - 1) + KW;
  constexpr int LP = (RAWL + 7) / 8 * 8;     // copy length
  constexpr int LR = LP + 8;                 // raw length
  constexpr int CPB = LP * 2 + 16;           // bytes per copy (8-dword bank offset per copy)
  constexpr int RAWB = KH * LR * 2;
  constexpr int CPYB = KH * 8 * CPB;
  constexpr int MAINB = RAWB + CPYB;
  constexpr int STB = 4 * 32 * 33 * 4;
  static_assert(KH * KW == 64, "64 taps");
  __shared__ __attribute__((aligned(16))) char smem[MAINB > STB ? MAINB : STB];
  bf16* raw = reinterpret_cast<bf16*>(smem);
  char* cpy = smem + RAWB;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, g2 = lane >> 5;
  const int CPR = (g.ow + BP - 1) / BP;
  const int64_t row = blockIdx.x / CPR;
  const int x0 = (int)(blockIdx.x - row * CPR) * BP;
  const int b = (int)(row / g.oh), oy = (int)(row - (int64_t)b * g.oh);
  const TX* xs = reinterpret_cast<const TX*>(g.x);

  for (int e = t; e < KH * LR; e += NT) {
    const int ky = e / LR, i = e - ky * LR;
    const int iy = oy + ky, ix = S * x0 + i;
    float v = 0.f;
    if (i < RAWL && iy < g.h && ix < g.wx) v = (float)xs[((int64_t)b * g.h + iy) * g.wx + ix];
    raw[e] = (bf16)v;
  }
  // weight fragments: k-step ks covers taps ks*16 .. +15, lane holds 8 of them for column lane&31
  bf16x8 fb[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    fb[ks] = *reinterpret_cast<const bf16x8*>(g.wt + (lane & 31) * 64 + ks * 16 + 8 * g2);
  __syncthreads();
  for (int pc = t; pc < KH * 8 * (LP / 8); pc += NT) {
    const int ky = pc / (8 * (LP / 8));
    const int rem = pc - ky * 8 * (LP / 8);
    const int sh = rem / (LP / 8), blk = rem - sh * (LP / 8);
    const unsigned short* r = reinterpret_cast<const unsigned short*>(raw) + ky * LR + blk * 8 + sh;
    uint32_t w4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w4[i] = (uint32_t)r[2 * i] | ((uint32_t)r[2 * i + 1] << 16);
    *reinterpret_cast<u32x4*>(cpy + (ky * 8 + sh) * CPB + blk * 16) = u32x4{w4[0], w4[1], w4[2], w4[3]};
  }
  __syncthreads();

  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const int rel = wave * 64 + i * 32 + (lane & 31);   // pixel within the chunk
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k0 = ks * 16 + 8 * g2;
      const int ky = k0 / KW, kx0 = k0 - ky * KW;
      const int q = S * rel + kx0;
      const int sh = q & 7;
      const bf16x8 fa = *reinterpret_cast<const bf16x8*>(cpy + (ky * 8 + sh) * CPB + (q - sh) * 2);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb[ks], acc[i], 0, 0, 0);
    }
  }
  __syncthreads();
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * 33);
  const int64_t mrow0 = row * g.ow;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      stage[((r & 3) + 8 * (r >> 2) + 4 * g2) * 33 + (lane & 31)] = acc[i][r];
    __syncthreads();
    const int prow = lane >> 1, c0 = (lane & 1) * 16;
    const int ox = x0 + wave * 64 + i * 32 + prow;
    if (ox < g.ow) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = stage[prow * 33 + c0 + c];
      epi_store16(g.e, mrow0 + ox, c0, 32, v);
    }
    __syncthreads();
  }
}

bool tapconv_ok(const MiaOperand& A, const MiaOperand& B, int64_t M, int64_t N, int64_t K, int compute, int split) {
  if (compute != MIA_BF16 || split > 1 || N != 32 || K != 64) return false;
  if (A.kind != MIA_OP_CONVROW || A.layout != MIA_LAYOUT_KC || A.pre != MIA_PRE_NONE) return false;
  if (A.dtype != MIA_BF16 && A.dtype != MIA_F32) return false;
  if (A.sh != 1 || A.sw != 1 || A.ph != 0 || A.pw != 0) return false;
  const bool conv1 = A.c == 2 && A.kh == 1 && A.kw == 32 && A.h == 1 && A.dtype == MIA_F32;
  const bool conv3 = A.c == 1 && A.kh == 8 && A.kw == 8;
  if (!conv1 && !conv3) return false;
  if (M != (int64_t)A.n * A.oh * A.ow) return false;
  if (B.kind != MIA_OP_DENSE || B.layout != MIA_LAYOUT_KC || B.dtype != MIA_BF16) return false;
  if (B.rows != 32 || B.cols != 64 || B.ld != 64 || (reinterpret_cast<uintptr_t>(B.ptr) & 15)) return false;
  return true;
}

// -------------------------------------------------------------------------- dense bf16 GEMM (LDS-DMA)
// C = A . B^T for bf16 DENSE operands in any KC/RC layout combination (AST linears fwd/dgrad/wgrad,
// EnvNet FC layers).  128x128x64 tiles, 4 waves (2x2, 64x64 each, MFMA 32x32x16), both operands
// staged global -> LDS with global_load_lds_dwordx4 (no register staging, no VALU address work
// in the loop beyond a pointer bump), double-buffered: the next K-tile's DMA is issued before the
// current tile's MFMAs, retired with a counted vmcnt + raw s_barrier.  LDS images are XOR-swizzled
// on the SOURCE address (the DMA destination is lane-linear): KC rows of 128 B permute their 16-B
// chunks by (row & 7) (conflict-free ds_read_b128 per 8 lanes); RC rows of 256 B permute their
// 32-B blocks by (k & 3) (conflict-free ds_read_b64_tr_b16 per 16 lanes).  Blocks are remapped so
// that neighbouring tiles share an XCD (bijective XCD swizzle) and walk M fastest (B-tile reuse).


typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;

// block-wide sum of one double per thread (4 waves), written by thread 0: a tile's sum of squares.
// `red` is NT/64 doubles of the caller's LDS (inside a GEMM kernel: its one staging array -- a second
// __shared__ object there makes hipcc wait vmcnt(0) at every K-step barrier); the leading barrier
// lets the caller's last reads of that space finish first.
__device__ __forceinline__ void tile_sqsum_store(double* dst, double v, double* red) {
  v = wave_sum_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    *dst = s;
  }
}

// MiaEpilogue.sqsum for a GEMM whose kernel did not produce it (other paths, split-K): one block
// per 128 x 128 tile of the f32 output C (ldc), same slots and per-tile order of accumulation
__global__ __launch_bounds__(NT) void tile_sqsum_kernel(const float* __restrict__ c, int64_t ldc, int64_t M, int64_t N,
                                                        int nbn, double* __restrict__ out) {
  const int bm = blockIdx.x / nbn, bn = blockIdx.x - (blockIdx.x / nbn) * nbn;
  const int64_t m0 = (int64_t)bm * 128, n0 = (int64_t)bn * 128;
  float sq = 0.f;
  for (int e = threadIdx.x; e < 128 * 128; e += NT) {
    const int64_t m = m0 + e / 128, n = n0 + e % 128;
    if (m < M && n < N) {
      const float v = c[m * ldc + n];
      sq = fmaf(v, v, sq);
    }
  }
  __shared__ double red[NT / 64];
  tile_sqsum_store(out + blockIdx.x, (double)sq, red);
}

// 16-B chunk swizzle of the k-contiguous (KC) 128 x 64 tile images: chunk c of row r sits at c ^ swz(r).
// A 32-row fragment's ds_read_b128 lane groups ({0-3, 12-15, 20-27} and its complement) hold rows 8 and
// 24 apart, which r & 7 maps to the same chunk of the same bank half (2-way conflicts); (r >> 1) & 7 gives
// the 8 even and the 8 odd rows of each group distinct chunks
__device__ __forceinline__ int dkc_swz(int r) { return (r >> 1) & 7; }

template <int L>
struct DLoader {
  // per-lane source pointers for this wave's 4 DMA instructions of a tile, advanced per K-tile
  const bf16* src[4];
  int64_t step;
  __device__ __forceinline__ void init(const bf16* base, int64_t ld, int64_t rows_or_cols, int64_t r0, int64_t kbeg,
                                       int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = wave * 4 + i;
      if constexpr (L == MIA_LAYOUT_KC) {
        const int r = 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ dkc_swz(r);
        int64_t row = r0 + r;
        if (row >= rows_or_cols) row = rows_or_cols - 1;
        src[i] = base + row * ld + kbeg + c * 8;
      } else {
        const int kr = 4 * j + (lane >> 4);
        const int p = lane & 15;
        const int c = 2 * ((p >> 1) ^ (kr & 3)) + (p & 1);
        int64_t col = r0 + c * 8;
        if (col + 8 > rows_or_cols) col = rows_or_cols - 8;
        src[i] = base + (kbeg + kr) * ld + col;
      }
    }
    step = L == MIA_LAYOUT_KC ? 64 : 64 * ld;
  }
  __device__ __forceinline__ void issue(char* tile, int wave) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_global_load_lds((glb_vp)src[i], (lds_vp)(tile + (wave * 4 + i) * 1024), 16, 0, 0);
      src[i] += step;
    }
  }
};

template <int L>
__device__ __forceinline__ bf16x8 dfrag(const char* tile, int rbase, int ks, int lane) {
  if constexpr (L == MIA_LAYOUT_KC) {
    const int rr = rbase + (lane & 31);
    const int c = 2 * ks + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(tile + rr * 128 + ((c ^ dkc_swz(rr)) * 16));
  } else {
    const int i16 = lane & 15, gq = lane >> 4;
    const int col = rbase + 16 * (gq & 1) + 4 * (i16 & 3);
    const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
    const char* p0 = tile + kr * 256 + (((col >> 4) ^ (kr & 3)) * 32) + (col & 15) * 2;
    // (hipcc waits vmcnt(0) -- for the next tile's DMA -- before the first of these builtin reads in
    // each K-step; an inline-asm variant without that wait measured the same on the wgrad shapes)
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * 256));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, cc);
  }
}


template <int LA, int LB, bool ADAM = false>
__global__ __launch_bounds__(NT) void dgemm_kernel(DArgs g) {
  constexpr int TILE = 128 * 64 * 2;
  __shared__ __attribute__((aligned(1024))) char smem[4 * TILE];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = g.nbm * g.nbn;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  int bm, bn;
  if (g.nfast) {  // grouped order: gm row blocks x all column tiles, M fastest inside a group
    const int gsize = g.gm * g.nbn;
    const int grp = wgid / gsize, rem = wgid - grp * gsize;
    const int gme = min(g.gm, g.nbm - grp * g.gm);
    bm = grp * g.gm + rem % gme;
    bn = rem / gme;
  } else {
    bm = wgid % g.nbm;
    bn = wgid / g.nbm;
  }
  const int64_t m0 = (int64_t)bm * 128, n0 = (int64_t)bn * 128;
  const int z = blockIdx.y;
  const int64_t kbeg = (int64_t)z * g.kper;
  int64_t kend = kbeg + g.kper;
  if (kend > g.K) kend = g.K;
  const int nk = kend > kbeg ? (int)((kend - kbeg) / 64) : 0;

  DLoader<LA> la;
  DLoader<LB> lb;
  la.init(g.a, g.lda, LA == MIA_LAYOUT_KC ? g.M : g.M, m0, kbeg, wave, lane);
  lb.init(g.b, g.ldb, g.N, n0, kbeg, wave, lane);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fused Adam (mode 2): the parameter rows of the tile's first 16-B group per lane -- p / m / v -- are
  // fetched before the main loop, so their HBM latency hides under it; later groups are fetched one
  // group ahead of their use in the epilogue
  f32x4 pv[2][4], mv[2][4], vv[2][4];
  const int acol = (lane & 31) * 4;
  auto adam_fetch = [&](int it0, int b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t off = (m0 + wave * 32 + (it0 + u) * 2 + (lane >> 5)) * g.adam.ld + n0 + acol;
      pv[b][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g.adam.p + off));
      mv[b][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g.adam.m + off));
      vv[b][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g.adam.v + off));
    }
  };
  if constexpr (ADAM) adam_fetch(0, 0);

  if (nk > 0) {
    la.issue(smem, wave);
    lb.issue(smem + TILE, wave);
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * 2 * TILE;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * 2 * TILE;
      la.issue(nxt, wave);
      lb.issue(nxt + TILE, wave);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* As = cur;
    const char* Bs = cur + TILE;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = dfrag<LA>(As, wm * 64 + i * 32, ks, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = dfrag<LB>(Bs, wn * 64 + j * 32, ks, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // plain f32 output of a full tile (the wide weight-gradient GEMMs, e.g. EnvNet FC1: 1.38 GB of f32
  // per step): the whole 128x128 tile is staged in the (now idle) 64 KB of LDS and written as whole
  // 512-B rows, two rows per wave store instruction, non-temporal (read next by the optimizer pass)
  const bool plain = ADAM || g.mode != 0 ||
                     (g.split == 1 && g.e.dtype == MIA_F32 && g.e.act == MIA_ACT_NONE && !g.e.bias &&
                      !g.e.accumulate && !g.e.rm_inner && g.e.alpha == 1.f && m0 + 128 <= g.M && n0 + 128 <= g.N &&
                      (g.e.ldc & 3) == 0 && ((reinterpret_cast<uintptr_t>(g.e.ptr)) & 15) == 0);
  if (plain) {
    // the tile's sum of squares straight from the accumulators (one fixed order shared by the stored
    // and the sums-only forms, so a deferred gradient's norm equals the materialised one's bit for bit)
    float sq = 0.f;
    if (g.e.sqsum) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) sq = fmaf(acc[i][j][r], acc[i][j][r], sq);
    }
    if (g.mode == 1) {  // sums only: nothing staged, nothing stored
      tile_sqsum_store(g.e.sqsum + (int64_t)bm * g.nbn + bn, (double)sq, reinterpret_cast<double*>(smem));
      return;
    }
    float* tile = reinterpret_cast<float*>(smem);  // [128][128], 32-dword halves swapped on row bit 2
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int col = wn * 64 + j * 32 + (lane & 31);
          tile[row * 128 + (col ^ (((row >> 2) & 1) << 5))] = acc[i][j][r];
        }
    __syncthreads();
    if constexpr (ADAM) {
      // Adam on the parameter rows this tile is the gradient of (torch single-tensor Adam, exactly
      // adam_kernel's arithmetic; the gradient is the f32 product itself, which is never stored)
      const DArgs::AdamEpi& A = g.adam;
      const float coef = A.coef[0];
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {
        const int b = grp & 1;
        if (grp + 1 < 4) adam_fetch((grp + 1) * 4, b ^ 1);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int row = wave * 32 + (grp * 4 + u) * 2 + (lane >> 5);
          const int64_t off = (m0 + row) * A.ld + n0 + acol;
          const f32x4 gv = *reinterpret_cast<const f32x4*>(tile + row * 128 + (acol ^ (((row >> 2) & 1) << 5)));
          f32x4 p4 = pv[b][u], m4 = mv[b][u], v4 = vv[b][u];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gg = fmaf(A.wd, p4[e], gv[e] * coef);
            m4[e] = m4[e] + (1.f - A.beta1) * (gg - m4[e]);
            v4[e] = fmaf((1.f - A.beta2) * gg, gg, v4[e] * A.beta2);
            const float denom = sqrtf(v4[e]) / A.bc2_sqrt + A.eps;
            p4[e] = p4[e] - A.lr_over_bc1 * (m4[e] / denom);
          }
          __builtin_nontemporal_store(p4, reinterpret_cast<f32x4*>(A.p + off));
          __builtin_nontemporal_store(m4, reinterpret_cast<f32x4*>(A.m + off));
          __builtin_nontemporal_store(v4, reinterpret_cast<f32x4*>(A.v + off));
          if (A.shadow) {
            const bf16x4 b4 = {(bf16)p4[0], (bf16)p4[1], (bf16)p4[2], (bf16)p4[3]};
            __builtin_nontemporal_store(b4, reinterpret_cast<bf16x4*>(A.shadow + off));
          }
        }
      }
      return;
    }
    float* out = reinterpret_cast<float*>(g.e.ptr);
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int row = wave * 32 + it * 2 + (lane >> 5);
      const int col = (lane & 31) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(tile + row * 128 + (col ^ (((row >> 2) & 1) << 5)));
      __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out + (m0 + row) * g.e.ldc + n0 + col));
    }
    if (g.e.sqsum) tile_sqsum_store(g.e.sqsum + (int64_t)bm * g.nbn + bn, (double)sq, reinterpret_cast<double*>(smem));
    return;
  }
  // the same full-tile staging for a bf16 output with optional bias / ReLU (AST qkv forward and the
  // plain backward-data GEMMs): 16 lanes cover one 256-B output row, 4 rows per store instruction
  const bool save = g.e.act == MIA_ACT_GELU_SAVE || g.e.act == MIA_ACT_GELU_SAVE_D;
  const bool save_d = g.e.act == MIA_ACT_GELU_SAVE_D;
  // drop-mode row map (MIA_RM_DROP): plain / bias / ReLU output only
  const bool drop = g.e.rm_inner && g.e.rm_offset == MIA_RM_DROP && g.e.rm_istride == 1 &&
                    (g.e.act == MIA_ACT_NONE || g.e.act == MIA_ACT_RELU);
  const bool plain16 = g.split == 1 && g.e.dtype == MIA_BF16 &&
                       (g.e.act == MIA_ACT_NONE || g.e.act == MIA_ACT_RELU || g.e.act == MIA_ACT_GELU ||
                        (save && g.e.aux_dtype == MIA_BF16 && (g.e.ldaux & 7) == 0 &&
                         ((reinterpret_cast<uintptr_t>(g.e.aux)) & 15) == 0)) &&
                       !g.e.accumulate && (!g.e.rm_inner || drop) &&
                       g.e.alpha == 1.f && m0 + 128 <= g.M && n0 + 128 <= g.N && (g.e.ldc & 7) == 0 &&
                       ((reinterpret_cast<uintptr_t>(g.e.ptr)) & 15) == 0;
  if (plain16) {
    float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int col = wn * 64 + j * 32 + (lane & 31);
          tile[row * 128 + (col ^ (((row >> 2) & 1) << 5))] = acc[i][j][r];
        }
    __syncthreads();
    const int col = (lane & 15) * 8;
    float bv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) bv[c] = g.e.bias ? g.e.bias[n0 + col + c] : 0.f;
    const bool relu = g.e.act == MIA_ACT_RELU, gelu = g.e.act == MIA_ACT_GELU || save;
    bf16* out = reinterpret_cast<bf16*>(g.e.ptr);
    auto pack = [](const float* f) {
      uint32_t w4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w4[q] = pk_bf16(f[2 * q], f[2 * q + 1]);
      }
      return make_uint4(w4[0], w4[1], w4[2], w4[3]);
    };
#pragma unroll 4
    for (int it = 0; it < 8; ++it) {
      const int row = wave * 32 + it * 4 + (lane >> 4);
      const int sw = ((row >> 2) & 1) << 5;
      const f32x4 a = *reinterpret_cast<const f32x4*>(tile + row * 128 + (col ^ sw));
      const f32x4 b = *reinterpret_cast<const f32x4*>(tile + row * 128 + ((col + 4) ^ sw));
      float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] += bv[c];
      if (save) {  // GELU_SAVE(_D): the pre-activation or gelu' goes to aux (MLP fc1, read by the backward)
        float d[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) d[c] = save_d ? gelu_erf_grad((float)(bf16)v[c]) : v[c];  // gelu' of bf16 u
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(const_cast<char*>(g.e.aux)) + (m0 + row) * g.e.ldaux +
                                  n0 + col) = pack(d);
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = relu ? fmaxf(v[c], 0.f) : (gelu ? gelu_erf(v[c]) : v[c]);
      int64_t prow = m0 + row;
      if (drop) {
        const int64_t x = prow % g.e.rm_inner;
        if (x >= g.e.rm_outer) continue;
        prow = (prow / g.e.rm_inner) * g.e.rm_outer + x;
      }
      *reinterpret_cast<uint4*>(out + prow * g.e.ldc + n0 + col) = pack(v);
    }
    return;
  }

  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * 33);
  double sqg = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        stage[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = acc[i][j][r];
      __syncthreads();
      const int row = lane >> 1, c0 = (lane & 1) * 16;
      const int64_t m = m0 + wm * 64 + i * 32 + row;
      const int64_t nb = n0 + wn * 64 + j * 32 + c0;
      if (m < g.M && nb < g.N) {
        float v[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] = stage[row * 33 + c0 + c];
        if (g.split > 1) {
          float* dst = g.ws + ((int64_t)z * g.M + m) * g.N + nb;
          if (nb + 16 <= g.N && (g.N & 3) == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              reinterpret_cast<float4*>(dst)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
          } else {
            for (int c = 0; c < 16; ++c)
              if (nb + c < g.N) dst[c] = v[c];
          }
        } else {
          epi_store16(g.e, m, nb, g.N, v);
          if (g.e.sqsum) {
            float sq = 0.f;
            for (int c = 0; c < 16; ++c)
              if (nb + c < g.N) sq = fmaf(v[c], v[c], sq);
            sqg += sq;
          }
        }
      }
      __syncthreads();
    }
  if (g.e.sqsum && g.split == 1)
    tile_sqsum_store(g.e.sqsum + (int64_t)bm * g.nbn + bn, sqg, reinterpret_cast<double*>(smem));
}

bool dgemm_ok(const MiaOperand& A, const MiaOperand& B, int64_t M, int64_t N, int64_t K, int compute) {
  if (compute != MIA_BF16 || K < 64 || K % 64 != 0 || M < 64 || N < 64) return false;
  if (A.kind != MIA_OP_DENSE || B.kind != MIA_OP_DENSE) return false;
  if (A.dtype != MIA_BF16 || B.dtype != MIA_BF16 || A.pre != MIA_PRE_NONE || B.pre != MIA_PRE_NONE) return false;
  if (A.ld % 8 || B.ld % 8 || (reinterpret_cast<uintptr_t>(A.ptr) & 15) || (reinterpret_cast<uintptr_t>(B.ptr) & 15))
    return false;
  if (A.layout == MIA_LAYOUT_KC) { if (A.rows != M || A.cols < K) return false; }
  else { if (A.rows < K || A.cols != M || M % 8) return false; }
  if (B.layout == MIA_LAYOUT_KC) { if (B.rows != N || B.cols < K) return false; }
  else { if (B.rows < K || B.cols != N || N % 8) return false; }
  if (cdiv(M, 128) * cdiv(N, 128) >= (1ll << 31)) return false;
  return true;
}

template <int LA, int LB, bool ADAM = false>
hipError_t dgemm_launch2(const DArgs& d, hipStream_t s) {
  dim3 grid((unsigned)(d.nbm * d.nbn), (unsigned)d.split);
  dgemm_kernel<LA, LB, ADAM><<<grid, NT, 0, s>>>(d);
  return hipGetLastError();
}

// Row-window conv applies when: bf16 compute, no split, A = CONV/KC with stride (1, 1|2),
// C in {32, 64}, KW*C a multiple of 128, B = the packed [N][KH*KW*C] bf16 weights, N in {32, 64}.
bool rowconv_ok(const MiaOperand& A, const MiaOperand& B, int64_t M, int64_t N, int64_t K, int compute, int split) {
  if (compute != MIA_BF16 || split > 1) return false;
  if (A.kind != MIA_OP_CONV || A.layout != MIA_LAYOUT_KC || A.sh != 1 || (A.sw != 1 && A.sw != 2)) return false;
  if (A.c != 32 && A.c != 64) return false;
  if ((A.kw * A.c) % 128 != 0 || A.kw > (A.sw == 1 ? 8 : 16)) return false;
  if (A.pre != MIA_PRE_NONE && A.pre != MIA_PRE_AFFINE && A.pre != MIA_PRE_AFFINE_RELU) return false;
  if (A.dtype != MIA_BF16 && A.dtype != MIA_F32) return false;
  if (B.kind != MIA_OP_DENSE || B.layout != MIA_LAYOUT_KC || B.dtype != MIA_BF16) return false;
  if (B.rows != N || B.cols != K || B.ld % 8 != 0 || (reinterpret_cast<uintptr_t>(B.ptr) & 15)) return false;
  if (N != 32 && N != 64) return false;
  if (K != (int64_t)A.kh * A.kw * A.c || M != (int64_t)A.n * A.oh * A.ow) return false;
  if (A.c == 64 && A.sw != 1) return false;
  if ((reinterpret_cast<uintptr_t>(A.ptr) & 15)) return false;
  return true;
}

template <typename TS, int BM, int NB, int S, int C, int KWMAX>
hipError_t rowconv_launch2(const RowArgs& r, bool pre, hipStream_t s) {
  dim3 grid((unsigned)cdiv(r.ow, BM), (unsigned)r.oh, (unsigned)r.n);
  if (pre) rowconv_kernel<TS, BM, NB, S, C, KWMAX, true><<<grid, NT, 0, s>>>(r);
  else rowconv_kernel<TS, BM, NB, S, C, KWMAX, false><<<grid, NT, 0, s>>>(r);
  return hipGetLastError();
}

template <typename TS>
hipError_t rowconv_launch1(const RowArgs& r, int S, int C, bool pre, hipStream_t s) {
  if (S == 2) {
    if (r.N == 64) return rowconv_launch2<TS, 256, 64, 2, 32, 16>(r, pre, s);  // conv2: 64 KB of weights per 256 px
    return rowconv_launch2<TS, 128, 32, 2, 32, 16>(r, pre, s);
  }
  if (C == 64) {
    if (r.N == 64) return rowconv_launch2<TS, 128, 64, 1, 64, 8>(r, pre, s);
    return rowconv_launch2<TS, 256, 32, 1, 64, 8>(r, pre, s);
  }
  if (r.N == 64) return rowconv_launch2<TS, 128, 64, 1, 32, 8>(r, pre, s);
  return rowconv_launch2<TS, 256, 32, 1, 32, 8>(r, pre, s);
}

// Many-slab reduction (split >= 32): 16 outputs x 16 slab lanes per block, fixed per-lane slab
// order and a fixed LDS tree -> deterministic; the plain kernel walks all slabs per thread.
__global__ __launch_bounds__(256) void splitk_reduce_wide_kernel(const float* ws, int split, int64_t M, int64_t N,
                                                                 EpiDev e) {
  __shared__ float red[16][17];
  const int64_t total = M * N;
  const int o = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const int64_t idx = (int64_t)blockIdx.x * 16 + o;
  float s = 0.f;
  if (idx < total)
    for (int z = zl; z < split; z += 16) s += ws[(int64_t)z * total + idx];
  red[zl][o] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float a = 0.f;
    for (int k = 0; k < 16; ++k) a += red[k][threadIdx.x];
    const int64_t id = (int64_t)blockIdx.x * 16 + threadIdx.x;
    if (id < total) epi_store(e, id / N, id % N, a);
  }
}

void launch_splitk_reduce(const float* ws, int split, int64_t M, int64_t N, const EpiDev& e, hipStream_t s) {
  const int64_t total = M * N;
  if (split >= 32 && total <= (1ll << 22)) {
    splitk_reduce_wide_kernel<<<(unsigned)cdiv(total, 16), 256, 0, s>>>(ws, split, M, N, e);
  } else {
    int blocks = (int)std::min<int64_t>(cdiv(total, 256), 8192);
    splitk_reduce_kernel<<<blocks, 256, 0, s>>>(ws, split, M, N, e);
  }
}

OpDev to_dev(const MiaOperand& o) {
  OpDev d;
  memset(&d, 0, sizeof(d));
  d.ptr = reinterpret_cast<const char*>(o.ptr);
  d.kind = o.kind; d.dtype = o.dtype; d.pre = o.pre;
  d.rows = o.rows; d.cols = o.cols; d.ld = o.ld;
  d.n = o.n; d.h = o.h; d.w = o.w; d.c = o.c; d.oh = o.oh; d.ow = o.ow;
  d.kh = o.kh; d.kw = o.kw; d.sh = o.sh; d.sw = o.sw; d.ph = o.ph; d.pw = o.pw;
  d.npix = o.n * o.oh * o.ow;
  d.ohw = o.oh * o.ow;
  d.kwc = o.kw * o.c;
  d.jtot = o.kh * o.kw * o.c;
  d.ps = o.pre_scale; d.pt = o.pre_shift;
  return d;
}

EpiDev to_dev(const MiaEpilogue& e) {
  EpiDev d;
  d.ptr = reinterpret_cast<char*>(e.ptr);
  d.dtype = e.dtype; d.act = e.act; d.accumulate = e.accumulate; d.aux_dtype = e.aux_dtype;
  d.ldc = e.ldc; d.rm_inner = e.rm_inner; d.rm_outer = e.rm_outer; d.rm_istride = e.rm_istride;
  d.rm_offset = e.rm_offset; d.bias = e.bias; d.aux = reinterpret_cast<const char*>(e.aux);
  d.ldaux = e.ldaux; d.alpha = e.alpha; d.act_scale = e.act_scale;
  d.sqsum = e.sqsum;
  return d;
}

int check_operand(const MiaOperand& o, const char* name) {
  MIA_CHECK_ARG(o.ptr != nullptr, "gemm: operand %s is null", name);
  MIA_CHECK_ARG(o.dtype == MIA_F32 || o.dtype == MIA_BF16, "gemm: operand %s dtype %d", name, o.dtype);
  MIA_CHECK_ARG(o.layout == MIA_LAYOUT_KC || o.layout == MIA_LAYOUT_RC, "gemm: operand %s layout", name);
  if (o.pre == MIA_PRE_AFFINE || o.pre == MIA_PRE_AFFINE_RELU)
    MIA_CHECK_ARG(o.pre_scale && o.pre_shift && o.kind != MIA_OP_CONVROW,
                  "gemm: operand %s affine pre-op needs scale/shift and a DENSE/CONV source", name);
  if (o.kind == MIA_OP_DENSE) {
    // ld < cols is allowed: overlapping rows are a valid read-only view (the (1, 2)-conv im2col of
    // a channels-last map is the map itself with ld = C, cols = 2C)
    MIA_CHECK_ARG(o.rows >= 0 && o.cols >= 0 && o.ld > 0, "gemm: operand %s dense extents", name);
  } else {
    MIA_CHECK_ARG(o.n > 0 && o.h > 0 && o.w > 0 && o.c > 0 && o.oh > 0 && o.ow > 0 && o.kh > 0 &&
                      o.kw > 0 && o.sh > 0 && o.sw > 0,
                  "gemm: operand %s conv geometry", name);
    MIA_CHECK_ARG((int64_t)o.n * o.oh * o.ow < (1ll << 31), "gemm: operand %s too many pixels", name);
    if (o.kind == MIA_OP_CONV) {
      MIA_CHECK_ARG(o.c % 8 == 0, "gemm: operand %s CONV needs c %% 8 == 0 (c=%d)", name, o.c);
    } else {
      MIA_CHECK_ARG((o.kw * o.c) % 8 == 0 && o.pw == 0, "gemm: operand %s CONVROW needs kw*c %% 8 == 0, pw == 0", name);
      MIA_CHECK_ARG((int64_t)(o.ow - 1) * o.sw + o.kw <= o.w, "gemm: operand %s CONVROW row overruns input", name);
    }
  }
  return 0;
}

template <typename T, int BM, int BN, int WM>
hipError_t launch_cfg(const GemmArgs& g, int LA, int LB, hipStream_t s) {
  dim3 grid((unsigned)cdiv(g.M, BM), (unsigned)cdiv(g.N, BN), (unsigned)g.split);
  if (LA == MIA_LAYOUT_KC && LB == MIA_LAYOUT_KC)
    igemm_kernel<T, BM, BN, WM, MIA_LAYOUT_KC, MIA_LAYOUT_KC><<<grid, NT, 0, s>>>(g);
  else if (LA == MIA_LAYOUT_KC && LB == MIA_LAYOUT_RC)
    igemm_kernel<T, BM, BN, WM, MIA_LAYOUT_KC, MIA_LAYOUT_RC><<<grid, NT, 0, s>>>(g);
  else if (LA == MIA_LAYOUT_RC && LB == MIA_LAYOUT_KC)
    igemm_kernel<T, BM, BN, WM, MIA_LAYOUT_RC, MIA_LAYOUT_KC><<<grid, NT, 0, s>>>(g);
  else
    igemm_kernel<T, BM, BN, WM, MIA_LAYOUT_RC, MIA_LAYOUT_RC><<<grid, NT, 0, s>>>(g);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_t(const GemmArgs& g, int LA, int LB, hipStream_t s) {
  if (g.N <= 32) return launch_cfg<T, 256, 32, 4>(g, LA, LB, s);
  if (g.N <= 64) return launch_cfg<T, 128, 64, 2>(g, LA, LB, s);
  if (g.M <= 32) return launch_cfg<T, 32, 128, 1>(g, LA, LB, s);
  if (g.M <= 64) return launch_cfg<T, 64, 128, 1>(g, LA, LB, s);
  return launch_cfg<T, 128, 128, 2>(g, LA, LB, s);
}

}  // namespace

extern "C" int64_t mia_gemm_workspace_bytes(int64_t M, int64_t N, int32_t split_k) {
  return split_k > 1 ? (int64_t)split_k * M * N * 4 : 0;
}

static int gemm_tile(const MiaOperand* A, const MiaOperand* B, const MiaEpilogue* E, int64_t M, int64_t N,
                     int64_t K, int32_t compute_dtype, int32_t split_k, void* workspace, mia_stream_t stream) {
  MIA_CHECK_ARG(A && B && E, "gemm: null descriptor");
  MIA_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "gemm: negative extent");
  MIA_CHECK_ARG(M < (1ll << 31) * 128 && N < 65535ll * 128, "gemm: extent too large");
  if (int r = check_operand(*A, "A")) return r;
  if (int r = check_operand(*B, "B")) return r;
  MIA_CHECK_ARG(E->ptr != nullptr, "gemm: output is null");
  MIA_CHECK_ARG(compute_dtype == MIA_F32 || compute_dtype == MIA_BF16, "gemm: compute dtype");
  if (E->act == MIA_DACT_NZ || E->act == MIA_DACT_GELU || E->act == MIA_ACT_ADD_AUX || E->act == MIA_ACT_GELU_SAVE ||
      E->act == MIA_ACT_GELU_SAVE_D || E->act == MIA_DACT_MUL)
    MIA_CHECK_ARG(E->aux != nullptr, "gemm: this epilogue needs aux");
  if (split_k < 1) split_k = 1;
  if (split_k > 1) MIA_CHECK_ARG(workspace != nullptr, "gemm: split_k needs workspace");
  if (M == 0 || N == 0) return 0;
  if (dgemm_ok(*A, *B, M, N, K, compute_dtype) && (split_k <= 1 || workspace)) {
    DArgs d;
    d.a = reinterpret_cast<const bf16*>(A->ptr); d.b = reinterpret_cast<const bf16*>(B->ptr);
    d.lda = A->ld; d.ldb = B->ld; d.M = M; d.N = N; d.K = K;
    d.split = split_k < 1 ? 1 : split_k;
    d.kper = cdiv(cdiv(K, d.split), 64) * 64;
    d.nbm = (int)cdiv(M, 128); d.nbn = (int)cdiv(N, 128);
    // tall GEMMs (AST linears: M = tokens, N <= 3072): grouped tile order (DArgs::gm) so each A row
    // block is read from HBM once (at batch 256 the activations exceed the 256 MB Infinity Cache; an
    // M-fastest walk re-streamed them once per column tile: 12-15 GB per launch, rocprof FETCH_SIZE)
    // and each B column tile once per group of gm row blocks
    d.nfast = (d.split == 1 && d.nbn <= 32 && d.nbm >= 4 * d.nbn) ? 1 : 0;
    d.gm = (int)std::max<int64_t>(1, std::min<int64_t>(16, (2ll << 20) / (128 * 2 * std::max<int64_t>(K, 64))));
    d.ws = reinterpret_cast<float*>(workspace);
    d.e = to_dev(*E);
    d.mode = 0;
    hipStream_t s = as_stream(stream);
    hipError_t err;
    const int la = A->layout, lb = B->layout;
    if (la == MIA_LAYOUT_KC && lb == MIA_LAYOUT_KC) err = dgemm_launch2<MIA_LAYOUT_KC, MIA_LAYOUT_KC>(d, s);
    else if (la == MIA_LAYOUT_KC) err = dgemm_launch2<MIA_LAYOUT_KC, MIA_LAYOUT_RC>(d, s);
    else if (lb == MIA_LAYOUT_KC) err = dgemm_launch2<MIA_LAYOUT_RC, MIA_LAYOUT_KC>(d, s);
    else err = dgemm_launch2<MIA_LAYOUT_RC, MIA_LAYOUT_RC>(d, s);
    if (err != hipSuccess) return mia::fail(-(int)err, "dgemm launch: %s", hipGetErrorString(err));
    if (d.split > 1) launch_splitk_reduce(d.ws, d.split, M, N, d.e, s);
    return 0;
  }
  if (tapconv_ok(*A, *B, M, N, K, compute_dtype, split_k)) {
    TapArgs r;
    r.x = reinterpret_cast<const char*>(A->ptr);
    r.n = A->n; r.h = A->h; r.wx = A->w * A->c; r.oh = A->oh; r.ow = A->ow;
    r.wt = reinterpret_cast<const bf16*>(B->ptr);
    r.e = to_dev(*E);
    const int64_t blocks = (int64_t)A->n * A->oh * cdiv(A->ow, 256);
    MIA_CHECK_ARG(blocks < (1ll << 31), "tapconv: too many chunks");
    hipStream_t s = as_stream(stream);
    if (A->c == 2) tapconv_kernel<float, 2, 1, 64><<<(unsigned)blocks, NT, 0, s>>>(r);
    else if (A->dtype == MIA_BF16) tapconv_kernel<bf16, 1, 8, 8><<<(unsigned)blocks, NT, 0, s>>>(r);
    else tapconv_kernel<float, 1, 8, 8><<<(unsigned)blocks, NT, 0, s>>>(r);
    MIA_LAUNCH_CHECK("tapconv");
    return 0;
  }
  if (rowconv_ok(*A, *B, M, N, K, compute_dtype, split_k)) {
    RowArgs r;
    r.x = reinterpret_cast<const char*>(A->ptr);
    r.xdt = A->dtype; r.pre = A->pre;
    r.n = A->n; r.h = A->h; r.w = A->w; r.oh = A->oh; r.ow = A->ow; r.kh = A->kh; r.kw = A->kw;
    r.ph = A->ph; r.pw = A->pw; r.ps = A->pre_scale; r.pt = A->pre_shift;
    r.wt = reinterpret_cast<const bf16*>(B->ptr); r.ldw = B->ld; r.N = N; r.M = M;
    r.e = to_dev(*E);
    const bool pre = A->pre != MIA_PRE_NONE;
    hipStream_t s = as_stream(stream);
    hipError_t err = A->dtype == MIA_BF16 ? rowconv_launch1<bf16>(r, A->sw, A->c, pre, s)
                                          : rowconv_launch1<float>(r, A->sw, A->c, pre, s);
    if (err != hipSuccess) return mia::fail(-(int)err, "rowconv launch: %s", hipGetErrorString(err));
    return 0;
  }
  if (workspace && tapwgrad_ok(*A, *B, M, N, K, compute_dtype, split_k)) {
    TapWArgs r{};
    r.x = reinterpret_cast<const char*>(B->ptr);
    r.dy = reinterpret_cast<const char*>(A->ptr);
    r.n = B->n; r.h = B->h; r.wx = B->w * B->c; r.oh = B->oh; r.ow = B->ow;
    r.Z = split_k; r.ws = reinterpret_cast<float*>(workspace);
    hipStream_t s = as_stream(stream);
    hipError_t err;
    if (B->c == 2) {  // frontend conv1: stride 2 over the waveform
      err = A->dtype == MIA_BF16 ? tapwgrad_launch<bf16, float, 2, 1, 64>(r, s)
                                 : tapwgrad_launch<float, float, 2, 1, 64>(r, s);
    } else if (B->dtype == MIA_BF16) {
      err = A->dtype == MIA_BF16 ? tapwgrad_launch<bf16, bf16, 1, 8, 8>(r, s)
                                 : tapwgrad_launch<float, bf16, 1, 8, 8>(r, s);
    } else {
      err = A->dtype == MIA_BF16 ? tapwgrad_launch<bf16, float, 1, 8, 8>(r, s)
                                 : tapwgrad_launch<float, float, 1, 8, 8>(r, s);
    }
    if (err != hipSuccess) return mia::fail(-(int)err, "tapwgrad launch: %s", hipGetErrorString(err));
    launch_splitk_reduce(r.ws, split_k, M, N, to_dev(*E), s);
    MIA_LAUNCH_CHECK("splitk_reduce");
    return 0;
  }
  if (workspace && rowwgrad_ok(*A, *B, M, N, K, compute_dtype, split_k) && A->dtype == MIA_BF16 && M == 32 &&
      B->c == 32 && B->kh == 8 && B->kw == 8 && B->sw == 1 && B->ph == 0 && B->pw == 0 &&
      B->pre == MIA_PRE_AFFINE_RELU && B->h == B->oh + 7 && B->w == B->ow + 7) {
    // trunk conv4 wgrad: rolling 8-row window per (clip, column chunk), one slab per block
    W8Args w8;
    w8.x = reinterpret_cast<const bf16*>(B->ptr);
    w8.dy = reinterpret_cast<const bf16*>(A->ptr);
    w8.ps = B->pre_scale; w8.pt = B->pre_shift;
    w8.n = B->n; w8.h = B->h; w8.w = B->w; w8.oh = B->oh; w8.ow = B->ow;
    const int64_t items = (int64_t)B->n * cdiv(B->ow, 128);
    w8.nblk = (int)std::min<int64_t>(std::min<int64_t>(split_k, 256), items);
    w8.ws = reinterpret_cast<float*>(workspace);
    hipStream_t s = as_stream(stream);
    hipError_t err = wgrad8_launch(w8, s);
    if (err != hipSuccess) return mia::fail(-(int)err, "wgrad8 launch: %s", hipGetErrorString(err));
    launch_splitk_reduce(w8.ws, w8.nblk, M, N, to_dev(*E), s);
    MIA_LAUNCH_CHECK("splitk_reduce");
    return 0;
  }
  if (workspace && rowwgrad_ok(*A, *B, M, N, K, compute_dtype, split_k)) {
    RowWArgs r;
    r.x = reinterpret_cast<const char*>(B->ptr);
    r.dy = reinterpret_cast<const char*>(A->ptr);
    r.pre = B->pre;
    r.n = B->n; r.h = B->h; r.w = B->w; r.oh = B->oh; r.ow = B->ow; r.kh = B->kh; r.kw = B->kw;
    r.ph = B->ph; r.pw = B->pw; r.ps = B->pre_scale; r.pt = B->pre_shift;
    r.Z = split_k; r.Ntot = N; r.ws = reinterpret_cast<float*>(workspace);
    const bool pre = B->pre != MIA_PRE_NONE;
    hipStream_t s = as_stream(stream);
    hipError_t err = A->dtype == MIA_BF16 ? rowwgrad_launch1<bf16>(r, (int)M, B->sw, B->c, pre, s)
                                          : rowwgrad_launch1<float>(r, (int)M, B->sw, B->c, pre, s);
    if (err != hipSuccess) return mia::fail(-(int)err, "rowwgrad launch: %s", hipGetErrorString(err));
    launch_splitk_reduce(r.ws, split_k, M, N, to_dev(*E), s);
    MIA_LAUNCH_CHECK("splitk_reduce");
    return 0;
  }
  GemmArgs g;
  g.a = to_dev(*A);
  g.b = to_dev(*B);
  g.e = to_dev(*E);
  g.M = M; g.N = N; g.K = K;
  g.split = split_k;
  g.kper = cdiv(cdiv(K, split_k), BK) * BK;
  g.ws = reinterpret_cast<float*>(workspace);
  hipStream_t s = as_stream(stream);
  hipError_t err = compute_dtype == MIA_BF16 ? launch_t<bf16>(g, A->layout, B->layout, s)
                                             : launch_t<float>(g, A->layout, B->layout, s);
  if (err != hipSuccess) return mia::fail(-(int)err, "gemm launch: %s", hipGetErrorString(err));
  if (split_k > 1) {
    launch_splitk_reduce(g.ws, split_k, M, N, g.e, s);
    MIA_LAUNCH_CHECK("splitk_reduce");
  }
  return 0;
}

extern "C" int64_t mia_gemm_sqsum_slots(int64_t M, int64_t N) { return cdiv(M, 128) * cdiv(N, 128); }

// The dense 128 x 128 kernel in its norm-only / fused-Adam modes (DArgs::mode): full tiles, no split.
static int dgemm_mode(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K, int mode,
                      double* sqsum, const DArgs::AdamEpi* adam, mia_stream_t stream) {
  MIA_CHECK_ARG(A && B, "gemm_wgrad: null descriptor");
  MIA_CHECK_ARG(dgemm_ok(*A, *B, M, N, K, MIA_BF16) && M % 128 == 0 && N % 128 == 0,
                "gemm_wgrad: needs bf16 dense operands, M and N multiples of 128, K a multiple of 64");
  DArgs d;
  memset(&d, 0, sizeof(d));
  d.a = reinterpret_cast<const bf16*>(A->ptr); d.b = reinterpret_cast<const bf16*>(B->ptr);
  d.lda = A->ld; d.ldb = B->ld; d.M = M; d.N = N; d.K = K;
  d.split = 1; d.kper = K;
  d.nbm = (int)(M / 128); d.nbn = (int)(N / 128);
  // sums only: row-block-major tile order (an XCD's concurrent tiles share their dY rows; 0.271 -> 0.259 ms
  // for FC1); the Adam form keeps column-block-major (row-major measured 2.14 -> 2.18 ms)
  d.nfast = mode == 1; d.gm = 1;
  d.e.dtype = MIA_F32; d.e.alpha = 1.f; d.e.sqsum = sqsum;
  d.mode = mode;
  if (adam) d.adam = *adam;
  hipStream_t s = as_stream(stream);
  hipError_t err;
  const int la = A->layout, lb = B->layout;
  if (mode == 2) {  // the weight-gradient layouts only (dY and X both K-major: RC x RC)
    MIA_CHECK_ARG(la == MIA_LAYOUT_RC && lb == MIA_LAYOUT_RC, "gemm_adam: needs RC operands");
    err = dgemm_launch2<MIA_LAYOUT_RC, MIA_LAYOUT_RC, true>(d, s);
  } else if (la == MIA_LAYOUT_KC && lb == MIA_LAYOUT_KC) err = dgemm_launch2<MIA_LAYOUT_KC, MIA_LAYOUT_KC>(d, s);
  else if (la == MIA_LAYOUT_KC) err = dgemm_launch2<MIA_LAYOUT_KC, MIA_LAYOUT_RC>(d, s);
  else if (lb == MIA_LAYOUT_KC) err = dgemm_launch2<MIA_LAYOUT_RC, MIA_LAYOUT_KC>(d, s);
  else err = dgemm_launch2<MIA_LAYOUT_RC, MIA_LAYOUT_RC>(d, s);
  if (err != hipSuccess) return mia::fail(-(int)err, "gemm_wgrad launch: %s", hipGetErrorString(err));
  return 0;
}

extern "C" int mia_gemm_sqsum_only(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K,
                                   double* sqsum, mia_stream_t stream) {
  MIA_CHECK_ARG(sqsum, "gemm_sqsum_only: null sqsum");
  return dgemm_mode(A, B, M, N, K, 1, sqsum, nullptr, stream);
}

extern "C" int mia_gemm_adam(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K, float* param,
                             float* exp_avg, float* exp_avg_sq, void* shadow_bf16, int64_t ld, const float* coef,
                             float lr_over_bc1, float bc2_sqrt, float beta1, float beta2, float eps, float weight_decay,
                             mia_stream_t stream) {
  MIA_CHECK_ARG(param && exp_avg && exp_avg_sq && coef, "gemm_adam: null pointer");
  MIA_CHECK_ARG(ld >= N && ld % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(exp_avg) |
                      reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(shadow_bf16) & 7) == 0,
                "gemm_adam: p / m / v must be 16-B aligned rows (ld %% 4 == 0), the shadow 8-B aligned");
  DArgs::AdamEpi a{param, exp_avg, exp_avg_sq, reinterpret_cast<bf16*>(shadow_bf16), coef, lr_over_bc1, bc2_sqrt,
                   beta1, beta2, eps, weight_decay, ld};
  return dgemm_mode(A, B, M, N, K, 2, nullptr, &a, stream);
}

// workspace layout of one mia_gemm call on paths 0-5: [split-K slabs][column-sum partials]
static int64_t colsum_ws_offset(int64_t M, int64_t N, int32_t split_k) {
  return cdiv(mia_gemm_workspace_bytes(M, N, split_k), 256) * 256;
}

extern "C" int64_t mia_gemm_workspace_bytes_ex(const MiaOperand* A, const MiaOperand* B, const MiaEpilogue* E,
                                               int64_t M, int64_t N, int64_t K, int32_t compute_dtype,
                                               int32_t split_k) {
  if (!A || !B || !E) return 0;
  if (mgemm::mg_ok(*A, *B, *E, M, N, K, compute_dtype))
    return mgemm::mg_workspace_bytes(M, N, K, E->colsum != nullptr, E->a_colsum != nullptr);
  if (E->a_colsum) {  // the GEMM's own workspace, then the column-sum pass over A
    MiaEpilogue e = *E;
    e.a_colsum = nullptr;
    return cdiv(mia_gemm_workspace_bytes_ex(A, B, &e, M, N, K, compute_dtype, split_k), 256) * 256 +
           (int64_t)MIA_COLSUM_MAXBLK * M * 4;
  }
  int64_t b = mia_gemm_workspace_bytes(M, N, split_k);
  if (E->colsum) b = colsum_ws_offset(M, N, split_k) + (int64_t)MIA_COLSUM_MAXBLK * N * 4;
  return b;
}

extern "C" int mia_gemm(const MiaOperand* A, const MiaOperand* B, const MiaEpilogue* E, int64_t M,
                        int64_t N, int64_t K, int32_t compute_dtype, int32_t split_k, void* workspace,
                        mia_stream_t stream) {
  MIA_CHECK_ARG(A && B && E, "gemm: null descriptor");
  if (E->ptr && M > 0 && N > 0 && K > 0 && mgemm::mg_ok(*A, *B, *E, M, N, K, compute_dtype))
    return mgemm::mg_run(*A, *B, *E, M, N, K, workspace, as_stream(stream));
  MIA_CHECK_ARG(!E->mx_q, "gemm: an MX-fp8 output copy needs the 256x256 kernel (bf16 dense operands, "
                "plain / GELU / GELU_SAVE bf16 output, ldc == N, N %% 32 == 0)");
  if (E->a_colsum) {  // other paths: the GEMM, then a column-sum pass over the k-by-m A
    MIA_CHECK_ARG(A->kind == MIA_OP_DENSE && A->layout == MIA_LAYOUT_RC && A->pre == MIA_PRE_NONE &&
                      (A->dtype == MIA_BF16 || A->dtype == MIA_F32) && A->rows >= K && A->cols == M,
                  "gemm: a_colsum needs a dense k-by-m (RC) A without pre-op");
    MIA_CHECK_ARG(workspace || M == 0 || K == 0, "gemm a_colsum: needs the workspace of mia_gemm_workspace_bytes_ex");
    MiaEpilogue e = *E;
    e.a_colsum = nullptr;
    if (int r = mia_gemm(A, B, &e, M, N, K, compute_dtype, split_k, workspace, stream)) return r;
    if (M == 0) return 0;
    void* ws = static_cast<char*>(workspace) +
               cdiv(mia_gemm_workspace_bytes_ex(A, B, &e, M, N, K, compute_dtype, split_k), 256) * 256;
    return mia_colsum(A->ptr, A->dtype, K, (int32_t)M, A->ld, E->a_colsum, ws, stream);
  }
  if (E->colsum) {
    MIA_CHECK_ARG(!E->sqsum && !E->accumulate && !E->rm_inner && E->ldc >= N &&
                      (E->dtype == MIA_BF16 || E->dtype == MIA_F32),
                  "gemm: colsum needs a plain row-major output");
    MIA_CHECK_ARG(workspace || M == 0 || N == 0, "gemm colsum: needs the workspace of mia_gemm_workspace_bytes_ex");
    if (int r = gemm_tile(A, B, E, M, N, K, compute_dtype, split_k, workspace, stream)) return r;
    if (M > 0 && N > 0) {
      void* ws = static_cast<char*>(workspace) + colsum_ws_offset(M, N, split_k);
      if (int r = mia_colsum(E->ptr, E->dtype, M, (int32_t)N, E->ldc, E->colsum, ws, stream)) return r;
    }
    return 0;
  }
  if (!E->sqsum) return gemm_tile(A, B, E, M, N, K, compute_dtype, split_k, workspace, stream);
  MIA_CHECK_ARG(E->dtype == MIA_F32 && E->act == MIA_ACT_NONE && !E->bias && !E->accumulate && !E->rm_inner &&
                    E->alpha == 1.f,
                "gemm: sqsum needs a plain f32 output");
  if (int r = gemm_tile(A, B, E, M, N, K, compute_dtype, split_k, workspace, stream)) return r;
  // the dense kernel writes the slots itself when it runs unsplit; every other path gets the pass
  const bool fused = dgemm_ok(*A, *B, M, N, K, compute_dtype) && split_k <= 1;
  if (!fused && M > 0 && N > 0) {
    const int64_t nb = mia_gemm_sqsum_slots(M, N);
    MIA_CHECK_ARG(nb < (1ll << 31), "gemm sqsum: too many tiles");
    tile_sqsum_kernel<<<(unsigned)nb, NT, 0, as_stream(stream)>>>(reinterpret_cast<const float*>(E->ptr), E->ldc, M,
                                                                   N, (int)cdiv(N, 128), E->sqsum);
    MIA_LAUNCH_CHECK("gemm sqsum");
  }
  return 0;
}

extern "C" int mia_gemm_path(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K,
                             int32_t compute_dtype, int32_t split_k) {
  if (!A || !B) return -1;
  MiaEpilogue e{};
  e.ptr = reinterpret_cast<void*>(256); e.dtype = MIA_BF16; e.ldc = N; e.alpha = 1.f;
  if (mgemm::mg_ok(*A, *B, e, M, N, K, compute_dtype)) return 7;
  if (dgemm_ok(*A, *B, M, N, K, compute_dtype)) return 5;
  if (tapconv_ok(*A, *B, M, N, K, compute_dtype, split_k)) return 4;
  if (rowconv_ok(*A, *B, M, N, K, compute_dtype, split_k)) return 1;
  if (rowwgrad_ok(*A, *B, M, N, K, compute_dtype, split_k)) return 2;
  if (tapwgrad_ok(*A, *B, M, N, K, compute_dtype, split_k)) return 3;
  return 0;
}

// G2[k] = sum_{b, p < w1} x[b][2p + k] (k < 64).  With r = k & 1, j0 = k >> 1 the window is
// x_r[j0 .. j0+w1) of the parity sequence x_r[j] = x[2j+r], so G2 = sum_b T_r - (head j < j0) -
// (tail j >= j0 + w1): C1_SPLIT blocks per clip sum disjoint ranges of the two parities (coalesced
// 8-byte loads), the first block of each clip also writes the per-k head/tail corrections.
constexpr int C1_SPLIT = 8;
__global__ __launch_bounds__(256) void conv1_colsum_kernel(const float* __restrict__ x, int t, int w1,
                                                           float* __restrict__ part) {
  const int b = blockIdx.x / C1_SPLIT, sp = blockIdx.x % C1_SPLIT, tid = threadIdx.x;
  const float* xb = x + (int64_t)b * t;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const int L = t / 2, per = (L + C1_SPLIT - 1) / C1_SPLIT;
  const int j1 = min(L, (sp + 1) * per);
  float e = 0.f, o = 0.f;
  for (int j = sp * per + tid; j < j1; j += 256) {
    const f32x2 v = *reinterpret_cast<const f32x2*>(xb + 2 * j);
    e += v[0];
    o += v[1];
  }
  __shared__ float red[2][256];
  red[0][tid] = e;
  red[1][tid] = o;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) { red[0][tid] += red[0][tid + h]; red[1][tid] += red[1][tid + h]; }
    __syncthreads();
  }
  // part[b][sp][0..1] = parity totals of this range; part[b][C1_SPLIT][k] = -(head + tail) of k
  float* pb = part + (int64_t)b * (C1_SPLIT * 2 + 64);
  if (tid < 2) pb[sp * 2 + tid] = red[tid][0];
  if (sp == 0 && tid < 64) {
    const int r = tid & 1, j0 = tid >> 1;
    float a = 0.f;
    for (int j = 0; j < j0; ++j) a -= xb[2 * j + r];
    for (int j = j0 + w1; j < L; ++j) a -= xb[2 * j + r];
    pb[C1_SPLIT * 2 + tid] = a;
  }
}

// per-channel sums over the Z block partials (dbp) and per-k G2 over the clips, in double with a
// block-wide tree (one block per output quantity: 96 channel sums + 64 G2 entries)
__global__ __launch_bounds__(256) void conv1_lin_sums_kernel(const float* __restrict__ dbp, int Z,
                                                             const float* __restrict__ g2part, int n,
                                                             double* __restrict__ out) {
  const int q = blockIdx.x, tid = threadIdx.x;
  double a = 0.0;
  if (q < 96) {
    const int ch = q % 32, which = q / 32;
    for (int z = tid; z < Z; z += 256) a += (double)dbp[((int64_t)z * 32 + ch) * 3 + which];
  } else {
    const int k = q - 96, r = k & 1;
    constexpr int PS = C1_SPLIT * 2 + 64;
    for (int b = tid; b < n; b += 256) {
      const float* pb = g2part + (int64_t)b * PS;
      double s = pb[C1_SPLIT * 2 + k];
      for (int sp = 0; sp < C1_SPLIT; ++sp) s += (double)pb[sp * 2 + r];
      a += s;
    }
  }
  __shared__ double red[256];
  red[tid] = a;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) out[q] = red[0];
}

// dgamma/dbeta, A/B/C per channel (double), dW = A G1 + B G2 + C G3, dbias = A sum dz + B P + C sum y
__global__ __launch_bounds__(256) void conv1_lin_final_kernel(const float* __restrict__ g13, const double* __restrict__ sums,
                                                              int64_t P, const float* gamma, const float* mean,
                                                              const float* invstd, float* dgamma, float* dbeta,
                                                              float* dw, float* dbias) {
  __shared__ double cA[32], cB[32], cC[32];
  const int t = threadIdx.x;
  if (t < 32) {
    const double sdz = sums[t], sdx = sums[32 + t], sy = sums[64 + t];
    dbeta[t] = (float)sdz;
    dgamma[t] = (float)sdx;
    const double is = invstd[t], A = (gamma ? (double)gamma[t] : 1.0) * is;
    const double mb = sdz / (double)P, mg = sdx / (double)P;
    const double B = -A * mb + A * is * mg * (double)mean[t], C = -A * is * mg;
    dbias[t] = (float)(A * sdz + B * (double)P + C * sy);
    cA[t] = A; cB[t] = B; cC[t] = C;
  }
  __syncthreads();
  for (int e = t; e < 32 * 64; e += 256) {
    const int ch = e / 64, k = e % 64;
    dw[e] = (float)(cA[ch] * (double)g13[e] + cB[ch] * sums[96 + k] + cC[ch] * (double)g13[2048 + e]);
  }
}

extern "C" int mia_fe_conv1_wgrad_bn(const float* x, const void* dact, const void* y1, int32_t n, int32_t t,
                                     const float* scale, const float* shift, const float* gamma, const float* mean,
                                     const float* invstd, float* dgamma, float* dbeta, float* dw,
                                     float* dbias, void* workspace, int32_t split, mia_stream_t stream) {
  MIA_CHECK_ARG(x && dact && y1 && scale && shift && mean && invstd && dgamma && dbeta && dw && dbias && workspace,
                "fe_conv1_wgrad_bn: null pointer");
  MIA_CHECK_ARG(n > 0 && t >= 64 && t % 2 == 0 && split > 0, "fe_conv1_wgrad_bn: bad sizes");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(dact) | reinterpret_cast<uintptr_t>(y1)) & 15) == 0,
                "fe_conv1_wgrad_bn: dact / y1 must be 16-byte aligned");
  const int w1 = (t - 64) / 2 + 1;
  float* ws = reinterpret_cast<float*>(workspace);
  TapWArgs r{};
  r.x = reinterpret_cast<const char*>(x);
  r.dy = reinterpret_cast<const char*>(dact);
  r.n = n; r.h = 1; r.wx = t; r.oh = 1; r.ow = w1;
  r.Z = split;
  r.ws = ws;                                       // [split][2][32][64]
  r.by = reinterpret_cast<const bf16*>(y1);
  r.bsc = scale; r.bsh = shift; r.bmean = mean; r.binvstd = invstd;
  r.dbp = ws + (int64_t)split * 2 * 2048;          // [split][32][3]
  r.bP = (int64_t)n * w1;
  float* g13 = r.dbp + (int64_t)split * 96;        // [2][32][64]
  float* g2p = g13 + 2 * 2048;                     // [n][C1_SPLIT*2 + 64]
  double* sums = reinterpret_cast<double*>(g2p + (int64_t)n * (C1_SPLIT * 2 + 64) + 1);  // [160], 8-B aligned below
  sums = reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(sums) + 7) & ~uintptr_t(7));
  hipStream_t s = as_stream(stream);
  hipError_t err = tapwgrad_launch<bf16, float, 2, 1, 64, true>(r, s);
  if (err != hipSuccess) return mia::fail(-(int)err, "fe_conv1_wgrad_bn launch: %s", hipGetErrorString(err));
  EpiDev e{};
  e.ptr = reinterpret_cast<char*>(g13); e.dtype = MIA_F32; e.act = MIA_ACT_NONE; e.ldc = 2 * 2048; e.alpha = 1.f;
  e.act_scale = 1.f;
  launch_splitk_reduce(ws, split, 1, 2 * 2048, e, s);  // slabs [split][4096] -> g13
  conv1_colsum_kernel<<<n * C1_SPLIT, 256, 0, s>>>(x, t, w1, g2p);
  conv1_lin_sums_kernel<<<96 + 64, 256, 0, s>>>(r.dbp, split, g2p, n, sums);
  conv1_lin_final_kernel<<<1, 256, 0, s>>>(g13, sums, r.bP, gamma, mean, invstd, dgamma, dbeta, dw, dbias);
  MIA_LAUNCH_CHECK("fe_conv1_wgrad_bn final");
  return 0;
}

extern "C" int mia_splitk_reduce(const float* ws, int32_t split_k, int64_t M, int64_t N,
                                 const MiaEpilogue* E, mia_stream_t stream) {
  MIA_CHECK_ARG(ws && E && E->ptr, "splitk_reduce: null pointer");
  EpiDev e = to_dev(*E);
  const int64_t total = M * N;
  if (total == 0) return 0;
  launch_splitk_reduce(ws, split_k, M, N, e, as_stream(stream));
  MIA_LAUNCH_CHECK("splitk_reduce");
  return 0;
}
