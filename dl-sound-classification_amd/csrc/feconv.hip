// EnvNet-v2 frontend conv2 (reference src/models/envnet_v2.py:19 Conv2d(32, 64, (1, 16), stride
// (1, 2)), input relu(bn1(conv1 output))) forward, and its backward-data, as persistent
// weight-stationary 1-D convolutions, bf16 MFMA, gfx950.
//
//   forward:  y2[b][o][co]      = bias[co] + sum_{kx,ci} W[co][kx][ci] * relu(bn1(y1))[b][2o+kx][ci]
//   dgrad:    da1[b][2m+r][ci]  = sum_{j,co} Wpar[r][ci][j][co] * dy2[b][m+j-7][co]      (r = 0, 1)
//
// Both are "64 output channels x K = 512" contractions over a window of input pixels (forward: 32
// channels x 16 taps at stride 2; dgrad: the two output parities stacked as 64 virtual channels,
// 64 channels x 8 taps at stride 1; the parity pair (2m, 2m+1) x 32 channels is one contiguous
// 64-element row of da1, so the dgrad output is a plain (pixel, 64) image with a per-clip stride).
// The op sits on the HBM/MFMA balance point (256 FLOP per HBM byte), so the kernel is built to
// stream: each wave keeps its 32 output channels x 512 weights in registers for the whole launch
// (A operand, 128 VGPRs); two 4-wave workgroups per CU walk (clip, 128-pixel) items; the input
// window of item i+2 is loaded raw into registers while item i computes, and item i+1's window
// (loaded one item earlier) is BN-affine+ReLU'd and bf16-packed on its way into the other half of
// a double-buffered LDS window (one LDS-only barrier per item; output stores are never waited
// for).  Every input byte is read from HBM once per item (window overlap 16 / 8 pixels), every
// output byte written once, weights never re-streamed (the row-window kernel re-read 64 KB of
// weights per 256 output pixels).  MFMA: D[co][px] = W[co][k] x window^T[k][px], the accumulator
// rows are output channels, so after one v_permlane32_swap per register pair each lane holds two
// runs of 8 contiguous channels of one pixel and stores them as 16-B vectors without an LDS pass.
// Measured at B=256 (tools/bench_fe.py): the load+store stream alone (no MFMA) takes 0.71 ms
// (5.1 TB/s), the MFMA work alone 0.30-0.37 ms; the kernel lands at 0.98-1.15 ms.
#include "common.h"

#include <type_traits>

namespace {

constexpr int F1_DEPTH = 4;  // fe_conv1: waveform items in flight per wave (3 ahead; 0.506 -> 0.49 ms, 6: no gain)
constexpr int FE_NT = 256;
constexpr int FE_BM = 128;  // output pixels per item (4 waves: 2 channel halves x 2 pixel halves)
constexpr int FE_N = 64;    // output channels

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int CIN, int KW, int S>
struct FeCfg {
  static constexpr int CG = CIN / 8;                    // 16-B chunks per pixel
  static constexpr int WPX = (FE_BM - 1) * S + KW;      // window pixels per item
  static constexpr int HALF = (WPX + 1) / 2;            // stride 2: even pixels, then odd pixels
  static constexpr int NSLOT = S == 1 ? WPX : 2 * HALF;
  static constexpr int PSB = CIN * 2 + 16;              // LDS bytes per pixel (conflict-free b128 reads)
  static constexpr int WBYTES = NSLOT * PSB;
  static constexpr int NCH = WPX * CG;
  static constexpr int LCH = (NCH + FE_NT - 1) / FE_NT;  // window chunks per thread
  static constexpr int KS = KW * CIN / 16;              // MFMA k-steps
  static_assert(FE_NT % CG == 0, "channel chunk must be constant per thread");
  static_assert(KS == 32, "weights-in-registers layout assumes K = 512");
};

struct FeArgs {
  const bf16* x;      // (n, win, CIN)
  const float* ps;    // pre-op scale/shift per input channel (BN1 affine, then ReLU) or null
  const float* pt;
  const bf16* w;      // (64, KW*CIN), k = kx*CIN + ci
  const float* bias;  // (64) or null
  bf16* y;            // y[b*ystride + m*64 + n], stored while m < wout and m*64+n < ylen
  int n, win, wout, pw, nitem;
  int64_t ystride, ylen;
};

template <int S, int HALF>
__device__ __forceinline__ int fe_slot(int p) {
  if constexpr (S == 1) return p;
  else return (p & 1) * HALF + (p >> 1);
}

__device__ __forceinline__ u32x4 fe_cook(u32x4 u, bool ok, bool pre, const float* sc, const float* sh) {
  if (!ok) return u32x4{0u, 0u, 0u, 0u};
  if (!pre) return u;
  uint32_t w4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = fmaxf(fmaf(__uint_as_float(u[i] << 16), sc[2 * i], sh[2 * i]), 0.f);
    const float hi = fmaxf(fmaf(__uint_as_float(u[i] & 0xffff0000u), sc[2 * i + 1], sh[2 * i + 1]), 0.f);
    w4[i] = pk_bf16(lo, hi);
  }
  return u32x4{w4[0], w4[1], w4[2], w4[3]};
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) { return pk_bf16(lo, hi); }

#ifdef FE_STAMP
__device__ unsigned long long g_fe_st[64 * 4 * 256 * 8];
#endif
template <int CIN, int KW, int S, bool PRE>
__global__ __launch_bounds__(FE_NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void feconv_kernel(FeArgs g) {
  using Cfg = FeCfg<CIN, KW, S>;
  __shared__ __attribute__((aligned(16))) char smem[2 * Cfg::WBYTES];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nh = wave & 1, pq = wave >> 1;
  const int cg = t % Cfg::CG;
  const int items = g.n * g.nitem;
  if ((int)blockIdx.x >= items) return;  // whole block

  // weights as MFMA A fragments: row co = nh*32 + (lane & 31), k = ks*16 + 8*(lane >> 5) .. +7
  bf16x8 wf[Cfg::KS];
  {
    const bf16* wr = g.w + (int64_t)(nh * 32 + (lane & 31)) * (KW * CIN) + 8 * (lane >> 5);
#pragma unroll
    for (int ks = 0; ks < Cfg::KS; ++ks) wf[ks] = *reinterpret_cast<const bf16x8*>(wr + ks * 16);
  }
  // after the half swap this lane owns channels c0..c0+7 and c0+16..c0+23 of its pixel; the bias
  // lives in LDS (read back per tile) to leave registers for the second window set
  const int c0 = nh * 32 + 8 * (lane >> 5);
  // (bias and the input pre-op scale/shift live in LDS and are read where used: registers go to the
  // weights, the accumulators and the two in-flight window sets)
  __shared__ __attribute__((aligned(16))) float sbias[FE_N];
  __shared__ __attribute__((aligned(16))) float spre[2][CIN];
  if (t < FE_N) sbias[t] = g.bias ? g.bias[t] : 0.f;
  if (PRE && t < CIN) {
    spre[0][t] = g.ps[t];
    spre[1][t] = g.pt[t];
  }

  // Two register sets of raw window chunks: while item k computes, item k+1's window (loaded during
  // item k-1) waits in one set and item k+2's loads are in flight into the other.
  u32x4 rawa[Cfg::LCH], rawb[Cfg::LCH];
  uint32_t oka = 0, okb = 0;
  // Buffer loads with 32-bit byte offsets (the host keeps a launch's input under 2 GB): a chunk
  // outside the window or the clip gets an offset past num_records and reads zeros, so no load
  // is predicated and no 64-bit address temporaries compete with the in-flight register sets.
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(g.x), (short)0, (int)((int64_t)g.n * g.win * CIN * 2), 0x00020000);
  auto load = [&](int it, u32x4 (&raw)[Cfg::LCH], uint32_t& rok) __attribute__((always_inline)) {
    it = it < items ? it : items - 1;  // past the end: a harmless redundant load
    const int b = it / g.nitem;
    const int px0 = (it - b * g.nitem) * FE_BM * S - g.pw;
    rok = 0;
#pragma unroll
    for (int s = 0; s < Cfg::LCH; ++s) {
      const int q = t + FE_NT * s;
      const int p = q / Cfg::CG;
      const int ix = px0 + p;
      const bool ok = p < Cfg::WPX && ix >= 0 && ix < g.win;
      const unsigned off = ok ? (unsigned)((b * g.win + ix) * Cfg::CG + cg) * 16u : 0x80000000u;
      raw[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      rok |= (uint32_t)ok << s;
    }
  };
  auto store = [&](int buf, const u32x4 (&raw)[Cfg::LCH], uint32_t rok) __attribute__((always_inline)) {
    float sc[8], sh[8];
    if constexpr (PRE) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&spre[0][cg * 8 + 4 * h]);
        const f32x4 c = *reinterpret_cast<const f32x4*>(&spre[1][cg * 8 + 4 * h]);
#pragma unroll
        for (int q = 0; q < 4; ++q) { sc[4 * h + q] = a[q]; sh[4 * h + q] = c[q]; }
      }
    }
#pragma unroll
    for (int s = 0; s < Cfg::LCH; ++s) {
      const int q = t + FE_NT * s;
      const int p = q / Cfg::CG;
      if (Cfg::NCH % FE_NT == 0 || p < Cfg::WPX)
        *reinterpret_cast<u32x4*>(smem + buf * Cfg::WBYTES + fe_slot<S, Cfg::HALF>(p) * Cfg::PSB + cg * 16) =
            fe_cook(raw[s], (rok >> s) & 1u, PRE, sc, sh);
    }
  };
  auto compute = [&](int buf, f32x16 (&acc)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const char* win = smem + buf * Cfg::WBYTES;
#pragma unroll
    for (int ks = 0; ks < Cfg::KS; ++ks) {
      constexpr int KPC = CIN / 16;  // k-steps per tap
      const int kx = ks / KPC;
      const int ci = (ks % KPC) * 16 + 8 * (lane >> 5);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int px = pq * 64 + i * 32 + (lane & 31);
        int slot;
        if constexpr (S == 1) slot = px + kx;
        else slot = (kx & 1) * Cfg::HALF + px + (kx >> 1);
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(win + slot * Cfg::PSB + ci * 2);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], fb, acc[i], 0, 0, 0);
      }
    }
  };
  // epilogue: rows of acc are channels nh*32 + (r&3) + 8*(r>>2) + 4*(lane>>5); swap halves so the
  // lane holds channels c0..c0+7 (v[0..7]) and c0+16..c0+23 (v[8..15]) of one pixel
  auto epilogue = [&](int item, const f32x16 (&acc)[2]) __attribute__((always_inline)) {
    const int b = item / g.nitem;
    const int m0 = (item - b * g.nitem) * FE_BM + pq * 64;
    bf16* yb = g.y + (int64_t)b * g.ystride;
    float bv[16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 u0 = *reinterpret_cast<const f32x4*>(sbias + c0 + 16 * h);
      const f32x4 u1 = *reinterpret_cast<const f32x4*>(sbias + c0 + 16 * h + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) { bv[8 * h + q] = u0[q]; bv[8 * h + 4 + q] = u1[q]; }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float v[16];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // (__float_as_uint of a copied element: clang folds __builtin_bit_cast of a vector-element
          // lvalue to element 0)
          const float lo = acc[i][8 * h + j], hi = acc[i][8 * h + 4 + j];
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
          v[8 * h + j] = __builtin_bit_cast(float, (unsigned)r[0]);
          v[8 * h + 4 + j] = __builtin_bit_cast(float, (unsigned)r[1]);
        }
      const int m = m0 + i * 32 + (lane & 31);
      if (m < g.wout) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int64_t e = (int64_t)m * FE_N + c0 + 16 * h;
          if (e < g.ylen) {
            const u32x4 o = {pack2(v[8 * h] + bv[8 * h], v[8 * h + 1] + bv[8 * h + 1]),
                             pack2(v[8 * h + 2] + bv[8 * h + 2], v[8 * h + 3] + bv[8 * h + 3]),
                             pack2(v[8 * h + 4] + bv[8 * h + 4], v[8 * h + 5] + bv[8 * h + 5]),
                             pack2(v[8 * h + 6] + bv[8 * h + 6], v[8 * h + 7] + bv[8 * h + 7])};
            *reinterpret_cast<u32x4*>(yb + e) = o;
          }
        }
      }
    }
  };
  // one item: issue item+2G's loads into `ld`, compute from LDS half `buf`, store the outputs, move
  // item+G's raw window (`st`, loaded one item earlier) into the other half, barrier (LDS only: the
  // global stores stay in flight across it)
#ifdef FE_STAMP  // timing builds only (tools/fe_stamps.py): s_memtime per item segment
  unsigned long long ts[8] = {};
  int kst = 0;
#define FT(k) ts[k] = __builtin_amdgcn_s_memtime()
#else
#define FT(k)
#endif
  auto step = [&](int item, int buf, u32x4 (&ld)[Cfg::LCH], uint32_t& ldok, const u32x4 (&st)[Cfg::LCH],
                  uint32_t stok) __attribute__((always_inline)) {
    FT(0);
    load(item + 2 * (int)gridDim.x, ld, ldok);
    FT(1);
    f32x16 acc[2];
    compute(buf, acc);
    FT(2);
    epilogue(item, acc);      // global stores issue behind the in-flight loads; nothing waits for them
    FT(3);
    store(buf ^ 1, st, stok);  // waits only for `st`'s loads (issued an item ago)
    FT(4);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    FT(5);
    __builtin_amdgcn_s_barrier();
#ifdef FE_STAMP
    FT(6);
    if (blockIdx.x < 64 && kst < 256 && lane == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) g_fe_st[(((int)blockIdx.x * 4 + wave) * 256 + kst) * 8 + k] = ts[k];
    }
    ++kst;
#endif
  };

  int item = blockIdx.x;
  load(item, rawa, oka);
  load(item + (int)gridDim.x, rawb, okb);
  __syncthreads();  // sbias / spre visible
  store(0, rawa, oka);
  __syncthreads();
  for (;;) {
    step(item, 0, rawa, oka, rawb, okb);
    item += gridDim.x;
    if (item >= items) break;
    step(item, 1, rawb, okb, rawa, oka);
    item += gridDim.x;
    if (item >= items) break;
  }
}

// Warp-specialised form of feconv_kernel: one 8-wave workgroup per CU.  Waves 0-3 only compute (weights in
// registers, 64 MFMAs per item from the LDS window, the swap epilogue's stores); waves 4-7 only feed: they keep
// FS_DEPTH items of raw window loads in flight in their own registers and cook (BN1 affine + ReLU, bf16 pack)
// the next item's window into the other half of the double-buffered LDS window.  One barrier per item hands
// the window over.  The two roles meet on every SIMD (one compute + one feeder wave each), so the feeders'
// VALU and load issue run under the compute waves' MFMAs instead of in a phase of their own.
constexpr int FS_NT = 512;
#ifndef FS_DEPTH
#define FS_DEPTH 3  // raw window loads in flight per feeder thread (items k+1 .. k+3)
#endif
#ifndef FS_FD
#define FS_FD 4  // k-steps of B fragments in flight per compute wave
#endif

// (lds_barrier, common.h: the feeders' window loads and the compute waves' output stores stay in flight across it)

template <int CIN, int KW, int S, bool PRE>
__global__ __launch_bounds__(FS_NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void feconv_ws_kernel(FeArgs g) {
  using Cfg = FeCfg<CIN, KW, S>;
  __shared__ __attribute__((aligned(16))) char smem[2 * Cfg::WBYTES];
  __shared__ __attribute__((aligned(16))) float sbias[FE_N];
  __shared__ __attribute__((aligned(16))) float spre[2][CIN];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int items = g.n * g.nitem;
  if ((int)blockIdx.x >= items) return;  // whole block
  const int nk = (items - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;  // items of this workgroup
  if (t < FE_N) sbias[t] = g.bias ? g.bias[t] : 0.f;
  if (PRE && t < CIN) {
    spre[0][t] = g.ps[t];
    spre[1][t] = g.pt[t];
  }
  if (wave < 4) {
    // ---- compute waves: (channel half nh, pixel half pq) of every item, as in feconv_kernel
    const int nh = wave & 1, pq = wave >> 1;
    bf16x8 wf[Cfg::KS];
    {
      const bf16* wr = g.w + (int64_t)(nh * 32 + (lane & 31)) * (KW * CIN) + 8 * (lane >> 5);
#pragma unroll
      for (int ks = 0; ks < Cfg::KS; ++ks) wf[ks] = *reinterpret_cast<const bf16x8*>(wr + ks * 16);
    }
    const int c0 = nh * 32 + 8 * (lane >> 5);
    lds_barrier();  // sbias / spre in
    lds_barrier();  // item 0's window in
#pragma unroll 1
    for (int k = 0; k < nk; ++k) {
      const int item = (int)blockIdx.x + k * (int)gridDim.x;
      f32x16 acc[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      const char* win = smem + (k & 1) * Cfg::WBYTES;
      // B fragments FS_FD k-steps ahead of their MFMAs (a register ring; one wave per SIMD computes, so nothing
      // else covers an LDS read's latency)
      auto frag = [&](int ks, int i) __attribute__((always_inline)) {
        constexpr int KPC = CIN / 16;
        const int kx = ks / KPC;
        const int ci = (ks % KPC) * 16 + 8 * (lane >> 5);
        const int px = pq * 64 + i * 32 + (lane & 31);
        int slot;
        if constexpr (S == 1) slot = px + kx;
        else slot = (kx & 1) * Cfg::HALF + px + (kx >> 1);
        return *reinterpret_cast<const bf16x8*>(win + slot * Cfg::PSB + ci * 2);
      };
#ifdef FS_PROBE_NOCOMPUTE  // timing probe only: no MFMA work (outputs are the bias)
      if (g.n < 0)
#endif
      {
        bf16x8 fr[FS_FD][2];
#pragma unroll
        for (int ks = 0; ks < FS_FD; ++ks)
#pragma unroll
          for (int i = 0; i < 2; ++i) fr[ks][i] = frag(ks, i);
#pragma unroll
        for (int ks = 0; ks < Cfg::KS; ++ks) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], fr[ks % FS_FD][i], acc[i], 0, 0, 0);
            if (ks + FS_FD < Cfg::KS) fr[ks % FS_FD][i] = frag(ks + FS_FD, i);
          }
        }
        // pin the ring (the scheduler otherwise sinks each read next to its MFMA): the first FS_FD k-steps' reads,
        // then per k-step its 2 MFMAs and the 2 reads FS_FD ahead
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * FS_FD, 0);
#pragma unroll
        for (int ks = 0; ks < Cfg::KS; ++ks) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          if (ks + FS_FD < Cfg::KS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
      }
      const int b = item / g.nitem;
      const int m0 = (item - b * g.nitem) * FE_BM + pq * 64;
      bf16* yb = g.y + (int64_t)b * g.ystride;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[16];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float lo = acc[i][8 * h + j], hi = acc[i][8 * h + 4 + j];
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
            v[8 * h + j] = __builtin_bit_cast(float, (unsigned)r[0]);
            v[8 * h + 4 + j] = __builtin_bit_cast(float, (unsigned)r[1]);
          }
        const int m = m0 + i * 32 + (lane & 31);
        if (m < g.wout) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int64_t e = (int64_t)m * FE_N + c0 + 16 * h;
            if (e < g.ylen) {
              const f32x4 u0 = *reinterpret_cast<const f32x4*>(sbias + c0 + 16 * h);
              const f32x4 u1 = *reinterpret_cast<const f32x4*>(sbias + c0 + 16 * h + 4);
              const u32x4 o = {pack2(v[8 * h] + u0[0], v[8 * h + 1] + u0[1]), pack2(v[8 * h + 2] + u0[2], v[8 * h + 3] + u0[3]),
                               pack2(v[8 * h + 4] + u1[0], v[8 * h + 5] + u1[1]), pack2(v[8 * h + 6] + u1[2], v[8 * h + 7] + u1[3])};
              *reinterpret_cast<u32x4*>(yb + e) = o;
            }
          }
        }
      }
      lds_barrier();  // this item's window reads are done; the next window is in
    }
  } else {
    // ---- feeder waves: thread ft plays feconv_kernel's thread t for the window loads and the staging
    const int ft = t - 256;
    const int cg = ft % Cfg::CG;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(g.x), (short)0, (int)((int64_t)g.n * g.win * CIN * 2), 0x00020000);
    auto load = [&](int k, u32x4 (&raw)[Cfg::LCH], uint32_t& rok) __attribute__((always_inline)) {
      int it = (int)blockIdx.x + k * (int)gridDim.x;
      it = it < items ? it : items - 1;  // past the end: a harmless redundant load
      const int b = it / g.nitem;
      const int px0 = (it - b * g.nitem) * FE_BM * S - g.pw;
      rok = 0;
#pragma unroll
      for (int s = 0; s < Cfg::LCH; ++s) {
        const int q = ft + FE_NT * s;
        const int p = q / Cfg::CG;
        const int ix = px0 + p;
        const bool ok = p < Cfg::WPX && ix >= 0 && ix < g.win;
        const unsigned off = ok ? (unsigned)((b * g.win + ix) * Cfg::CG + cg) * 16u : 0x80000000u;
#ifdef FS_PROBE_NOLOAD  // timing probe only: no window loads (the staged windows are zeros)
        raw[s] = u32x4{0u, 0u, 0u, 0u};
        (void)off;
#else
        raw[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
#endif
        rok |= (uint32_t)ok << s;
      }
    };
    auto stage = [&](int buf, const u32x4 (&raw)[Cfg::LCH], uint32_t rok) __attribute__((always_inline)) {
      float sc[8], sh[8];
      if constexpr (PRE) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(&spre[0][cg * 8 + 4 * h]);
          const f32x4 c = *reinterpret_cast<const f32x4*>(&spre[1][cg * 8 + 4 * h]);
#pragma unroll
          for (int q = 0; q < 4; ++q) { sc[4 * h + q] = a[q]; sh[4 * h + q] = c[q]; }
        }
      }
#pragma unroll
      for (int s = 0; s < Cfg::LCH; ++s) {
        const int q = ft + FE_NT * s;
        const int p = q / Cfg::CG;
        if (Cfg::NCH % FE_NT == 0 || p < Cfg::WPX)
          *reinterpret_cast<u32x4*>(smem + buf * Cfg::WBYTES + fe_slot<S, Cfg::HALF>(p) * Cfg::PSB + cg * 16) =
              fe_cook(raw[s], (rok >> s) & 1u, PRE, sc, sh);
      }
    };
    u32x4 raw[FS_DEPTH][Cfg::LCH];
    uint32_t rok[FS_DEPTH];
#pragma unroll
    for (int d = 0; d < FS_DEPTH; ++d) load(d, raw[d], rok[d]);
    lds_barrier();  // sbias / spre in
    stage(0, raw[0], rok[0]);
    lds_barrier();  // item 0's window in
    // iteration k: item k + FS_DEPTH's loads into the set item k used, item k + 1's window staged into half
    // (k + 1) & 1 (its loads were issued FS_DEPTH - 1 items ago), barrier.  Unrolled by 12 (a multiple of 2 and
    // of FS_DEPTH) so the register set and the LDS half are compile-time.
    static_assert(12 % FS_DEPTH == 0, "feeder unroll");
    auto iter = [&](auto KC, int k) __attribute__((always_inline)) {
      constexpr int R = decltype(KC)::value;  // k % 12
      constexpr int SET = R % FS_DEPTH, NXT = (R + 1) % FS_DEPTH;
      load(k + FS_DEPTH, raw[SET], rok[SET]);
      if (k + 1 < nk) stage((R + 1) & 1, raw[NXT], rok[NXT]);
      lds_barrier();  // the staged window is in LDS
    };
    // iterations k .. k + 11, stopping after the workgroup's last item
    auto step = [&](auto KC, int k) __attribute__((always_inline)) {
      const int kk = k + decltype(KC)::value;
      if (kk < nk) iter(KC, kk);
      return kk + 1 < nk;
    };
#pragma unroll 1
    for (int k = 0; k < nk; k += 12) {
      using std::integral_constant;
      (void)(step(integral_constant<int, 0>{}, k) && step(integral_constant<int, 1>{}, k) &&
             step(integral_constant<int, 2>{}, k) && step(integral_constant<int, 3>{}, k) &&
             step(integral_constant<int, 4>{}, k) && step(integral_constant<int, 5>{}, k) &&
             step(integral_constant<int, 6>{}, k) && step(integral_constant<int, 7>{}, k) &&
             step(integral_constant<int, 8>{}, k) && step(integral_constant<int, 9>{}, k) &&
             step(integral_constant<int, 10>{}, k) && step(integral_constant<int, 11>{}, k));
    }
  }
}

// ---------------------------------------------------------------- conv1 forward + BN1 statistics
//   y1[b][o][c] = bias[c] + sum_{k<64} w[c][k] * x[b][2o+k]        (envnet_v2.py:15, 1 -> 32 channels)
// Wave-persistent (no barriers): a wave owns (clip, 32-pixel) items; the 4 weight fragments (32
// channels x 64 taps) stay in registers as the MFMA A operand; the item's 126-sample waveform
// segment is one 8-byte load per lane (the next item's is in flight while this one computes),
// rounded to bf16 into a per-wave LDS strip from which the Toeplitz B fragments are read.  After the half swap each lane holds
// 16 channels of one pixel (2 x 16-B chunks, regrouped through a per-wave LDS image into two 1 KB
// runs of whole rows, stored non-temporal), and the BN1 batch statistics of the stored (bf16)
// values are accumulated on the fly about K[c] = bias[c] (the waveform is zero-mean, so the
// shifted sums are well conditioned) -> per-wave partial [C][2] -> bn finalize in double.
struct F1Args {
  const float* x;     // (n, t)
  const bf16* w;      // (32, 64)
  const float* bias;  // (32)
  bf16* y;            // (n, w1, 32)
  float* part;        // [waves][32][2] shifted sums, or null
  int n, t, w1, nitem;
};

template <bool STATS>
__global__ __launch_bounds__(256) void fe_conv1_kernel(F1Args g) {
  // per-wave LDS: the item's 126-sample segment as bf16 dwords (2 samples each), twice: copy 0 at
  // dword 0 and copy 1 shifted by one dword at dword 96 (+32 banks), so every 8-sample B fragment
  // is two 8-byte-aligned ds_read_b64 from the copy matching its start parity, conflict-free
  __shared__ __attribute__((aligned(16))) uint32_t seg[4][160];
  __shared__ __attribute__((aligned(16))) char stage[4][2048];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
  const int items = g.n * g.nitem;
  uint32_t* sg = seg[wv];
  bf16x8 wa[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) wa[ks] = *reinterpret_cast<const bf16x8*>(g.w + (lane & 31) * 64 + ks * 16 + 8 * (lane >> 5));
  const int c0 = 8 * (lane >> 5);
  float bv[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { bv[i] = g.bias[c0 + i]; bv[8 + i] = g.bias[c0 + 16 + i]; }
  float s1[16], s2[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { s1[i] = 0.f; s2[i] = 0.f; }

  typedef float f32x2 __attribute__((ext_vector_type(2)));
  // lane l loads samples 2l, 2l+1 of the item's segment x[b][2*o0 .. 2*o0+125] (clamped in-clip)
  auto load = [&](int it) __attribute__((always_inline)) {
    it = it < items ? it : items - 1;
    const int b = it / g.nitem;
    const int o0 = (it - b * g.nitem) * 32;
    int s0 = 2 * o0 + 2 * lane;
    s0 = s0 < g.t - 2 ? s0 : g.t - 2;
    return *reinterpret_cast<const f32x2*>(g.x + (int64_t)b * g.t + s0);
  };
  auto run = [&](int it, f32x2 xr) __attribute__((always_inline)) {
    const uint32_t d = pk_bf16(xr[0], xr[1]);
    wave_sync();  // the previous item's fragment reads are done
    sg[lane] = d;
    if (lane >= 1) sg[96 + lane - 1] = d;
    wave_sync();
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    const int o = lane & 31;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int D = o + 4 * (lane >> 5) + 8 * ks;  // first dword of this lane's 8 samples
      const uint32_t* src = (D & 1) ? sg + 96 + D - 1 : sg + D;
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 p0 = *reinterpret_cast<const u32x2*>(src);
      const u32x2 p1 = *reinterpret_cast<const u32x2*>(src + 2);
      const u32x4 f = {p0[0], p0[1], p1[0], p1[1]};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ks], __builtin_bit_cast(bf16x8, f), acc, 0, 0, 0);
    }
    float v[16];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a0 = acc[8 * h + j], a1 = acc[8 * h + 4 + j];
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a1), false, false);
        v[8 * h + j] = __builtin_bit_cast(float, (unsigned)sw[0]);
        v[8 * h + 4 + j] = __builtin_bit_cast(float, (unsigned)sw[1]);
      }
    const int b = it / g.nitem;
    const int op0 = (it - b * g.nitem) * 32;
    const int op = op0 + o;
    // the item's 32 pixels x 64 B are one contiguous 2 KB run of y1: staged through a per-wave LDS
    // image (16-B chunk k of row r at chunk k ^ ((r >> 1) & 3): conflict-free writes and reads) and
    // stored as two 1 KB runs (16 rows x 4 chunks per instruction, non-temporal: y1 is next read
    // after ~2 GB of other traffic) instead of 32 half rows: 0.65 -> 0.50 ms at B = 256
    char* stg = stage[wv];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = 8 * h + 2 * i;
        w4[i] = pk_bf16(v[e] + bv[e], v[e + 1] + bv[e + 1]);
        if constexpr (STATS) {
          if (op < g.w1) {
            const float d0 = __uint_as_float(w4[i] << 16) - bv[e], d1 = __uint_as_float(w4[i] & 0xffff0000u) - bv[e + 1];
            s1[e] += d0; s2[e] = fmaf(d0, d0, s2[e]);
            s1[e + 1] += d1; s2[e + 1] = fmaf(d1, d1, s2[e + 1]);
          }
        }
      }
      const int k = (lane >> 5) + 2 * h;
      *reinterpret_cast<u32x4*>(stg + o * 64 + ((k ^ ((o >> 1) & 3)) << 4)) = u32x4{w4[0], w4[1], w4[2], w4[3]};
    }
    wave_sync();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 16 * h + (lane >> 2), k = lane & 3;
      const u32x4 q = *reinterpret_cast<const u32x4*>(stg + r * 64 + ((k ^ ((r >> 1) & 3)) << 4));
      if (op0 + r < g.w1) __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(g.y + ((int64_t)b * g.w1 + op0 + r) * 32 + 8 * k));
    }
  };

  int it = gw;
  // the waveform loads (8 B per lane) run F1_DEPTH - 1 items ahead of their use
  if (it < items) {
    f32x2 xr[F1_DEPTH];
#pragma unroll
    for (int d = 0; d + 1 < F1_DEPTH; ++d) xr[d] = load(it + d * nw);
    bool more = true;
    while (more) {
#pragma unroll
      for (int u = 0; u < F1_DEPTH; ++u) {
        xr[(u + F1_DEPTH - 1) % F1_DEPTH] = load(it + (F1_DEPTH - 1) * nw);
        run(it, xr[u]);
        it += nw;
        if (it >= items) { more = false; break; }
      }
    }
  }
  if constexpr (STATS) {
    // sum over the 32 lanes that hold the same channels (lane bit 5 fixed), fixed butterfly order
#pragma unroll
    for (int i = 0; i < 16; ++i) {
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) {
        s1[i] += __shfl_xor(s1[i], m, 64);
        s2[i] += __shfl_xor(s2[i], m, 64);
      }
    }
    if ((lane & 31) == 0) {
      float* dst = g.part + (int64_t)gw * 64;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dst[(c0 + i) * 2] = s1[i];
        dst[(c0 + i) * 2 + 1] = s2[i];
        dst[(c0 + 16 + i) * 2] = s1[8 + i];
        dst[(c0 + 16 + i) * 2 + 1] = s2[8 + i];
      }
    }
  }
}

// ---------------------------------------------------------------- trunk conv3 forward + BN stats
//   y3[b][oy][ox][c] = bias[c] + sum_{ky,kx<8} w[c][ky][kx] * X0[b][oy+ky][ox+kx]   (envnet_v2.py:31,
// the 1 -> 32 channel 8x8 conv on the pooled frontend image).  Wave-persistent like conv1: the 4
// weight fragments (32 channels x 64 taps) are the MFMA A operand; per (clip, output row, 32-px)
// item the wave stages the 8 input rows x 40 samples it needs into a per-wave LDS strip as four
// copies shifted by 0..3 samples (80-B rows, copies 704 B = 48 banks apart: conflict-free 16-B staging
// writes and 8-B fragment reads; the 88-B pitch before cost 2-way staging conflicts, 0.305 -> 0.262 ms),
// so every 8-sample B fragment
// (k-step ks: kernel rows 2ks, 2ks+1 on the lane halves, kx = 0..7) is two aligned ds_read_b64 and
// the 32 lanes of a half hit 32 distinct bank pairs; BN3 statistics accumulate in the epilogue.
struct F3Args {
  const bf16* x;      // (n, h, w) 1-channel image
  const bf16* w;      // (32, 64) taps ky*8 + kx
  const float* bias;  // (32)
  bf16* y;            // (n, h-7, w-7, 32)
  float* part;        // [waves][32][2] or null
  int n, h, wd, oh, ow, nseg;
};

template <bool STATS>
__global__ __launch_bounds__(256) void fe_conv3_kernel(F3Args g) {
  constexpr int ROWB = 80, CPYB = 704;  // 80-B rows (conflict-free staging writes), copies 704 B apart (48 banks: conflict-free reads)
  __shared__ __attribute__((aligned(16))) char strip[4][4 * CPYB];
  __shared__ __attribute__((aligned(16))) char stage[4][2048];  // the item's 32 px x 64 B output run
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
  const int items = g.n * g.oh * g.nseg;
  char* sg = strip[wv];
  bf16x8 wa[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) wa[ks] = *reinterpret_cast<const bf16x8*>(g.w + (lane & 31) * 64 + ks * 16 + 8 * (lane >> 5));
  const int c0 = 8 * (lane >> 5);
  float bv[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { bv[i] = g.bias[c0 + i]; bv[8 + i] = g.bias[c0 + 16 + i]; }
  float s1[16], s2[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { s1[i] = 0.f; s2[i] = 0.f; }

  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  // staging lane l < 40: input row r = l / 5 of the item, samples 8q .. 8q+11 (q = l % 5) as three
  // 8-byte loads (row pitch 2*wd bytes is 8-byte aligned for wd % 4 == 0); past the row end -> 0
  struct Raw { u32x2 v[3]; };
  auto load = [&](int it) __attribute__((always_inline)) {
    Raw R;
    it = it < items ? it : items - 1;
    const int seg = it % g.nseg, rest = it / g.nseg;
    const int oy = rest % g.oh, b = rest / g.oh;
    const int l = lane < 40 ? lane : 0;
    const int r = l / 5, q = l % 5;
    const int col = seg * 32 + 8 * q;
    const bf16* src = g.x + ((int64_t)b * g.h + oy + r) * g.wd;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int c = col + 4 * k;
      R.v[k] = c + 4 <= g.wd ? *reinterpret_cast<const u32x2*>(src + c) : u32x2{0u, 0u};
    }
    return R;
  };
  auto run = [&](int it, const Raw& R) __attribute__((always_inline)) {
    wave_sync();  // the previous item's fragment reads are done
    if (lane < 40) {
      const int r = lane / 5, q = lane % 5;
      const uint32_t d[6] = {R.v[0][0], R.v[0][1], R.v[1][0], R.v[1][1], R.v[2][0], R.v[2][1]};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        // copy c dword i = samples (8q + c + 2i, +1)
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = c + 2 * i;  // first sample index within this lane's 12
          o[i] = (e & 1) ? ((d[e >> 1] >> 16) | (d[(e >> 1) + 1] << 16)) : d[e >> 1];
        }
        *reinterpret_cast<u32x4*>(sg + c * CPYB + r * ROWB + 16 * q) = u32x4{o[0], o[1], o[2], o[3]};
      }
    }
    wave_sync();
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    const int o = lane & 31, cp = o & 3, dw = (o - cp) >> 1;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const char* src = sg + cp * CPYB + (2 * ks + (lane >> 5)) * ROWB + dw * 4;
      const u32x2 p0 = *reinterpret_cast<const u32x2*>(src);
      const u32x2 p1 = *reinterpret_cast<const u32x2*>(src + 8);
      const u32x4 f = {p0[0], p0[1], p1[0], p1[1]};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[ks], __builtin_bit_cast(bf16x8, f), acc, 0, 0, 0);
    }
    float v[16];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a0 = acc[8 * h + j], a1 = acc[8 * h + 4 + j];
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a1), false, false);
        v[8 * h + j] = __builtin_bit_cast(float, (unsigned)sw[0]);
        v[8 * h + 4 + j] = __builtin_bit_cast(float, (unsigned)sw[1]);
      }
    const int seg = it % g.nseg, rest = it / g.nseg;
    const int oy = rest % g.oh, b = rest / g.oh;
    const int ox0 = seg * 32, ox = ox0 + o;
    // as fe_conv1: the item's 32 output pixels x 64 B regrouped through the per-wave LDS image into two
    // 1 KB runs of whole rows, stored non-temporal
    char* stg = stage[wv];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = 8 * h + 2 * i;
        w4[i] = pk_bf16(v[e] + bv[e], v[e + 1] + bv[e + 1]);
        if constexpr (STATS) {
          if (ox < g.ow) {
            const float d0 = __uint_as_float(w4[i] << 16) - bv[e], d1 = __uint_as_float(w4[i] & 0xffff0000u) - bv[e + 1];
            s1[e] += d0; s2[e] = fmaf(d0, d0, s2[e]);
            s1[e + 1] += d1; s2[e + 1] = fmaf(d1, d1, s2[e + 1]);
          }
        }
      }
      const int k = (lane >> 5) + 2 * h;
      *reinterpret_cast<u32x4*>(stg + o * 64 + ((k ^ ((o >> 1) & 3)) << 4)) = u32x4{w4[0], w4[1], w4[2], w4[3]};
    }
    wave_sync();
    bf16* yrow = g.y + (((int64_t)b * g.oh + oy) * g.ow + ox0) * 32;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 16 * h + (lane >> 2), k = lane & 3;
      const u32x4 q = *reinterpret_cast<const u32x4*>(stg + r * 64 + ((k ^ ((r >> 1) & 3)) << 4));
      if (ox0 + r < g.ow) __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(yrow + r * 32 + 8 * k));
    }
  };

  int it = gw;
  if (it < items) {
    Raw ra = load(it), rb;
    for (;;) {
      rb = load(it + nw);
      run(it, ra);
      it += nw;
      if (it >= items) break;
      ra = load(it + nw);
      run(it, rb);
      it += nw;
      if (it >= items) break;
    }
  }
  if constexpr (STATS) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) {
        s1[i] += __shfl_xor(s1[i], m, 64);
        s2[i] += __shfl_xor(s2[i], m, 64);
      }
    }
    if ((lane & 31) == 0) {
      float* dst = g.part + (int64_t)gw * 64;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dst[(c0 + i) * 2] = s1[i];
        dst[(c0 + i) * 2 + 1] = s2[i];
        dst[(c0 + 16 + i) * 2] = s1[8 + i];
        dst[(c0 + 16 + i) * 2 + 1] = s2[8 + i];
      }
    }
  }
}

// ---------------------------------------------------------------- conv2 weight gradient
//   dW[co][kx*32 + ci] = sum_{b,o} dy2[b][o][co] * relu(bn1(y1))[b][2o+kx][ci]      (64 x 512, K = pixels)
// Persistent, gradient-stationary: one 8-wave workgroup per CU walks (clip, 128-pixel) items and
// keeps its 64 x 512 partial sum in registers (wave w: kernel taps kx = 2w, 2w+1 for all 64 output
// channels, 4 tiles = 64 VGPRs) for the whole launch; per item the dY tile [128 px][64 co] and the
// BN+ReLU'd input window [270 px][32 ci] (even/odd pixel split, so the stride-2 taps are
// consecutive slots) go through a double-buffered LDS stage with two register sets of raw loads in
// flight (items k+1, k+2), and both MFMA operands are transposed LDS reads (ds_read_b64_tr_b16).
// Every input byte is read once per item (window overlap 14 px); one f32 slab per workgroup, summed
// by the split-K reducer.
constexpr int FW_NT = 512;
constexpr int FW_BP = 128;

struct FwArgs {
  const bf16* dy;     // (n, wout, 64)
  const bf16* x;      // (n, win, 32)
  const float* ps;    // BN1 scale/shift (+ReLU) on x, or null
  const float* pt;
  int n, win, wout, nitem;
  float* ws;          // slab [blockIdx.x][64][512]
};

typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 fw_tr(const char* p0, int stride) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * stride));
  const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, c);
}

template <bool PRE>
__global__ __launch_bounds__(FW_NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void fe_wgrad_kernel(FwArgs g) {
  constexpr int C = 32, KW = 16;
  constexpr int WPX = (FW_BP - 1) * 2 + KW;   // 270 window pixels
  constexpr int HALF = (WPX + 1) / 2;         // 135: odd pixels start here
  constexpr int PSB = 64;                     // window pixel stride (conflict-free transposed reads)
  constexpr int DSB = 192;                    // dY pixel stride (48 dwords: 4 rows hit disjoint banks)
  constexpr int WBY = 2 * HALF * PSB;
  constexpr int DBY = FW_BP * DSB;
  constexpr int BUF = WBY + DBY;
  constexpr int WCH = WPX * 4;                // 16-B window chunks per item (1080)
  constexpr int WL = (WCH + FW_NT - 1) / FW_NT;  // 3
  constexpr int DL = FW_BP * 8 / FW_NT;          // 2
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  __shared__ __attribute__((aligned(16))) float spre[2][C];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int items = g.n * g.nitem;
  if (PRE && t < C) {
    spre[0][t] = g.ps[t];
    spre[1][t] = g.pt[t];
  }
  const int cgw = t & 3;   // window chunk: 8 input channels
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(g.x), (short)0, (int)((int64_t)g.n * g.win * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(g.dy), (short)0, (int)((int64_t)g.n * g.wout * 64 * 2), 0x00020000);

  u32x4 wa[WL], wb[WL], da[DL], db[DL];
  auto load = [&](int it, u32x4 (&w)[WL], u32x4 (&d)[DL]) __attribute__((always_inline)) {
    it = it < items ? it : items - 1;
    const int b = it / g.nitem;
    const int o0 = (it - b * g.nitem) * FW_BP;
#pragma unroll
    for (int s = 0; s < WL; ++s) {
      const int q = t + FW_NT * s;
      const int p = q >> 2;
      const int ix = 2 * o0 + p;
      const bool ok = q < WCH && ix < g.win;
      const unsigned off = ok ? (unsigned)((b * g.win + ix) * 4 + cgw) * 16u : 0x80000000u;
      w[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
#pragma unroll
    for (int s = 0; s < DL; ++s) {
      const int q = t + FW_NT * s;
      const int p = q >> 3, cc = q & 7;
      const bool ok = o0 + p < g.wout;
      const unsigned off = ok ? (unsigned)((b * g.wout + o0 + p) * 8 + cc) * 16u : 0x80000000u;
      d[s] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(dr, off, 0, 0));
    }
  };
  // zero-filled raw chunks (padding) must stay zero after the pre-op: the window tail past the
  // clip reads zeros, and relu(0*sc + sh) != 0, so the valid bit is recomputed from the item here
  auto store = [&](int it, int buf, const u32x4 (&w)[WL], const u32x4 (&d)[DL]) __attribute__((always_inline)) {
    it = it < items ? it : items - 1;
    const int b = it / g.nitem;
    const int o0 = (it - b * g.nitem) * FW_BP;
    char* win = smem + buf * BUF;
    char* dyt = win + WBY;
    float sc[8], sh[8];
    if constexpr (PRE) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&spre[0][cgw * 8 + 4 * h]);
        const f32x4 c = *reinterpret_cast<const f32x4*>(&spre[1][cgw * 8 + 4 * h]);
#pragma unroll
        for (int q = 0; q < 4; ++q) { sc[4 * h + q] = a[q]; sh[4 * h + q] = c[q]; }
      }
    }
#pragma unroll
    for (int s = 0; s < WL; ++s) {
      const int q = t + FW_NT * s;
      const int p = q >> 2;
      if (q < WCH) {
        u32x4 v = w[s];
        if constexpr (PRE) {
          if (2 * o0 + p < g.win) {
            uint32_t w4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float lo = fmaxf(fmaf(__uint_as_float(v[i] << 16), sc[2 * i], sh[2 * i]), 0.f);
              const float hi = fmaxf(fmaf(__uint_as_float(v[i] & 0xffff0000u), sc[2 * i + 1], sh[2 * i + 1]), 0.f);
              w4[i] = pk_bf16(lo, hi);
            }
            v = u32x4{w4[0], w4[1], w4[2], w4[3]};
          }
        }
        const int slot = (p & 1) * HALF + (p >> 1);
        *reinterpret_cast<u32x4*>(win + slot * PSB + cgw * 16) = v;
      }
    }
#pragma unroll
    for (int s = 0; s < DL; ++s) {
      const int q = t + FW_NT * s;
      *reinterpret_cast<u32x4*>(dyt + (q >> 3) * DSB + (q & 7) * 16) = d[s];
    }
  };

  f32x16 acc[2][2];  // [mt][j]: output channels mt*32.., taps kx = 2*wave + j
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int i16 = lane & 15, gq = lane >> 4;
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* win = smem + buf * BUF;
    const char* dyt = win + WBY;
    constexpr int KS = FW_BP / 16;
    auto frags = [&](int ks, bf16x8 (&fa)[2], bf16x8 (&fb)[2]) __attribute__((always_inline)) {
      const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        fa[mt] = fw_tr(dyt + kr * DSB + (mt * 32 + 16 * (gq & 1) + 4 * (i16 & 3)) * 2, DSB);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int kx = 2 * wave + j;
        const int ci = 16 * (gq & 1) + 4 * (i16 & 3);
        const int slot = (kx & 1) * HALF + kr + (kx >> 1);
        fb[j] = fw_tr(win + slot * PSB + ci * 2, PSB);
      }
    };
    // the next k-step's 8 transposed reads are issued under this k-step's 4 MFMAs (2 per MFMA, pinned): the
    // compiler otherwise issues each k-step's reads after the previous MFMAs and drains lgkmcnt(0) before the 2nd
    // (bit-identical, fe_conv2_wgrad 1.134 -> 1.111 ms standalone)
    bf16x8 fa[2][2], fb[2][2];
    frags(0, fa[0], fb[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c = ks & 1;
      if (ks + 1 < KS) frags(ks + 1, fa[c ^ 1], fb[c ^ 1]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mt][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[c][mt], fb[c][j], acc[mt][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }
  };

  const int G = gridDim.x;
  int item = blockIdx.x;
  if (item < items) {
    load(item, wa, da);
    load(item + G, wb, db);
    __syncthreads();  // spre visible
    store(item, 0, wa, da);
    __syncthreads();
    for (;;) {
      load(item + 2 * G, wa, da);
      compute(0);
      store(item + G, 1, wb, db);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      item += G;
      if (item >= items) break;
      load(item + 2 * G, wb, db);
      compute(1);
      store(item + G, 0, wa, da);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      item += G;
      if (item >= items) break;
    }
  }
  // slab [64][512]: column n = kx*32 + ci
  float* dst = g.ws + (int64_t)blockIdx.x * 64 * 512;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = (2 * wave + j) * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        dst[(int64_t)m * 512 + n] = acc[mt][j][r];
      }
    }
}

int fe_grid(int items) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return items < 2 * ncu ? items : 2 * ncu;  // two workgroups per CU: their item phases drift apart, so
                                              // one's VALU epilogue/staging overlaps the other's MFMAs
}

// clips per launch so that one launch's input stays below 2 GB (32-bit buffer offsets)
int fe_clips_per_launch(int64_t clip_bytes) { return (int)(((1ll << 31) - 1) / clip_bytes); }

int fe_grid1(int items) {  // one workgroup per CU
  const int two = fe_grid(1 << 30);
  return items < two / 2 ? items : two / 2;
}

// dw[e] = sum over slabs (fixed order: deterministic)
__global__ __launch_bounds__(256) void fw_reduce_kernel(const float* __restrict__ ws, int slabs, int len,
                                                        float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= len) return;
  float acc = 0.f;
  for (int k = 0; k < slabs; ++k) acc += ws[(int64_t)k * len + e];
  out[e] = acc;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// conv2 forward form: warp-specialised unless MIA_FECONV_WS=0 (A/B runs, tools/bench_fe.py FE_AB=1)
bool fe_ws() { const char* e = getenv("MIA_FECONV_WS"); return !(e && e[0] == '0'); }

}  // namespace

extern "C" int mia_fe_conv2_fwd(const void* y1, const float* scale, const float* shift, const void* w,
                                const float* bias, void* y2, int32_t n, int32_t w1, int32_t w2,
                                mia_stream_t stream) {
  MIA_CHECK_ARG(y1 && w && y2 && n > 0 && w1 >= 16, "fe_conv2_fwd: bad arguments");
  MIA_CHECK_ARG(!scale == !shift, "fe_conv2_fwd: scale and shift go together");
  MIA_CHECK_ARG(w2 == (w1 - 16) / 2 + 1, "fe_conv2_fwd: w2 must be (w1-16)/2+1 (got w1=%d w2=%d)", w1, w2);
  MIA_CHECK_ARG(aligned16(y1) && aligned16(w) && aligned16(y2), "fe_conv2_fwd: operands must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int per = fe_clips_per_launch((int64_t)w1 * 32 * 2);
  MIA_CHECK_ARG(per > 0, "fe_conv2_fwd: one clip exceeds 2 GB");
  for (int c = 0; c < n; c += per) {
    const int nc = n - c < per ? n - c : per;
    FeArgs a{reinterpret_cast<const bf16*>(y1) + (int64_t)c * w1 * 32, scale, shift, reinterpret_cast<const bf16*>(w),
             bias, reinterpret_cast<bf16*>(y2) + (int64_t)c * w2 * FE_N, nc, w1, w2, 0, (int)cdiv(w2, FE_BM),
             (int64_t)w2 * FE_N, (int64_t)w2 * FE_N};
    // warp-specialised (one 8-wave workgroup per CU); MIA_FECONV_WS=0 selects the two-workgroup form for A/B runs
    if (fe_ws()) {
      const int grid = fe_grid1(nc * a.nitem);
      if (scale) feconv_ws_kernel<32, 16, 2, true><<<grid, FS_NT, 0, s>>>(a);
      else feconv_ws_kernel<32, 16, 2, false><<<grid, FS_NT, 0, s>>>(a);
    } else {
      const int grid = fe_grid(nc * a.nitem);
      if (scale) feconv_kernel<32, 16, 2, true><<<grid, FE_NT, 0, s>>>(a);
      else feconv_kernel<32, 16, 2, false><<<grid, FE_NT, 0, s>>>(a);
    }
    MIA_LAUNCH_CHECK("fe_conv2_fwd");
  }
  return 0;
}

extern "C" int mia_fe_conv2_dgrad(const void* dy2, const void* wpar, void* da1, int32_t n, int32_t w1,
                                  int32_t w2, mia_stream_t stream) {
  MIA_CHECK_ARG(dy2 && wpar && da1 && n > 0 && w1 >= 16, "fe_conv2_dgrad: bad arguments");
  MIA_CHECK_ARG(w2 == (w1 - 16) / 2 + 1, "fe_conv2_dgrad: w2 must be (w1-16)/2+1 (got w1=%d w2=%d)", w1, w2);
  MIA_CHECK_ARG(aligned16(dy2) && aligned16(wpar) && aligned16(da1), "fe_conv2_dgrad: operands must be 16-byte aligned");
  MIA_CHECK_ARG(((int64_t)w1 * 32) % 8 == 0, "fe_conv2_dgrad: clip stride must keep 16-byte alignment");
  const int wout = (w1 + 1) / 2;  // parity pairs (2m, 2m+1)
  const int per = fe_clips_per_launch((int64_t)w2 * 64 * 2);
  MIA_CHECK_ARG(per > 0, "fe_conv2_dgrad: one clip exceeds 2 GB");
  for (int c = 0; c < n; c += per) {
    const int nc = n - c < per ? n - c : per;
    FeArgs a{reinterpret_cast<const bf16*>(dy2) + (int64_t)c * w2 * 64, nullptr, nullptr,
             reinterpret_cast<const bf16*>(wpar), nullptr, reinterpret_cast<bf16*>(da1) + (int64_t)c * w1 * 32, nc,
             w2, wout, 7, (int)cdiv(wout, FE_BM), (int64_t)w1 * 32, (int64_t)w1 * 32};
    // (the warp-specialised form measured no faster here: its stream side alone takes 0.77 ms, DESIGN round 6)
#ifdef FS_DGRAD  // A/B builds only
    feconv_ws_kernel<64, 8, 1, false><<<fe_grid1(nc * a.nitem), FS_NT, 0, as_stream(stream)>>>(a);
#else
    feconv_kernel<64, 8, 1, false><<<fe_grid(nc * a.nitem), FE_NT, 0, as_stream(stream)>>>(a);
#endif
    MIA_LAUNCH_CHECK("fe_conv2_dgrad");
  }
  return 0;
}

extern "C" int mia_fe_conv2_wgrad(const void* dy2, const void* y1, const float* scale, const float* shift,
                                  float* dw, int32_t n, int32_t w1, int32_t w2, void* workspace, int64_t ws_bytes,
                                  mia_stream_t stream) {
  MIA_CHECK_ARG(dy2 && y1 && dw && workspace && n > 0 && w1 >= 16, "fe_conv2_wgrad: bad arguments");
  MIA_CHECK_ARG(!scale == !shift, "fe_conv2_wgrad: scale and shift go together");
  MIA_CHECK_ARG(w2 == (w1 - 16) / 2 + 1, "fe_conv2_wgrad: w2 must be (w1-16)/2+1 (got w1=%d w2=%d)", w1, w2);
  MIA_CHECK_ARG(aligned16(dy2) && aligned16(y1), "fe_conv2_wgrad: operands must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int per = fe_clips_per_launch((int64_t)w1 * 32 * 2);
  MIA_CHECK_ARG(per > 0, "fe_conv2_wgrad: one clip exceeds 2 GB");
  const int nitem = (int)cdiv(w2, FW_BP);
  // one slab per workgroup of every launch, summed by one reduce at the end
  int slabs = 0;
  for (int c = 0; c < n; c += per) slabs += fe_grid1(((n - c) < per ? (n - c) : per) * nitem);
  MIA_CHECK_ARG((int64_t)slabs * 64 * 512 * 4 <= ws_bytes, "fe_conv2_wgrad: workspace too small (%lld B needed)",
                (long long)slabs * 64 * 512 * 4);
  int slab0 = 0;
  for (int c = 0; c < n; c += per) {
    const int nc = n - c < per ? n - c : per;
    FwArgs a{reinterpret_cast<const bf16*>(dy2) + (int64_t)c * w2 * 64, reinterpret_cast<const bf16*>(y1) + (int64_t)c * w1 * 32,
             scale, shift, nc, w1, w2, nitem, reinterpret_cast<float*>(workspace) + (int64_t)slab0 * 64 * 512};
    const int grid = fe_grid1(nc * nitem);
    if (scale) fe_wgrad_kernel<true><<<grid, FW_NT, 0, s>>>(a);
    else fe_wgrad_kernel<false><<<grid, FW_NT, 0, s>>>(a);
    MIA_LAUNCH_CHECK("fe_conv2_wgrad");
    slab0 += grid;
  }
  fw_reduce_kernel<<<64 * 512 / 256, 256, 0, s>>>(reinterpret_cast<const float*>(workspace), slabs, 64 * 512, dw);
  MIA_LAUNCH_CHECK("fe_conv2_wgrad reduce");
  return 0;
}

extern "C" int mia_fe_conv1_fwd(const float* x, const void* w, const float* bias, void* y1, float* partial,
                                int32_t nwaves, int32_t n, int32_t t, mia_stream_t stream) {
  MIA_CHECK_ARG(x && w && bias && y1 && n > 0 && t >= 64 && t % 2 == 0, "fe_conv1_fwd: bad arguments");
  MIA_CHECK_ARG(nwaves > 0 && nwaves % 4 == 0, "fe_conv1_fwd: nwaves must be a positive multiple of 4");
  MIA_CHECK_ARG(aligned16(w) && aligned16(y1) && (reinterpret_cast<uintptr_t>(x) & 7) == 0,
                "fe_conv1_fwd: y1/w must be 16-byte and x 8-byte aligned");
  const int w1 = (t - 64) / 2 + 1;
  F1Args a{x, reinterpret_cast<const bf16*>(w), bias, reinterpret_cast<bf16*>(y1), partial, n, t, w1,
           (int)cdiv(w1, 32)};
  MIA_CHECK_ARG((int64_t)n * a.nitem < (1ll << 31), "fe_conv1_fwd: too many items");
  if (partial) fe_conv1_kernel<true><<<nwaves / 4, 256, 0, as_stream(stream)>>>(a);
  else fe_conv1_kernel<false><<<nwaves / 4, 256, 0, as_stream(stream)>>>(a);
  MIA_LAUNCH_CHECK("fe_conv1_fwd");
  return 0;
}

extern "C" int mia_fe_conv3_fwd(const void* x, const void* w, const float* bias, void* y, float* partial,
                                int32_t nwaves, int32_t n, int32_t h, int32_t wd, mia_stream_t stream) {
  MIA_CHECK_ARG(x && w && bias && y && n > 0 && h >= 8 && wd >= 8, "fe_conv3_fwd: bad arguments");
  MIA_CHECK_ARG(nwaves > 0 && nwaves % 4 == 0, "fe_conv3_fwd: nwaves must be a positive multiple of 4");
  MIA_CHECK_ARG(wd % 4 == 0, "fe_conv3_fwd: image width must be a multiple of 4 (8-byte row alignment)");
  MIA_CHECK_ARG(aligned16(w) && aligned16(y) && (reinterpret_cast<uintptr_t>(x) & 7) == 0,
                "fe_conv3_fwd: w/y must be 16-byte and x 8-byte aligned");
  F3Args a{reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(w), bias, reinterpret_cast<bf16*>(y),
           partial, n, h, wd, h - 7, wd - 7, (int)cdiv(wd - 7, 32)};
  MIA_CHECK_ARG((int64_t)n * a.oh * a.nseg < (1ll << 31), "fe_conv3_fwd: too many items");
  if (partial) fe_conv3_kernel<true><<<nwaves / 4, 256, 0, as_stream(stream)>>>(a);
  else fe_conv3_kernel<false><<<nwaves / 4, 256, 0, as_stream(stream)>>>(a);
  MIA_LAUNCH_CHECK("fe_conv3_fwd");
  return 0;
}

#ifdef FE_STAMP
extern "C" int mia_fe_stamps_copy(void* dst, int64_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fe_st), (size_t)bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
