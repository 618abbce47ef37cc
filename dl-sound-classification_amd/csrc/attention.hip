// Fused multi-head attention, head_dim 64, bf16 MFMA (v_mfma_f32_32x32x16_bf16), gfx950.
// timm Attention with F.scaled_dot_product_attention (reference src/models/ast.py:38,60-61).
//
// Layouts: qkv (B, N, 3, H, 64) bf16 = the qkv Linear output as is; out / dout (B, N, H, 64) bf16
// (= the proj Linear input); lse (B, H, N) f32 in natural-log units of the scaled scores.
//
// Forward (q on the lane): each wave owns 32 queries; per 64-key tile staged in LDS it computes
// S^T = K . Q^T (accumulator column = query = lane, 16 keys per lane in registers), so the online
// softmax row max / sum are in-lane plus one lane^32 exchange; P^T is fed straight from the
// accumulator registers as the B operand of O^T += V^T . P^T (V^T fragments by ds_read_b64_tr_b16),
// so the rescale of O by exp(m_old - m_new) is per lane too.
// Backward (deterministic, no atomics): a key-parallel kernel computes S and dP with the key on the
// lane and accumulates dV^T, dK^T in registers while sweeping the query tiles; a query-parallel
// kernel recomputes S^T, dP^T with the query on the lane and accumulates dQ^T.
#include "common.h"

#include <type_traits>

#include "attn_common.h"

namespace {

// S^T - m for one 64-key tile: [key half] accumulators (rows = keys, lane column = query)
__device__ __forceinline__ void fwd_qk(f32x16 (&s)[2], const bf16* K_, const bf16x8 (&qf)[4], bf16x8 one,
                                       bf16x8 mrow, int lane) {
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    s[kh] = mfma(frag_row_sw(K_, 32 * kh + (lane & 31), 0, lane), qf[0], zero16());
#pragma unroll
    for (int ks = 1; ks < 4; ++ks) s[kh] = mfma(frag_row_sw(K_, 32 * kh + (lane & 31), ks, lane), qf[ks], s[kh]);
    s[kh] = mfma(one, mrow, s[kh]);
  }
}

struct FwdAcc {
  f32x16 o[2];  // O^T [d half]: rows = d, lane column = query
  float l;      // this lane's half of the row sum
  float mb;     // running max (log2 units, bf16-exact)
  bf16x8 mrow;  // fifth-k-step fragment: element 0 of the low lane half = -mb
};

// p = exp2(s - d) -> bf16 P^T fragments, row-sum partials
__device__ __forceinline__ void fwd_exp(const f32x16 (&s)[2], float d, bf16x8 (&pf)[4], float& la, float& lb) {
  la = 0.f; lb = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float p = __builtin_amdgcn_exp2f(s[c >> 1][8 * (c & 1) + j] - d);
      if (c & 1) lb += p; else la += p;
      pf[c][j] = (bf16)p;
    }
  }
}

// kvalid = keys of the tile inside the sequence (>= 64: all): a wave-uniform mask that only the peeled first
// tile (the sequence's last key tile: the kernel walks the keys backwards) passes at run time; the loop's
// tiles pass 64, so no mask instruction is emitted there (as a run-time mask on every tile the compiler
// if-converted it into 32 compares + 32 selects per tile)
template <bool FIRST>
__device__ __forceinline__ void fwd_softmax(f32x16 (&s)[2], FwdAcc& a, bf16x8 (&pf)[4], int kvalid, int lane) {
  if (kvalid < 64) {
    const int lim = kvalid - 4 * (lane >> 5);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2);
      if (row >= lim) s[0][r] = -INFINITY;
      if (row + 32 >= lim) s[1][r] = -INFINITY;
    }
  }
  float la, lb;
  if (!FIRST) fwd_exp(s, 0.f, pf, la, lb);
  if (FIRST || __builtin_expect(__any(la + lb > FWD_SUM_LIMIT), 0)) {
    // rare path: move m to (at least) this tile's max, rounded up to bf16
    float mx = fmaxf(s[0][0], s[1][0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));
    mx = half_exchange_max(mx);
    const float mn = FIRST ? bf16_ceil(mx) : fmaxf(a.mb, bf16_ceil(a.mb + mx));
    const float d = mn - a.mb;
    if (!FIRST) {
      const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
      for (int r = 0; r < 16; ++r) { a.o[0][r] *= alpha; a.o[1][r] *= alpha; }
      a.l *= alpha;
    }
    fwd_exp(s, d, pf, la, lb);
    a.mb = mn;
    a.mrow[0] = (lane < 32) ? (bf16)(-mn) : (bf16)0.f;
  }
  a.l += la + lb;
}

__device__ __forceinline__ void fwd_pv(FwdAcc& a, const bf16* V_, const bf16x8 (&pf)[4], int lane) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) a.o[dh] = mfma(frag_tr_sw(V_, 16 * c, 32 * dh, lane), pf[c], a.o[dh]);
  }
}

// MX (fp8-mixed): the bf16 output is also written as OCP MX-fp8 (e4m3 q8 [B*N][H*64], E8M0 s8
// [B*N][H*2]) -- the proj MX GEMM's A operand.  Lanes l and l ^ 32 hold the 32 d of one block of one
// query (16 each), so a block's amax is one lane-pair exchange.
template <bool MX>
__global__ __launch_bounds__(256, 3) void attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                          float* __restrict__ lse, int N, int H, int nqb,
                                                          float scale_log2, uint8_t* __restrict__ q8,
                                                          uint8_t* __restrict__ s8, bf16* __restrict__ qs_out) {
  __shared__ __attribute__((aligned(1024))) bf16 Ks[3][64 * 64];
  __shared__ __attribute__((aligned(1024))) bf16 Vs[3][64 * 64];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int w = xcd_work_item(blockIdx.x, gridDim.x);
  const int bh = w / nqb, qb = w - bh * nqb, b = bh / H, hd = bh % H;
  const int64_t ldt = (int64_t)3 * H * D;
  const bf16* base = qkv + (int64_t)b * N * ldt + hd * D;
  const int ntiles = (N + 63) / 64;
  const unsigned tile_bytes = (unsigned)(64 * ldt * 2);
  TileDMA kdma, vdma;
  kdma.init(base + H * D, ldt, N, wave, lane);
  vdma.init(base + 2 * H * D, ldt, N, wave, lane);
  // key tiles in reverse order: the sequence's partial last tile is the peeled first tile (FIRST), so the
  // key mask exists only there and the loop's tiles carry no mask instructions
  kdma.issue(Ks[0], (unsigned)(ntiles - 1) * tile_bytes, wave);
  vdma.issue(Vs[0], (unsigned)(ntiles - 1) * tile_bytes, wave);
  // a wave past the last query computes on zero queries (finite, never stored): no branch in the loop
  const int q = qb * FWD_Q + wave * 32 + (lane & 31);
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8 r = load_frag_global(base + (int64_t)q * ldt, ks, lane, q < N);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[ks][j] = (bf16)((float)r[j] * scale_log2);
  }
  settle(qf);
  if (qs_out != nullptr && q < N) {  // Q' for the backward (its prep then skips it): row (b, q, h), d = 16 ks + 8 (lane >> 5)..
    bf16* qrow = qs_out + (((int64_t)b * N + q) * H + hd) * D + 8 * (lane >> 5);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) *reinterpret_cast<bf16x8*>(qrow + 16 * ks) = qf[ks];
  }
  if (ntiles > 1) {
    kdma.issue(Ks[1], (unsigned)(ntiles - 2) * tile_bytes, wave);
    vdma.issue(Vs[1], (unsigned)(ntiles - 2) * tile_bytes, wave);
  }
  bf16x8 one;
#pragma unroll
  for (int j = 0; j < 8; ++j) one[j] = (bf16)0.f;
  one[0] = (lane < 32) ? (bf16)1.f : (bf16)0.f;
  FwdAcc a;
  a.o[0] = zero16(); a.o[1] = zero16();
  a.l = 0.f; a.mb = 0.f;
  a.mrow = one;
  a.mrow[0] = (bf16)0.f;
  f32x16 s[2];
  bf16x8 pf[4];
  // one tile in slot P of the 3-slot ring: tile j + 2's DMA flies under this tile's work and tile j + 1's
  auto tile = [&](auto first, auto, auto slot, int j) __attribute__((always_inline)) {
    constexpr int P = decltype(slot)::value;
    constexpr int PN = (P + 2) % 3;
    const bool ahead = j + 2 < ntiles;
    const int kt = ntiles - 1 - j;  // key tile
    if (ahead) {
      kdma.issue(Ks[PN], (unsigned)(kt - 2) * tile_bytes, wave);
      vdma.issue(Vs[PN], (unsigned)(kt - 2) * tile_bytes, wave);
    }
    fwd_qk(s, Ks[P], qf, one, a.mrow, lane);
    __builtin_amdgcn_s_setprio(1);  // the softmax's VALU issues ahead of the co-resident waves' MFMA streams
    fwd_softmax<decltype(first)::value>(s, a, pf, decltype(first)::value ? N - kt * 64 : 64, lane);
    __builtin_amdgcn_s_setprio(0);
    fwd_pv(a, Vs[P], pf, lane);
    if (ahead) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile j + 1's pieces have landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  using T = std::true_type;
  using F = std::false_type;
  using P0 = std::integral_constant<int, 0>;
  if (ntiles > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 and the Q fragments
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  tile(T{}, F{}, P0{}, 0);
  ring3_guarded<1>(1, ntiles, [&](auto tl, auto sl, int j) __attribute__((always_inline)) { tile(F{}, tl, sl, j); });
  const float lt = half_exchange_sum(a.l);
  const float inv = 1.f / lt;
  if constexpr (MX) {
    // every lane takes part in the pair exchange; queries past the end store nothing
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      float v[16], am = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) { v[r] = (float)(bf16)(a.o[dh][r] * inv); am = fmaxf(am, fabsf(v[r])); }
      am = fmaxf(am, __shfl_xor(am, 32, 64));
      const int e = mx_exponent(am);
      if (q < N) {
        uint8_t* qrow = q8 + ((int64_t)b * N + q) * H * D + hd * D + 32 * dh;
#pragma unroll
        for (int g2 = 0; g2 < 2; ++g2) {  // registers 8 g2 .. 8 g2 + 7 = d runs 16 g2 + {0..3, 8..11} (+4 high lanes)
          const uint2 p = mx_pack8(v + 8 * g2, e);
          *reinterpret_cast<uint32_t*>(qrow + 16 * g2 + 4 * (lane >> 5)) = p.x;
          *reinterpret_cast<uint32_t*>(qrow + 16 * g2 + 8 + 4 * (lane >> 5)) = p.y;
        }
        if (lane < 32) s8[((int64_t)b * N + q) * H * 2 + hd * 2 + dh] = (uint8_t)(e + 127);
      }
    }
  }
  if (q < N) {
    bf16* orow = out + ((int64_t)b * N + q) * H * D + hd * D;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {  // registers 4g4..4g4+3 = 4 consecutive d
      const int d0 = 8 * g4 + 4 * (lane >> 5);
      bf16x4 v0, v1;
#pragma unroll
      for (int i = 0; i < 4; ++i) { v0[i] = (bf16)(a.o[0][4 * g4 + i] * inv); v1[i] = (bf16)(a.o[1][4 * g4 + i] * inv); }
      *reinterpret_cast<bf16x4*>(orow + d0) = v0;
      *reinterpret_cast<bf16x4*>(orow + 32 + d0) = v1;
    }
    if (lane < 32) lse[(int64_t)bh * N + q] = (a.mb + log2f(lt)) / LOG2E;
  }
}
template __global__ void attn_fwd_kernel<false>(const bf16*, bf16*, float*, int, int, int, float, uint8_t*, uint8_t*,
                                                bf16*);
template __global__ void attn_fwd_kernel<true>(const bf16*, bf16*, float*, int, int, int, float, uint8_t*, uint8_t*,
                                               bf16*);


// Key-parallel dK / dV.  One wave = 32 keys (key on the lane), 4 waves = 128 keys per block; the
// block sweeps 64-query tiles of Q', dO and their fragment rows (LDS-DMA, double-buffered).  With
// the key on the lane the S / dP accumulators are query rows x key columns and are used as the B
// operands of dV^T += dO^T P and dK^T += Q'^T dS directly (no LDS round trip); dK, dV accumulate in
// registers over the whole sequence: no atomics, deterministic.
constexpr int BWD_K = 128;

// qvalid = queries of the tile inside the sequence (>= 64: all): a wave-uniform mask that only the peeled first
// tile (the last query tile: the kernel walks the queries backwards) passes at run time
__device__ __forceinline__ void dkdv_tile(f32x16 (&dk)[2], f32x16 (&dv)[2], const bf16* Q_, const bf16* G_,
                                          const bf16* F_, const bf16x8 (&kf)[4], const bf16x8 (&vf)[4], bf16x8 one,
                                          int qvalid, int lane) {
  // the row fragments of query half sq (Q', dO, the two fifth-k-step rows), loaded one half ahead: half 1's
  // fly under half 0's softmax and dV / dK products instead of one LDS latency in front of every MFMA
  bf16x8 fr[2][10];
  auto load = [&](int sq, bf16x8 (&f)[10]) __attribute__((always_inline)) {
    const int qr = sq * 32 + (lane & 31);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f[ks] = frag_row_sw(Q_, qr, ks, lane);
      f[4 + ks] = frag_row_sw(G_, qr, ks, lane);
    }
    f[8] = row_frag(F_ + qr * 8);
    f[9] = row_frag(F_ + 512 + qr * 8);
  };
  load(0, fr[0]);
  // S / dP of both query halves first: half 1's ten MFMAs issue before half 0's exp / dS VALU, so that VALU
  // runs under them instead of in front of half 0's dV / dK products
  f32x16 scs[2], dps[2];
#pragma unroll
  for (int sq = 0; sq < 2; ++sq) {
    const bf16x8 (&f)[10] = fr[sq];
    f32x16 sc = mfma(f[0], kf[0], zero16());
    f32x16 dp = mfma(f[4], vf[0], zero16());
#pragma unroll
    for (int ks = 1; ks < 4; ++ks) {
      sc = mfma(f[ks], kf[ks], sc);
      dp = mfma(f[4 + ks], vf[ks], dp);
    }
    scs[sq] = mfma(f[8], one, sc);
    dps[sq] = mfma(f[9], one, dp);
    if (sq == 0) load(1, fr[1]);
  }
#pragma unroll
  for (int sq = 0; sq < 2; ++sq) {
    f32x16 sc = scs[sq], dp = dps[sq];
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = __builtin_amdgcn_exp2f(sc[r]);
    if (qvalid < 64) {  // the sequence's last, partial query tile: rows past it contribute nothing
      const int lim = qvalid - sq * 32 - 4 * (lane >> 5);
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = ((r & 3) + 8 * (r >> 2)) < lim ? sc[r] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] *= sc[r];
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      const bf16x8 pf = acc_frag(sc, sk), df = acc_frag(dp, sk);
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        dv[dh] = mfma(frag_tr_sw(G_, sq * 32 + 16 * sk, 32 * dh, lane), pf, dv[dh]);
        dk[dh] = mfma(frag_tr_sw(Q_, sq * 32 + 16 * sk, 32 * dh, lane), df, dk[dh]);
      }
    }
  }
}

__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                               const bf16* __restrict__ qs, const bf16* __restrict__ frag,
                                                               bf16* __restrict__ dqkv, int N, int H, int nkb,
                                                               float dk_scale) {
  __shared__ __attribute__((aligned(1024))) bf16 Qs[2][64 * 64];
  __shared__ __attribute__((aligned(1024))) bf16 Gs[2][64 * 64];
  __shared__ __attribute__((aligned(1024))) bf16 Fs[2][64 * 16];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int w = xcd_work_item(blockIdx.x, gridDim.x);
  const int bh = w / nkb, kb = w - bh * nkb, b = bh / H, hd = bh % H;
  const int64_t ldt = (int64_t)3 * H * D, ldo = (int64_t)H * D;
  const bf16* base = qkv + (int64_t)b * N * ldt + hd * D;
  const int ntiles = (N + 63) / 64;
  const unsigned tile_bytes = (unsigned)(64 * ldo * 2);
  TileDMA qd, gd;
  FragDMA fd;
  qd.init(qs + (int64_t)b * N * ldo + hd * D, ldo, N, wave, lane);
  gd.init(dout + (int64_t)b * N * ldo + hd * D, ldo, N, wave, lane);
  fd.init(frag + (int64_t)bh * 2 * N * 8, N);
  // query tiles in reverse order: the partial last query tile is the peeled first tile, the only one that
  // carries the query mask
  qd.issue(Qs[0], (unsigned)(ntiles - 1) * tile_bytes, wave);
  gd.issue(Gs[0], (unsigned)(ntiles - 1) * tile_bytes, wave);
  fd.issue(Fs[0], (unsigned)(ntiles - 1) * 64u, wave, lane);
  const int key = kb * BWD_K + wave * 32 + (lane & 31);
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = load_frag_global(base + (int64_t)key * ldt + H * D, ks, lane, key < N);
    vf[ks] = load_frag_global(base + (int64_t)key * ldt + 2 * H * D, ks, lane, key < N);
  }
  settle(kf);
  settle(vf);
  const bf16x8 one = ones3(lane);
  f32x16 dk[2], dv[2];
  dk[0] = zero16(); dk[1] = zero16(); dv[0] = zero16(); dv[1] = zero16();
  auto tile = [&](auto first, auto par, int j) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    const int qt = ntiles - 1 - j;  // query tile
    if (j + 1 < ntiles) {
      qd.issue(Qs[P ^ 1], (unsigned)(qt - 1) * tile_bytes, wave);
      gd.issue(Gs[P ^ 1], (unsigned)(qt - 1) * tile_bytes, wave);
      fd.issue(Fs[P ^ 1], (unsigned)(qt - 1) * 64u, wave, lane);
    }
    dkdv_tile(dk, dv, Qs[P], Gs[P], Fs[P], kf, vf, one, decltype(first)::value ? N - qt * 64 : 64, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  using T = std::true_type;
  using F = std::false_type;
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  tile(T{}, P0{}, 0);
  for (int j = 1; j < ntiles; j += 2) {  // no remainder code (see ring3_guarded)
    tile(F{}, P1{}, j);
    if (j + 1 < ntiles) tile(F{}, P0{}, j + 1);
  }
  if (key >= N) return;
  bf16* krow = dqkv + ((int64_t)b * N + key) * ldt + H * D + hd * D;
  bf16* vrow = krow + H * D;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int d0 = 8 * g4 + 4 * (lane >> 5);
    bf16x4 a0, a1, c0, c1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a0[i] = (bf16)(dk[0][4 * g4 + i] * dk_scale);
      a1[i] = (bf16)(dk[1][4 * g4 + i] * dk_scale);
      c0[i] = (bf16)dv[0][4 * g4 + i];
      c1[i] = (bf16)dv[1][4 * g4 + i];
    }
    *reinterpret_cast<bf16x4*>(krow + d0) = a0;
    *reinterpret_cast<bf16x4*>(krow + 32 + d0) = a1;
    *reinterpret_cast<bf16x4*>(vrow + d0) = c0;
    *reinterpret_cast<bf16x4*>(vrow + 32 + d0) = c1;
  }
}

// Query-parallel dQ.  One wave = 32 queries (query on the lane), 4 waves = 128 per block, sweeping
// 64-key tiles of K and V (LDS-DMA, 3-slot ring): S'^T = K Q'^T - L2, dP'^T = V dO^T - delta with the
// row constants as per-lane f32 adds (the accumulator column is the lane's query), dQ^T += K^T dS^T
// with dS^T straight from the accumulators.
constexpr int BWD_Q = 128;

// kvalid = keys of the tile inside the sequence (>= 64: all): a wave-uniform mask that only the peeled first
// tile (the last key tile: the kernel walks the keys backwards) passes at run time; the loop passes 64
__device__ __forceinline__ void dq_tile(f32x16 (&acc)[2], const bf16* K_, const bf16* V_, const bf16x8 (&qf)[4],
                                        const bf16x8 (&gf)[4], float nl, float nd, int kvalid, int lane) {
  // S / dP of both key halves first: half 1's MFMAs issue before half 0's exp / dS VALU (as dkdv_tile)
  f32x16 scs[2], dps[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const int kr = 32 * kh + (lane & 31);
    f32x16 sc = mfma(frag_row_sw(K_, kr, 0, lane), qf[0], zero16());
    f32x16 dp = mfma(frag_row_sw(V_, kr, 0, lane), gf[0], zero16());
#pragma unroll
    for (int ks = 1; ks < 4; ++ks) {
      sc = mfma(frag_row_sw(K_, kr, ks, lane), qf[ks], sc);
      dp = mfma(frag_row_sw(V_, kr, ks, lane), gf[ks], dp);
    }
    scs[kh] = sc;
    dps[kh] = dp;
  }
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    f32x16 sc = scs[kh], dp = dps[kh];
    // the lane's column is one query: its row constants are two per-lane scalars (VALU adds beside the
    // other waves' MFMAs instead of two fifth-k-step MFMAs per key half)
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = __builtin_amdgcn_exp2f(sc[r] + nl);
    if (kvalid < 64) {
      const int lim = kvalid - 32 * kh - 4 * (lane >> 5);
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = ((r & 3) + 8 * (r >> 2)) < lim ? sc[r] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = (dp[r] + nd) * sc[r];
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      const bf16x8 dsf = acc_frag(dp, sk);
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) acc[dh] = mfma(frag_tr_sw(K_, 32 * kh + 16 * sk, 32 * dh, lane), dsf, acc[dh]);
    }
  }
}

__global__ __launch_bounds__(256, 3) void attn_bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ out,
                                                             const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                             bf16* __restrict__ frag, bf16* __restrict__ dqkv,
                                                             int N, int H, int nqb, float scale, float scale_log2) {
  __shared__ __attribute__((aligned(1024))) bf16 Ks[3][64 * 64];
  __shared__ __attribute__((aligned(1024))) bf16 Vs[3][64 * 64];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int w = xcd_work_item(blockIdx.x, gridDim.x);
  const int bh = w / nqb, qb = w - bh * nqb, b = bh / H, hd = bh % H;
  const int64_t ldt = (int64_t)3 * H * D, ldo = (int64_t)H * D;
  const bf16* base = qkv + (int64_t)b * N * ldt + hd * D;
  const int ntiles = (N + 63) / 64;
  const unsigned tile_bytes = (unsigned)(64 * ldt * 2);
  TileDMA kd, vd;
  kd.init(base + H * D, ldt, N, wave, lane);
  vd.init(base + 2 * H * D, ldt, N, wave, lane);
  // key tiles in reverse order (as the forward): only the peeled first tile can be partial
  kd.issue(Ks[0], (unsigned)(ntiles - 1) * tile_bytes, wave);
  vd.issue(Vs[0], (unsigned)(ntiles - 1) * tile_bytes, wave);
  const int q = qb * BWD_Q + wave * 32 + (lane & 31);
  const bool qv = q < N;
  bf16x8 qf[4], gf[4];
  float dsum = 0.f;  // this lane's half of delta = sum_d dO * O
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8 r = load_frag_global(base + (int64_t)q * ldt, ks, lane, qv);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[ks][j] = (bf16)((float)r[j] * scale_log2);
    gf[ks] = load_frag_global(dout + ((int64_t)b * N + q) * ldo + hd * D, ks, lane, qv);
    const bf16x8 o = load_frag_global(out + ((int64_t)b * N + q) * ldo + hd * D, ks, lane, qv);
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum = fmaf((float)o[j], (float)gf[ks][j], dsum);
  }
  // this lane's query's row constants -L2 = -lse log2 e and -delta in f32 (the prep pass's job, done here:
  // this kernel runs before dK/dV and leaves their fragment rows, three bf16 parts each, for it);
  // zero for a query past the end (p = 1, dS = 0)
  float nl = 0.f, nd = 0.f;
  {
    dsum += __shfl_xor(dsum, 32, 64);
    if (qv) {
      nl = -lse[(int64_t)bh * N + q] * LOG2E;
      nd = -dsum;
      if (lane < 32) {
        bf16x8 f0, f1;
#pragma unroll
        for (int j = 0; j < 8; ++j) { f0[j] = (bf16)0.f; f1[j] = (bf16)0.f; }
        split3(nl, f0);
        split3(nd, f1);
        *reinterpret_cast<bf16x8*>(frag + ((int64_t)bh * 2 * N + q) * 8) = f0;
        *reinterpret_cast<bf16x8*>(frag + ((int64_t)(bh * 2 + 1) * N + q) * 8) = f1;
      }
    }
  }
  settle(qf);
  settle(gf);
  asm volatile("" ::"v"(nl), "v"(nd));
  if (ntiles > 1) {
    kd.issue(Ks[1], (unsigned)(ntiles - 2) * tile_bytes, wave);
    vd.issue(Vs[1], (unsigned)(ntiles - 2) * tile_bytes, wave);
  }
  f32x16 acc[2];
  acc[0] = zero16(); acc[1] = zero16();
  // one tile in slot P of the 3-slot ring: tile j + 2's DMA flies under this tile's work and tile j + 1's
  auto tile = [&](auto first, auto slot, int j) __attribute__((always_inline)) {
    constexpr int P = decltype(slot)::value;
    constexpr int PN = (P + 2) % 3;
    const bool ahead = j + 2 < ntiles;
    const int kt = ntiles - 1 - j;  // key tile
    if (ahead) {
      kd.issue(Ks[PN], (unsigned)(kt - 2) * tile_bytes, wave);
      vd.issue(Vs[PN], (unsigned)(kt - 2) * tile_bytes, wave);
    }
    dq_tile(acc, Ks[P], Vs[P], qf, gf, nl, nd, decltype(first)::value ? N - kt * 64 : 64, lane);
    if (ahead) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  if (ntiles > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 and the Q / dO fragments
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  tile(std::true_type{}, std::integral_constant<int, 0>{}, 0);
  ring3_guarded<1>(1, ntiles, tile);
  if (!qv) return;
  bf16* qrow = dqkv + ((int64_t)b * N + q) * ldt + hd * D;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int d0 = 8 * g4 + 4 * (lane >> 5);
    bf16x4 v0, v1;
#pragma unroll
    for (int i = 0; i < 4; ++i) { v0[i] = (bf16)(acc[0][4 * g4 + i] * scale); v1[i] = (bf16)(acc[1][4 * g4 + i] * scale); }
    *reinterpret_cast<bf16x4*>(qrow + d0) = v0;
    *reinterpret_cast<bf16x4*>(qrow + 32 + d0) = v1;
  }
}

// ------------------------------------------------------------------------------ fused backward
// One pass per (b, h, 256-key block) computes S, dP and dS ONCE and all three products from them:
// dV^T += dO^T P and dK^T += Q'^T dS in registers (key on the lane, as the key-parallel kernel above),
// and the block's share of dQ = dS K (dS^T staged in LDS, K^T read from an LDS image of the block's keys):
// five MFMA products per tile instead of the seven of the two-kernel form (whose query-parallel kernel
// recomputes S and dP with the query on the lane).
//
// dQ sums over the key blocks of one (b, h).  No float atomics (the sum would depend on arrival order):
// an ORDERED HAND-OFF.  Key block kb walks the query tiles rotated by FB_LAG * kb (tile T at step
// (T + FB_LAG kb) mod nt), and the blocks add their partial of tile T in the fixed order of the steps at
// which they reach it: a running f32 sum in the workspace, the last block of the order writing bf16 dQ.
// The tile's dQ^T is four 32 x 32 sub-tiles; waves 0-3 each own one (the partial of waves 4-7 -- the other
// key half -- reaches them through LDS behind a per-wave LDS flag) and hand it off on their own: every
// byte of the running sum is stored and loaded `sc1` (16 B per lane, to registers), the storing wave waits
// vmcnt(0) before its `sc1` flag store, the consuming wave polls that flag with `sc1` loads before it loads
// (MI355X_MICROARCH.md, visibility table row 1 with one storing wave per flag; Guideline 16 R1).  So a step
// has ONE workgroup barrier (dS^T complete; dS^T is double-buffered).  Within a step a wave publishes its
// previous sum before the barrier and polls for its next tile after it, so with a lag of >= 2 steps between
// consecutive contributions a block only ever waits for an event earlier in (step, phase) order: a chain
// cannot wait on itself.  The spin is bounded anyway (FB_SPIN_TICKS of the 100 MHz real-time counter) and a
// timeout is recorded in the workspace's error word (mia_attn_bwd_error_offset) instead of hanging the GPU.
// Bit-reproducible: the order is a fixed function of (kb, T, N).
constexpr int FB_K = 256;        // keys per workgroup: 8 waves x 32
constexpr int FB_LAG = 3;        // rotation lag between consecutive key blocks of one (b, h)
constexpr int FB_SUB = 4096;     // bytes of one 32 x 32 f32 dQ^T sub-tile in register order
constexpr int FB_TILE = 4 * FB_SUB;
constexpr int FB_OP = 80;        // bytes per query row of a wave's staged bf16 dQ sub-tile (32 d + pad)
constexpr unsigned long long FB_SPIN_TICKS = 20000000ull;  // 200 ms at 100 MHz

// LDS map (one __shared__ array)
constexpr int FBL_Q = 0;                        // [2][64][64] bf16 Q' tiles (sw_off)
constexpr int FBL_G = FBL_Q + 2 * 8192;         // [2][64][64] bf16 dO tiles (sw_off)
constexpr int FBL_F = FBL_G + 2 * 8192;         // [2][2][64][8] bf16 fifth-k-step rows
constexpr int FBL_K = FBL_F + 2 * 2048;         // [256][64] bf16 the block's keys (sw_off)
constexpr int FBL_S = FBL_K + 32768;            // [2][256][64] bf16 dS^T (sw_off), double-buffered
constexpr int FBL_R = FBL_S + 2 * 32768;        // [4][4096 B] key-half partials; reused as staged bf16 dQ
constexpr int FBL_FL = FBL_R + 4 * FB_SUB;      // [4] int LDS flags: partial of step j ready (j + 1)
constexpr int FBL_BYTES = FBL_FL + 64;

// wave-uniform: poll `flag` until it reads `want` (bounded; a timeout sets the error word, and once it is
// set every later wait of the launch gives up at once, so a broken chain still drains the grid quickly)
__device__ __forceinline__ void fb_wait(const unsigned* flag, unsigned want, unsigned* err) {
  if (fb_ld_flag(flag) == want) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    __builtin_amdgcn_s_sleep(4);
    if (fb_ld_flag(flag) == want) return;
    if (fb_ld_flag(err) != 0u) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > FB_SPIN_TICKS) {
      fb_st_flag(err, 1u);
      return;
    }
  }
}

// the tile key block kb processes at step j, and its position in tile T's chain of contributions
__device__ __forceinline__ int fb_tile(int j, int kb, int nt) {
  const int t = j - FB_LAG * kb;
  return t < 0 ? t + nt : t;
}
__device__ __forceinline__ int fb_pos(int kb, int T, int nkb, int nt) {
  auto step = [&](int k) { const int s = T + FB_LAG * k; return s >= nt ? s - nt : s; };
  const int mine = step(kb);
  int p = 0;
  for (int k = 0; k < nkb; ++k) p += step(k) < mine;
  return p;
}

// one 64-row tile by LDS-DMA with 8 waves: wave w loads rows 8w .. 8w + 7 (one 1-KB piece)
struct TileDMA8 {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned voff;
  __device__ __forceinline__ void init(const bf16* g, int64_t ld, int N, int wave, int lane) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g, 0, (int)(((int64_t)(N - 1) * ld + 64) * 2), 0x00020000);
    const int r = 8 * wave + (lane >> 3);
    voff = (unsigned)((r * (int)ld + ((lane & 7) ^ swz(r)) * 8) * 2);
  }
  __device__ __forceinline__ void issue(char* tile, unsigned row0_bytes, int wave) const {
    lds_dma16(rsrc, tile + wave * 1024, voff, row0_bytes);
  }
};

// S', dP' of 32 queries x this wave's 32 keys -> dS; dV^T, dK^T MFMAs; dS^T (bf16) into the LDS image.
// K row fragments from the block's LDS image Kt, V fragments in registers; `mid` runs between the halves.
// qn = valid queries in the tile (>= 64: all); masking p by (query valid and key valid) is one select per
// element with a per-lane bound, cheaper than a second copy of the body
template <class Mid>
__device__ __forceinline__ void fb_tile_body(f32x16 (&dk)[2], f32x16 (&dv)[2], const bf16* Q_, const bf16* G_,
                                             const bf16* F_, const bf16* Kt, bf16* dsT, const bf16x8 (&vf)[4],
                                             bf16x8 one, bool key_ok, int qn, int wave, int lane, Mid&& mid) {
  const int krow = 32 * wave + (lane & 31);
#pragma unroll
  for (int sq = 0; sq < 2; ++sq) {
    if (sq == 1) mid();
    const int qr = sq * 32 + (lane & 31);
    f32x16 sc = mfma(frag_row_sw(Q_, qr, 0, lane), frag_row_sw(Kt, krow, 0, lane), zero16());
    f32x16 dp = mfma(frag_row_sw(G_, qr, 0, lane), vf[0], zero16());
#pragma unroll
    for (int ks = 1; ks < 4; ++ks) {
      sc = mfma(frag_row_sw(Q_, qr, ks, lane), frag_row_sw(Kt, krow, ks, lane), sc);
      dp = mfma(frag_row_sw(G_, qr, ks, lane), vf[ks], dp);
    }
    sc = mfma(row_frag(F_ + qr * 8), one, sc);
    dp = mfma(row_frag(F_ + 512 + qr * 8), one, dp);
    // rows of this lane: sq * 32 + acc_row(r) = sq * 32 + 4h + (r & 3) + 8 (r >> 2); valid iff < qn, and
    // only if this lane's key is valid: one per-lane bound, lim = key_ok ? qn - sq * 32 - 4h : 0
    const int lim = key_ok ? qn - sq * 32 - 4 * (lane >> 5) : 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = __builtin_amdgcn_exp2f(sc[r]);
      p = ((r & 3) + 8 * (r >> 2)) < lim ? p : 0.f;
      sc[r] = p;
      dp[r] *= p;
    }
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      const bf16x8 pf = acc_frag(sc, sk), df = acc_frag(dp, sk);
      // dS^T[key][q]: elements 0..3 = queries 16 sk + 4h + 0..3, 4..7 = 16 sk + 8 + 4h + 0..3 (of this sq)
      const int qa = sq * 32 + 16 * sk + 4 * (lane >> 5);
      *reinterpret_cast<bf16x4*>(dsT + sw_off(krow, qa)) = bf16x4{df[0], df[1], df[2], df[3]};
      *reinterpret_cast<bf16x4*>(dsT + sw_off(krow, qa + 8)) = bf16x4{df[4], df[5], df[6], df[7]};
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        dv[dh] = mfma(frag_tr_sw(G_, sq * 32 + 16 * sk, 32 * dh, lane), pf, dv[dh]);
        dk[dh] = mfma(frag_tr_sw(Q_, sq * 32 + 16 * sk, 32 * dh, lane), df, dk[dh]);
      }
    }
  }
}

__global__ __launch_bounds__(512) void attn_bwd_fused_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                             const bf16* __restrict__ qs, const bf16* __restrict__ frag,
                                                             bf16* __restrict__ dqkv, float* chain, unsigned* flags,
                                                             unsigned* err, int N, int H, int nkb, float scale,
                                                             float dk_scale) {
  __shared__ __attribute__((aligned(1024))) char lds[FBL_BYTES];
  const int t = threadIdx.x, lane0 = t & 63;
  int lane = lane0;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int w = xcd_work_item(blockIdx.x, gridDim.x);  // the key blocks of one (b, h): consecutive, one XCD
  const int bh = w / nkb, kb = w - bh * nkb, b = bh / H, hd = bh % H;
  const int nt = (N + 63) / 64;
  const int64_t ldt = (int64_t)3 * H * D, ldo = (int64_t)H * D;
  const bf16* base = qkv + (int64_t)b * N * ldt + hd * D;
  const unsigned tile_bytes = (unsigned)(64 * ldo * 2);
  bf16* const Kt = reinterpret_cast<bf16*>(lds + FBL_K);
  volatile int* const lflag = reinterpret_cast<volatile int*>(lds + FBL_FL);
  // the block's 256 keys -> Kt (wave w: its own 32 keys, 4 pieces; keys past N read as zeros)
  {
    const __amdgpu_buffer_rsrc_t kr =
        __builtin_amdgcn_make_buffer_rsrc((void*)(base + H * D), 0, (int)(((int64_t)(N - 1) * ldt + 64) * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = 32 * wave + 8 * i + (lane >> 3);  // local key row
      const unsigned vo = (unsigned)(((lane >> 3) * (int)ldt + ((lane & 7) ^ swz(rl)) * 8) * 2);
      lds_dma16(kr, lds + FBL_K + (4 * wave + i) * 1024, vo,
                (unsigned)((int64_t)(kb * FB_K + 32 * wave + 8 * i) * ldt * 2));
    }
  }
  if (t < 4) lflag[t] = 0;
  TileDMA8 qd, gd;
  FragDMA fd;
  qd.init(qs + (int64_t)b * N * ldo + hd * D, ldo, N, wave, lane);
  gd.init(dout + (int64_t)b * N * ldo + hd * D, ldo, N, wave, lane);
  fd.init(frag + (int64_t)bh * 2 * N * 8, N);
  {
    const int T0 = fb_tile(0, kb, nt);
    qd.issue(lds + FBL_Q, (unsigned)T0 * tile_bytes, wave);
    gd.issue(lds + FBL_G, (unsigned)T0 * tile_bytes, wave);
    fd.issue(reinterpret_cast<bf16*>(lds + FBL_F), (unsigned)T0 * 64u, wave, lane);
  }
  const int key = kb * FB_K + wave * 32 + (lane & 31);
  const bool key_ok = key < N;
  bf16x8 vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) vf[ks] = load_frag_global(base + (int64_t)key * ldt + 2 * H * D, ks, lane, key_ok);
  settle(vf);
  const bf16x8 one = ones3(lane);
  f32x16 dk[2], dv[2];
  dk[0] = zero16(); dk[1] = zero16(); dv[0] = zero16(); dv[1] = zero16();
  // the running dQ sums of this (b, h): [nt][4 sub-tiles][16 regs / 4][64 lanes][4] f32, and their flags
  // [nt][4]: flag (T, s) = number of key blocks whose partial of sub-tile s of tile T is in the sum
  const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(chain + (int64_t)bh * nt * (FB_TILE / 4)), 0, nt * FB_TILE, 0x00020000);
  unsigned* const fl = flags + (int64_t)bh * nt * 4;
  const int last = nkb - 1;
  const int dh = wave & 1, qh = (wave >> 1) & 1, kh = wave >> 2;  // this wave's dQ^T sub-tile and key half
  const int sub = wave & 3;
  // (pos 0 at step 0 for every block: its first tile never waits)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int prev_T = -1;
  bool prev_pub = false;  // this wave stored tile prev_T's running sum last step (kh == 0): publish it
  unsigned prev_val = 0;
  // one step; the buffer parity P is a compile-time constant (the loop is unrolled by 2), so every LDS
  // operand address is a per-lane offset + an immediate
  auto step = [&](int j, auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    const int T = fb_tile(j, kb, nt), pos = fb_pos(kb, T, nkb, nt);
    if (j + 1 < nt) {
      const int T1 = fb_tile(j + 1, kb, nt);
      qd.issue(lds + FBL_Q + (P ^ 1) * 8192, (unsigned)T1 * tile_bytes, wave);
      gd.issue(lds + FBL_G + (P ^ 1) * 8192, (unsigned)T1 * tile_bytes, wave);
      fd.issue(reinterpret_cast<bf16*>(lds + FBL_F + (P ^ 1) * 2048), (unsigned)T1 * 64u, wave, lane);
    }
    const bf16* Q_ = reinterpret_cast<const bf16*>(lds + FBL_Q + P * 8192);
    const bf16* G_ = reinterpret_cast<const bf16*>(lds + FBL_G + P * 8192);
    const bf16* F_ = reinterpret_cast<const bf16*>(lds + FBL_F + P * 2048);
    bf16* const dsT = reinterpret_cast<bf16*>(lds + FBL_S + P * 32768);
    // the running sum of this wave's sub-tile of T so far (its own poll matched at the end of the last
    // step), sc1 to registers, issued half way through the tile body (flies under the second half)
    u32x4 run[4];
    auto load_run = [&]() __attribute__((always_inline)) {
      if (kh == 0 && pos > 0) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          run[g] = __builtin_amdgcn_raw_buffer_load_b128(cr, lane * 16, T * FB_TILE + sub * FB_SUB + g * 1024, 16);
      }
    };
    fb_tile_body(dk, dv, Q_, G_, F_, Kt, dsT, vf, one, key_ok, N - T * 64, wave, lane, load_run);
    // this wave's loads (next tile's DMA, the running sum) and last step's running-sum stores are done:
    // publish last step's sum (the storing wave itself, behind its own vmcnt(0))
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (prev_pub && lane == 0) fb_st_flag(fl + prev_T * 4 + sub, prev_val);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // the one barrier of the step: dS^T of all 256 keys, next tile's operands
    __builtin_amdgcn_sched_barrier(0);
    // dQ^T (32 d x 32 q sub-tile (dh, qh)) over this wave's key half: K^T from Kt, dS^T from dsT
    f32x16 dq = zero16();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int k0 = kh * 128 + 16 * ks;
      dq = mfma(frag_tr_sw(Kt, k0, 32 * dh, lane), frag_tr_sw(dsT, k0, 32 * qh, lane), dq);
    }
    float* const red = reinterpret_cast<float*>(lds + FBL_R + sub * FB_SUB);
    prev_pub = false;
    if (kh == 1) {  // the other key half's partial -> LDS, then its LDS flag
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(red + g * 256 + lane * 4) = f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lflag[sub] = j + 1;
    } else {
      while (lflag[sub] != j + 1) __builtin_amdgcn_s_sleep(1);
      const bool final = pos == last;
      f32x4 v[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        v[g] = *reinterpret_cast<const f32x4*>(red + g * 256 + lane * 4) +
               f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
        if (pos > 0) v[g] += __builtin_bit_cast(f32x4, run[g]);
      }
      if (!final) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[g]), cr, lane * 16,
                                                 T * FB_TILE + sub * FB_SUB + g * 1024, 16);
        prev_pub = true;
        prev_val = (unsigned)(pos + 1);
      } else {
        // bf16 dQ of the sub-tile staged in this wave's (consumed) partial slot as [32 q][32 d] rows, then
        // stored as 64-B row pieces: query 32 qh + (lane & 31), d = 32 dh + 8 g + 4 h + 0..3
        char* const st = reinterpret_cast<char*>(red);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the partial is in registers
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4*>(st + (lane & 31) * FB_OP + (8 * g + 4 * (lane >> 5)) * 2) =
              bf16x4{(bf16)(v[g][0] * scale), (bf16)(v[g][1] * scale), (bf16)(v[g][2] * scale),
                     (bf16)(v[g][3] * scale)};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int pc = lane + 64 * i, r = pc >> 2, c = pc & 3, q = T * 64 + 32 * qh + r;
          const uint4 x = *reinterpret_cast<const uint4*>(st + r * FB_OP + c * 16);
          if (q < N) *reinterpret_cast<uint4*>(dqkv + ((int64_t)b * N + q) * ldt + hd * D + 32 * dh + c * 8) = x;
        }
      }
      // the next tile's predecessor for this sub-tile (published before its barrier of this step or earlier)
      if (j + 1 < nt) {
        const int T1 = fb_tile(j + 1, kb, nt), p1 = fb_pos(kb, T1, nkb, nt);
        if (p1 > 0) fb_wait(fl + T1 * 4 + sub, (unsigned)p1, err);
      }
    }
    prev_T = T;
  };
  {
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    int j = 0;
    for (; j + 1 < nt; j += 2) {
      step(j, P0{});
      step(j + 1, P1{});
    }
    if (j < nt) step(j, P0{});
  }
  // the last step's running sum: drained by its storing wave, then published
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (prev_pub && lane == 0) fb_st_flag(fl + prev_T * 4 + sub, prev_val);
  // dK, dV: staged through a dS^T image as [key][d] rows, stored as whole 128-B rows
  bf16* const stg = reinterpret_cast<bf16*>(lds + FBL_S);
#pragma unroll
  for (int which = 0; which < 2; ++which) {
    const f32x16* acc = which == 0 ? dk : dv;
    const float sc = which == 0 ? dk_scale : 1.f;
    __syncthreads();
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * h2 + 8 * g + 4 * (lane >> 5);
        *reinterpret_cast<bf16x4*>(stg + sw_off(32 * wave + (lane & 31), d0)) =
            bf16x4{(bf16)(acc[h2][4 * g] * sc), (bf16)(acc[h2][4 * g + 1] * sc), (bf16)(acc[h2][4 * g + 2] * sc),
                   (bf16)(acc[h2][4 * g + 3] * sc)};
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 64 * i + (t >> 3), c = t & 7, k = kb * FB_K + r;
      const uint4 v = *reinterpret_cast<const uint4*>(stg + sw_off(r, c * 8));
      if (k < N) *reinterpret_cast<uint4*>(dqkv + ((int64_t)b * N + k) * ldt + (1 + which) * H * D + hd * D + c * 8) = v;
    }
  }
}

// ------------------------------------------------------------------------------ f32 path
// Reference-precision kernels (exact f32 arithmetic, no flash tiling) used when the model runs
// in f32 for parity; one wave per query (forward, dQ) or per key (dK/dV); scores staged in LDS.
constexpr int MAXN = 3328;

__global__ __launch_bounds__(256) void attn_fwd_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                           float* __restrict__ lse, int N, int H, float scale) {
  __shared__ float sc[4][MAXN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, hd = bh % H;
  const int q = blockIdx.x * 4 + wave;
  if (q >= N) return;
  const int64_t ldt = (int64_t)3 * H * D;
  const float* base = qkv + (int64_t)b * N * ldt + hd * D;
  float qv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) qv[d] = base[(int64_t)q * ldt + d] * scale;
  float mx = -INFINITY;
  for (int k = lane; k < N; k += 64) {
    const float* kr = base + (int64_t)k * ldt + H * D;
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) s = fmaf(qv[d], kr[d], s);
    sc[wave][k] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int k = lane; k < N; k += 64) {
    const float p = expf(sc[wave][k] - mx);
    sc[wave][k] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  wave_sync();
  float o = 0.f;
  for (int k = 0; k < N; ++k) o = fmaf(sc[wave][k], base[(int64_t)k * ldt + 2 * H * D + lane], o);
  out[((int64_t)b * N + q) * H * D + hd * D + lane] = o / sum;
  if (lane == 0) lse[(int64_t)bh * N + q] = mx + logf(sum);
}

__global__ void attn_delta_f32_kernel(const float* __restrict__ out, const float* __restrict__ dout,
                                      float* __restrict__ delta, int B, int N, int H) {
  const int64_t total = (int64_t)B * N * H;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int hd = (int)(i % H);
    const int64_t bq = i / H;
    const int q = (int)(bq % N), b = (int)(bq / N);
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(out[i * D + d], dout[i * D + d], s);
    delta[((int64_t)b * H + hd) * N + q] = s;
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq_f32_kernel(const float* __restrict__ qkv, const float* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ delta, float* __restrict__ dqkv,
                                                              int N, int H, float scale) {
  __shared__ float sc[4][MAXN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, hd = bh % H;
  const int q = blockIdx.x * 4 + wave;
  if (q >= N) return;
  const int64_t ldt = (int64_t)3 * H * D, ldo = (int64_t)H * D;
  const float* base = qkv + (int64_t)b * N * ldt + hd * D;
  float qv[D], gv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    qv[d] = base[(int64_t)q * ldt + d] * scale;
    gv[d] = dout[((int64_t)b * N + q) * ldo + hd * D + d];
  }
  const float L = lse[(int64_t)bh * N + q], dl = delta[(int64_t)bh * N + q];
  for (int k = lane; k < N; k += 64) {
    const float* kr = base + (int64_t)k * ldt + H * D;
    const float* vr = kr + H * D;
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) { s = fmaf(qv[d], kr[d], s); dp = fmaf(gv[d], vr[d], dp); }
    const float p = expf(s - L);
    sc[wave][k] = p * (dp - dl);
  }
  wave_sync();
  float a = 0.f;
  for (int k = 0; k < N; ++k) a = fmaf(sc[wave][k], base[(int64_t)k * ldt + H * D + lane], a);
  dqkv[((int64_t)b * N + q) * ldt + hd * D + lane] = a * scale;
}

__global__ __launch_bounds__(256) void attn_bwd_dkdv_f32_kernel(const float* __restrict__ qkv,
                                                                const float* __restrict__ dout,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                float* __restrict__ dqkv, int N, int H, float scale) {
  __shared__ float sp[4][MAXN];
  __shared__ float sd[4][MAXN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, hd = bh % H;
  const int k = blockIdx.x * 4 + wave;
  if (k >= N) return;
  const int64_t ldt = (int64_t)3 * H * D, ldo = (int64_t)H * D;
  const float* base = qkv + (int64_t)b * N * ldt + hd * D;
  float kv[D], vv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    kv[d] = base[(int64_t)k * ldt + H * D + d] * scale;
    vv[d] = base[(int64_t)k * ldt + 2 * H * D + d];
  }
  for (int q = lane; q < N; q += 64) {
    const float* qr = base + (int64_t)q * ldt;
    const float* gr = dout + ((int64_t)b * N + q) * ldo + hd * D;
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) { s = fmaf(kv[d], qr[d], s); dp = fmaf(vv[d], gr[d], dp); }
    const float p = expf(s - lse[(int64_t)bh * N + q]);
    sp[wave][q] = p;
    sd[wave][q] = p * (dp - delta[(int64_t)bh * N + q]);
  }
  wave_sync();
  float dv = 0.f, dk = 0.f;
  for (int q = 0; q < N; ++q) {
    dv = fmaf(sp[wave][q], dout[((int64_t)b * N + q) * ldo + hd * D + lane], dv);
    dk = fmaf(sd[wave][q], base[(int64_t)q * ldt + lane], dk);
  }
  dqkv[((int64_t)b * N + k) * ldt + H * D + hd * D + lane] = dk * scale;
  dqkv[((int64_t)b * N + k) * ldt + 2 * H * D + hd * D + lane] = dv;
}

}  // namespace

extern "C" int mia_attn_fwd(const void* qkv, void* out, float* lse, int32_t dtype, int32_t B, int32_t N, int32_t H,
                            float scale, mia_stream_t stream) {
  MIA_CHECK_ARG(qkv && out && lse, "attn_fwd: null pointer");
  MIA_CHECK_ARG(B > 0 && N > 0 && H > 0 && (int64_t)B * H < 65536, "attn_fwd: bad shape");
  if (dtype == MIA_F32) {
    MIA_CHECK_ARG(N <= MAXN, "attn_fwd f32: N must be <= %d", MAXN);
    attn_fwd_f32_kernel<<<dim3((unsigned)cdiv(N, 4), (unsigned)(B * H)), 256, 0, as_stream(stream)>>>(
        (const float*)qkv, (float*)out, lse, N, H, scale);
    MIA_LAUNCH_CHECK("attn_fwd_f32");
    return 0;
  }
  MIA_CHECK_ARG(dtype == MIA_BF16, "attn_fwd: dtype");
  MIA_CHECK_ARG((int64_t)N * 3 * H * D * 2 < (1ll << 31), "attn_fwd: one sequence must span < 2 GiB");
  const int nqb = (int)cdiv(N, FWD_Q);
  MIA_CHECK_ARG((int64_t)nqb * B * H < (1ll << 31), "attn_fwd: grid too large");
  attn_fwd_kernel<false><<<(unsigned)(nqb * B * H), 256, 0, as_stream(stream)>>>(
      (const bf16*)qkv, (bf16*)out, lse, N, H, nqb, scale * LOG2E, nullptr, nullptr, nullptr);
  MIA_LAUNCH_CHECK("attn_fwd");
  return 0;
}

extern "C" int mia_attn_fwd_mx(const void* qkv, void* out, float* lse, void* q8, void* s8, int32_t B, int32_t N,
                               int32_t H, float scale, mia_stream_t stream) {
  MIA_CHECK_ARG(qkv && out && lse && q8 && s8, "attn_fwd_mx: null pointer");
  MIA_CHECK_ARG(B > 0 && N > 0 && H > 0 && (int64_t)B * H < 65536, "attn_fwd_mx: bad shape");
  MIA_CHECK_ARG((int64_t)N * 3 * H * D * 2 < (1ll << 31), "attn_fwd_mx: one sequence must span < 2 GiB");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(q8) & 3) == 0, "attn_fwd_mx: q8 must be 4-B aligned");
  const int nqb = (int)cdiv(N, FWD_Q);
  MIA_CHECK_ARG((int64_t)nqb * B * H < (1ll << 31), "attn_fwd_mx: grid too large");
  attn_fwd_kernel<true><<<(unsigned)(nqb * B * H), 256, 0, as_stream(stream)>>>(
      (const bf16*)qkv, (bf16*)out, lse, N, H, nqb, scale * LOG2E, (uint8_t*)q8, (uint8_t*)s8, nullptr);
  MIA_LAUNCH_CHECK("attn_fwd_mx");
  return 0;
}

// bf16 workspace: [Q' rows x 64 bf16][fragment rows: rows x 32 B][fused form: flags (B*H*nt u32) + error
// word, one 256-B-aligned block zeroed per call][running dQ sums: B*H*nt x 16 KB f32]
static int64_t round256(int64_t x) { return (x + 255) / 256 * 256; }
static int64_t fb_flags_offset(int32_t B, int32_t N, int32_t H) {
  const int64_t rows = (int64_t)B * N * H;
  return round256(rows * D * 2 + rows * 32);
}
static int64_t fb_flags_bytes(int32_t B, int32_t N, int32_t H) {
  return round256(((int64_t)B * H * cdiv(N, 64) * 4 + 1) * 4);  // [B*H][nt][4 sub-tiles] + error word
}

// the fused form needs every gap between consecutive contributions to a tile to be >= 2 steps
// (nt - FB_LAG (nkb - 1) >= 2 at the wrap; FB_LAG >= 2 elsewhere): true for every N (nt >= 4 nkb - 3)
static bool fb_ok(int32_t N) {
  const int nt = (int)cdiv(N, 64), nkb = (int)cdiv(N, FB_K);
  return nkb == 1 || nt - FB_LAG * (nkb - 1) >= 2;
}

// the part of the bf16 workspace the forward fills (mia_attn_fwd_save_q) and the two-kernel backward reads:
// Q' + the fragment rows (the one-pass form's flags and running dQ sums follow it)
extern "C" int64_t mia_attn_saved_q_bytes(int32_t B, int32_t N, int32_t H) { return fb_flags_offset(B, N, H); }

extern "C" int64_t mia_attn_bwd_workspace_bytes(int32_t dtype, int32_t B, int32_t N, int32_t H) {
  const int64_t rows = (int64_t)B * N * H;
  if (dtype == MIA_F32) return rows * 4;  // delta
  return fb_flags_offset(B, N, H) + fb_flags_bytes(B, N, H) + (int64_t)B * H * cdiv(N, 64) * FB_TILE;
}

// byte offset in the bf16 workspace of the fused backward's error word: 0 after a call = every dQ hand-off
// matched; non-zero = a bounded wait gave up (dQ of that call is not valid)
extern "C" int64_t mia_attn_bwd_error_offset(int32_t B, int32_t N, int32_t H) {
  return fb_flags_offset(B, N, H) + (int64_t)B * H * cdiv(N, 64) * 16;
}

static int attn_bwd_impl(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                         void* work, int32_t dtype, int32_t B, int32_t N, int32_t H, float scale, int q_ready,
                         int fused, mia_stream_t stream) {
  MIA_CHECK_ARG(qkv && out && dout && lse && dqkv && work, "attn_bwd: null pointer");
  MIA_CHECK_ARG(B > 0 && N > 0 && H > 0 && (int64_t)B * H < 65536, "attn_bwd: bad shape");
  hipStream_t s = as_stream(stream);
  const int64_t rows = (int64_t)B * N * H;
  if (dtype == MIA_F32) {
    MIA_CHECK_ARG(N <= MAXN, "attn_bwd f32: N must be <= %d", MAXN);
    float* delta = (float*)work;
    attn_delta_f32_kernel<<<(unsigned)std::min<int64_t>(cdiv(rows, 256), 16384), 256, 0, s>>>(
        (const float*)out, (const float*)dout, delta, B, N, H);
    MIA_LAUNCH_CHECK("attn_delta_f32");
    dim3 g4((unsigned)cdiv(N, 4), (unsigned)(B * H));
    attn_bwd_dq_f32_kernel<<<g4, 256, 0, s>>>((const float*)qkv, (const float*)dout, lse, delta, (float*)dqkv, N, H,
                                              scale);
    MIA_LAUNCH_CHECK("attn_bwd_dq_f32");
    attn_bwd_dkdv_f32_kernel<<<g4, 256, 0, s>>>((const float*)qkv, (const float*)dout, lse, delta, (float*)dqkv, N,
                                                H, scale);
    MIA_LAUNCH_CHECK("attn_bwd_dkdv_f32");
    return 0;
  }
  MIA_CHECK_ARG(dtype == MIA_BF16, "attn_bwd: dtype");
  MIA_CHECK_ARG(rows * 8 < (1ll << 31), "attn_bwd: B*N*H too large");
  MIA_CHECK_ARG((int64_t)N * 3 * H * D * 2 < (1ll << 31), "attn_bwd: one sequence must span < 2 GiB");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(work) & 15) == 0, "attn_bwd: workspace must be 16-B aligned");
  bf16* qs = (bf16*)work;
  bf16* frag = qs + rows * D;
  const float scale_log2 = scale * LOG2E;
  const bool one_pass = fused && fb_ok(N);
  // the prep pass: Q' when the forward did not leave it, the row-constant fragments for the one-pass
  // form (the two-kernel form's dQ kernel computes its own and writes them for dK/dV)
  if (!q_ready || one_pass) {
    attn_bwd_prep_kernel<<<(unsigned)cdiv(rows * 8, 256), 256, 0, s>>>((const bf16*)qkv, (const bf16*)out,
                                                                       (const bf16*)dout, lse, qs, frag, B, N, H,
                                                                       scale_log2, q_ready ? 0 : 1);
    MIA_LAUNCH_CHECK("attn_bwd_prep");
  }
  if (one_pass) {
    const int nkb = (int)cdiv(N, FB_K);
    MIA_CHECK_ARG((int64_t)nkb * B * H < (1ll << 31) && (int64_t)cdiv(N, 64) * FB_TILE < (1ll << 31),
                  "attn_bwd: grid too large");
    char* wb = reinterpret_cast<char*>(work);
    unsigned* flags = reinterpret_cast<unsigned*>(wb + fb_flags_offset(B, N, H));
    float* chain = reinterpret_cast<float*>(wb + fb_flags_offset(B, N, H) + fb_flags_bytes(B, N, H));
    // every flag and the error word start at 0 in each call (stream-ordered, no host sync)
    hipError_t e = hipMemsetAsync(flags, 0, (size_t)fb_flags_bytes(B, N, H), s);
    if (e != hipSuccess) return mia::fail(-(int)e, "attn_bwd: memset: %s", hipGetErrorString(e));
    attn_bwd_fused_kernel<<<(unsigned)(nkb * B * H), 512, 0, s>>>(
        (const bf16*)qkv, (const bf16*)dout, qs, frag, (bf16*)dqkv, chain, flags,
        flags + (int64_t)B * H * cdiv(N, 64) * 4, N, H, nkb, scale, 1.f / LOG2E);
    MIA_LAUNCH_CHECK("attn_bwd_fused");
    return 0;
  }
  const int nkb = (int)cdiv(N, BWD_K), nqb = (int)cdiv(N, BWD_Q);
  attn_bwd_dq_kernel<<<(unsigned)(nqb * B * H), 256, 0, s>>>((const bf16*)qkv, (const bf16*)out, (const bf16*)dout,
                                                             lse, frag, (bf16*)dqkv, N, H, nqb, scale, scale_log2);
  MIA_LAUNCH_CHECK("attn_bwd_dq");
  attn_bwd_dkdv_kernel<<<(unsigned)(nkb * B * H), 256, 0, s>>>((const bf16*)qkv, (const bf16*)dout, qs, frag,
                                                               (bf16*)dqkv, N, H, nkb, 1.f / LOG2E);
  MIA_LAUNCH_CHECK("attn_bwd_dkdv");
  return 0;
}

extern "C" int mia_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                            void* work, int32_t dtype, int32_t B, int32_t N, int32_t H, float scale,
                            mia_stream_t stream) {
  return attn_bwd_impl(qkv, out, dout, lse, dqkv, work, dtype, B, N, H, scale, 0, 0, stream);
}

// the bf16 backward in its two-kernel form (key-parallel dK/dV + query-parallel dQ, each recomputing S and
// dP; what mia_attn_bwd / mia_attn_bwd_saved_q run); q_ready = the forward wrote Q' into `work`
// (mia_attn_fwd_save_q)
extern "C" int mia_attn_bwd_two_pass(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                                     void* work, int32_t B, int32_t N, int32_t H, float scale, int32_t q_ready,
                                     mia_stream_t stream) {
  return attn_bwd_impl(qkv, out, dout, lse, dqkv, work, MIA_BF16, B, N, H, scale, q_ready, 0, stream);
}

// the bf16 backward in its fused one-pass form (S, dP, dS once per tile; dQ by the ordered hand-off):
// five MFMA products per tile instead of seven, but at B = 256, N = 1645 it measured 8.5-8.6 ms per layer
// against 8.2 ms for the two-kernel form, so it is not the default
extern "C" int mia_attn_bwd_fused(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                                  void* work, int32_t B, int32_t N, int32_t H, float scale, int32_t q_ready,
                                  mia_stream_t stream) {
  return attn_bwd_impl(qkv, out, dout, lse, dqkv, work, MIA_BF16, B, N, H, scale, q_ready, 1, stream);
}

// bf16 forward that also writes Q' (the backward's scaled query operand) into the backward workspace
// `work` (mia_attn_bwd_workspace_bytes); q8 / s8 non-null = the MX-fp8 form (mia_attn_fwd_mx)
extern "C" int mia_attn_fwd_save_q(const void* qkv, void* out, float* lse, void* q8, void* s8, void* work, int32_t B,
                                   int32_t N, int32_t H, float scale, mia_stream_t stream) {
  MIA_CHECK_ARG(qkv && out && lse && work && (!q8 == !s8), "attn_fwd_save_q: null pointer");
  MIA_CHECK_ARG(B > 0 && N > 0 && H > 0 && (int64_t)B * H < 65536, "attn_fwd_save_q: bad shape");
  MIA_CHECK_ARG((int64_t)N * 3 * H * D * 2 < (1ll << 31), "attn_fwd_save_q: one sequence must span < 2 GiB");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(work) & 15) | (q8 ? reinterpret_cast<uintptr_t>(q8) & 3 : 0)) == 0,
                "attn_fwd_save_q: work must be 16-B and q8 4-B aligned");
  const int nqb = (int)cdiv(N, FWD_Q);
  MIA_CHECK_ARG((int64_t)nqb * B * H < (1ll << 31), "attn_fwd_save_q: grid too large");
  if (q8)
    attn_fwd_kernel<true><<<(unsigned)(nqb * B * H), 256, 0, as_stream(stream)>>>(
        (const bf16*)qkv, (bf16*)out, lse, N, H, nqb, scale * LOG2E, (uint8_t*)q8, (uint8_t*)s8, (bf16*)work);
  else
    attn_fwd_kernel<false><<<(unsigned)(nqb * B * H), 256, 0, as_stream(stream)>>>(
        (const bf16*)qkv, (bf16*)out, lse, N, H, nqb, scale * LOG2E, nullptr, nullptr, (bf16*)work);
  MIA_LAUNCH_CHECK("attn_fwd_save_q");
  return 0;
}

// the bf16 backward when the forward already wrote Q' into `work` (mia_attn_fwd_save_q)
extern "C" int mia_attn_bwd_saved_q(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                                    void* work, int32_t B, int32_t N, int32_t H, float scale, mia_stream_t stream) {
  return attn_bwd_impl(qkv, out, dout, lse, dqkv, work, MIA_BF16, B, N, H, scale, 1, 0, stream);
}
