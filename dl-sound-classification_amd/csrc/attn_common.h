// Device helpers shared by the attention kernels (attention.hip: forward, two-kernel and fused backward;
// attn_bwd.hip: the one-pass training backward), gfx950.  Everything is in an anonymous namespace: each
// translation unit gets its own copy (all inline / constexpr, plus the small prep kernel).
#pragma once
#include "common.h"

#include <type_traits>

namespace {

constexpr int D = 64;
constexpr int LROW = 72;  // LDS row stride in bf16 (144 B): conflict-free ds_read_b128 rows
// Stride of a tile read ONLY transposed (forward V): 96 bf16 = 48 dwords puts the 4 rows of one
// ds_read_b64_tr_b16 group on disjoint 16-bank windows (rows 0..3 -> banks 0, 48, 32, 16); at the
// 36-dword LROW stride rows r and r + 2 overlap by 8 banks (2-way conflicts, SQ_LDS_BANK_CONFLICT).
constexpr int VROW = 96;
constexpr float LOG2E = 1.4426950408889634f;

typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// 64 rows x 64 bf16 from global (row stride `ld` elements) into LDS [64][LROW]; rows >= nvalid -> 0
__device__ __forceinline__ void stage64(bf16* lds, const bf16* g, int64_t ld, int nvalid, int t) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = t + 256 * s;
    const int row = c >> 3, c16 = c & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < nvalid) v = *reinterpret_cast<const uint4*>(g + row * ld + c16 * 8);
    *reinterpret_cast<uint4*>(lds + row * LROW + c16 * 8) = v;
  }
}

__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int sw_off(int r, int col) { return r * 64 + (((col >> 3) ^ swz(r)) << 3) + (col & 7); }

// Register-staged tile copy, split so the global loads of tile t+1 fly under tile t's MFMAs
// (issue early / write late): 64 rows x 64 bf16 = 2 x 16 B per thread.
struct Stage64 {
  uint4 v[2];
  // rows >= nvalid re-read the last valid row (finite data; the scores of such keys are masked to
  // -inf so their V rows meet p = 0): an unconditional load keeps hipcc from branching around it
  __device__ __forceinline__ void load(const bf16* g, int64_t ld, int nvalid, int t) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = t + 256 * s;
      const int row = min(c >> 3, nvalid - 1), c16 = c & 7;
      v[s] = *reinterpret_cast<const uint4*>(g + row * ld + c16 * 8);
    }
  }
  __device__ __forceinline__ void store_sw(bf16* lds, int t) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = t + 256 * s;
      const int r = c >> 3;
      *reinterpret_cast<uint4*>(lds + r * 64 + (((c & 7) ^ swz(r)) << 3)) = v[s];
    }
  }
  template <int ROW = LROW>
  __device__ __forceinline__ void store(bf16* lds, int t) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = t + 256 * s;
      *reinterpret_cast<uint4*>(lds + (c >> 3) * ROW + (c & 7) * 8) = v[s];
    }
  }
};

// Row fragment: tile[row][16ks + 8h + j], j = 0..7 (A operand rows / B operand columns).
__device__ __forceinline__ bf16x8 frag_row(const bf16* lds, int row, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + row * LROW + ks * 16 + 8 * (lane >> 5));
}

// Transposed fragment in the accumulator k-order: element j = tile[k0 + 8(j>>2) + 4h + (j&3)][c0 + (lane&31)]
// (two ds_read_b64_tr_b16: 4 consecutive tile rows x 16 columns per 16-lane group).
template <int ROW = LROW>
__device__ __forceinline__ bf16x8 frag_tr(const bf16* lds, int k0, int c0, int lane) {
  const int i16 = lane & 15, g = lane >> 4, h = lane >> 5;
  const int col = c0 + 16 * (g & 1) + 4 * (i16 & 3);
  const int r = k0 + 4 * h + (i16 >> 2);
  const bf16* p0 = lds + r * ROW + col;
  const bf16* p1 = p0 + 8 * ROW;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p1));
  s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, c);
}

// Swizzled [rows][64] bf16 tile for a tile read BOTH as rows (ds_read_b128) and transposed
// (ds_read_b64_tr_b16): 16-B chunk c of row r sits at chunk c ^ swz(r).  Rows r, r + 1 use opposite
// bank halves (128-B rows); over the 8 same-parity rows of a ds_read_b128 16-lane group swz takes 8
// distinct values, and rows r, r + 2 of a transposed read differ in swz bit 2, so their 4-chunk
// column blocks land in opposite 64-B halves: both kinds of read are conflict-free, no padding.

__device__ __forceinline__ bf16x8 frag_row_sw(const bf16* lds, int row, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + sw_off(row, ks * 16 + 8 * (lane >> 5)));
}

__device__ __forceinline__ bf16x8 frag_tr_sw(const bf16* lds, int k0, int c0, int lane) {
  const int i16 = lane & 15, g = lane >> 4, h = lane >> 5;
  const int col = c0 + 16 * (g & 1) + 4 * (i16 & 3);
  const int r = k0 + 4 * h + (i16 >> 2);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(lds + sw_off(r, col)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(lds + sw_off(r + 8, col)));
  s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, c);
}

// Make the compiler wait for global loads of loop-invariant fragments HERE (before the tile loop): otherwise
// it re-checks them with a vmcnt at the loop head of every iteration, and vmcnt also counts the loop's
// own in-flight tile DMAs (lds_dma16), so every tile would wait for its successor's load.
template <int n>
__device__ __forceinline__ void settle(const bf16x8 (&f)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) asm volatile("" ::"v"(f[i]));
}
__device__ __forceinline__ void settle1(const bf16x8& f) { asm volatile("" ::"v"(f)); }

// accumulator registers 8s..8s+7 -> bf16 operand fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)a[8 * s + j];
  return f;
}

__device__ __forceinline__ bf16x8 load_frag_global(const bf16* row, int ks, int lane, bool valid) {
  if (!valid) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
    return z;
  }
  return *reinterpret_cast<const bf16x8*>(row + ks * 16 + 8 * (lane >> 5));
}

// v_max3_f32 as one instruction: fmaxf on MFMA results otherwise gets a canonicalising v_max per
// operand (IEEE mode) and no max3 fusion
__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// max(x[lane], x[lane ^ 32]) without an LDS round trip (v_permlane32_swap exchanges the halves)
__device__ __forceinline__ float half_exchange_max(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ __forceinline__ float half_exchange_sum(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

// row index of accumulator register r for this lane half
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ------------------------------------------------------------------------------ forward
// XCD-aware block order: consecutive work items (the query blocks of one (b, h), which stream the
// same K/V) land on ONE XCD so K/V come from that XCD's L2, not from HBM once per XCD.  Blocks are
// dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch), so slot s of XCD x
// takes work item x * (total / 8) + s.  Pure speed mapping: any placement gives the same result.
__device__ __forceinline__ int xcd_work_item(int L, int total) {
  return (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);
}

// Tiles s0 .. ntiles - 1 of a 3-slot ring with no remainder code: the last round's second and third
// tiles are guarded inside the loop (wave-uniform branches), so every tile is the loop's own code and
// register allocation (straight-line remainder copies spilled)
template <int S0, class Body>
__device__ __forceinline__ void ring3_guarded(int s0, int ntiles, Body&& body) {
  using F = std::false_type;
  using C0 = std::integral_constant<int, S0 % 3>;
  using C1 = std::integral_constant<int, (S0 + 1) % 3>;
  using C2 = std::integral_constant<int, (S0 + 2) % 3>;
  for (int j = s0; j < ntiles; j += 3) {
    body(F{}, C0{}, j);
    if (j + 1 < ntiles) body(F{}, C1{}, j + 1);
    if (j + 2 < ntiles) body(F{}, C2{}, j + 2);
  }
}

// Tiles s0 .. ntiles - 1 of a 3-slot LDS ring (K/V or Q/dO tiles arrive by LDS-DMA two tiles ahead of
// their use), slot = tile % 3 as a compile-time constant (tile s0's slot is S0 % 3, so every LDS address
// is base + immediate); the last tile is the TAIL form when `tail`.  body(tail_t, slot_t, j).
template <int S0, class Body>
__device__ __forceinline__ void ring3(int s0, int ntiles, bool tail, Body&& body) {
  using T = std::true_type;
  using F = std::false_type;
  using C0 = std::integral_constant<int, S0 % 3>;
  using C1 = std::integral_constant<int, (S0 + 1) % 3>;
  using C2 = std::integral_constant<int, (S0 + 2) % 3>;
  int j = s0;
  for (; j + 3 < ntiles; j += 3) {
    body(F{}, C0{}, j);
    body(F{}, C1{}, j + 1);
    body(F{}, C2{}, j + 2);
  }
  const int r = ntiles - j;
  if (r == 1) {
    if (tail) body(T{}, C0{}, j);
    else body(F{}, C0{}, j);
  } else if (r == 2) {
    body(F{}, C0{}, j);
    if (tail) body(T{}, C1{}, j + 1);
    else body(F{}, C1{}, j + 1);
  } else if (r == 3) {
    body(F{}, C0{}, j);
    body(F{}, C1{}, j + 1);
    if (tail) body(T{}, C2{}, j + 2);
    else body(F{}, C2{}, j + 2);
  }
}

// Forward structure (the loop is vector-issue bound at head dim 64, so the design is a VALU diet):
//  * one wave = 32 queries (query on the lane), 4 waves = 128 queries per block, <= 168 registers so
//    three waves share each SIMD and one wave's softmax issues beside the others' MFMAs;
//  * K / V tiles arrive by LDS-DMA (global_load_lds_dwordx4, no staging registers, no ds_write),
//    double-buffered: tile j+1 is requested before tile j is computed;
//  * Q is pre-scaled by scale * log2(e) (bf16) and the running max m is rounded UP to a
//    bf16-representable value, so "- m" rides the QK^T MFMA chain as a fifth k-step
//    (ones column of K x (-m) row of Q): the scores leave the MFMA as s - m, p = exp2(.) directly;
//  * the running max is not recomputed per tile: m only has to keep every p finite and O in range,
//    so a tile whose exp-sum stays <= 2^16 (each p <= 2^16) is accepted as is, and only a tile that
//    exceeds it (or the first tile) takes the wave-uniform rare path that computes the tile max,
//    moves m, rescales O / l and recomputes the tile's p.
constexpr int FWD_Q = 128;
constexpr float FWD_SUM_LIMIT = 65536.f;

typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;

// 16 B per lane from a buffer into LDS (buffer_load_dwordx4 ... lds, M0 = the wave's LDS destination) as
// inline asm: issued through the builtin, the compiler treats the in-flight DMA as a possible writer of
// every LDS location and puts vmcnt(0) in front of the next ds_read -- in these kernels the NEXT tile's
// DMA, so every tile waited for its successor's load.  Here the kernels' own counted vmcnt + barrier
// order the DMA against its readers (each issue site says which), and M0 is saved and restored.
// The wait states the compiler pads around its own LDS-DMA are written into the string, since nothing inside
// an asm statement is padded (gfx9 manually-inserted wait states):
//  * s_nop 0 between the M0 write and the buffer_load ... lds that reads it (SALU writes M0 -> LDS-DMA: 1 state;
//    the builtin form emits exactly this nop).  Without it the DMA may take the PREVIOUS M0 -- `keep`, the
//    value this statement restores -- and write its 1 KB to a stale LDS address;
//  * s_nop 4 opening the string: the descriptor / soffset SGPRs may come from a v_readfirstlane the compiler
//    placed just before (VALU writes SGPR -> VMEM reads that SGPR: 5 states).
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t rsrc, const void* lds, unsigned voff, unsigned soff) {
  const unsigned a = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_vp)lds);
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(a), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

// x rounded toward +inf to a bf16-representable float (its negation is exact in bf16)
__device__ __forceinline__ float bf16_ceil(float x) {
  unsigned u = __builtin_bit_cast(unsigned, x);
  if (!(u & 0x80000000u)) u += 0xFFFFu;
  return __builtin_bit_cast(float, u & 0xFFFF0000u);
}

// One 64-row x 64-col bf16 tile (8 KB, sw_off layout) by LDS-DMA: 8 pieces of 1 KB = 8 rows each,
// wave w issues pieces 2w and 2w + 1; lane i of a piece fills 16-B slot (i & 7) of row 8p + (i >> 3),
// i.e. it loads chunk (i & 7) ^ swz(row) of that row (the swizzle rides the SOURCE address).  Buffer
// loads: the per-lane byte offset is fixed, the tile start rides soffset (no VALU per tile), and rows
// past the sequence end fall outside the descriptor's range and read as zeros (their keys are masked,
// their V rows meet p = 0).
struct TileDMA {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned voff[2];
  __device__ __forceinline__ void init(const bf16* g, int64_t ld, int N, int wave, int lane) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g, 0, (int)(((int64_t)(N - 1) * ld + 64) * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 8 * (2 * wave + i) + (lane >> 3);
      voff[i] = (unsigned)((r * (int)ld + ((lane & 7) ^ swz(r)) * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(bf16* tile, unsigned row0_bytes, int wave) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) lds_dma16(rsrc, tile + (2 * wave + i) * 512, voff[i], row0_bytes);
  }
};


// ------------------------------------------------------------------------------ backward
// Both backward kernels recompute P from the SAME MFMA operands the forward used (Q' = bf16(q * scale
// * log2 e) against K), so P sums to one exactly as the forward's lse normalised it.  The per-query
// row constants ride the MFMA chains as a fifth k-step, each split into three bf16 parts (exact to
// f32): S' = Q'K^T - L2 (L2 = lse * log2 e) gives p = exp2(S') directly, and dP' = dO V^T - delta
// gives dS = p * dP' with one multiply.
//
// prep: per (b, q, h) row, Q' (B, N, H, 64) bf16 and the fragment rows (B*H, 2, N, 8) bf16:
// part 0 = [-L2 (3 parts), 0 x 5], part 1 = [-delta (3 parts), 0 x 5], delta = sum_d dO * O.
// 8 lanes per row.
// x = h + m + l (three bf16 parts, exact to f32 rounding) into elements 0..2 of f
__device__ __forceinline__ void split3(float x, bf16x8& f) {
  const bf16 h = (bf16)x;
  const float r1 = x - (float)h;
  const bf16 m = (bf16)r1;
  f[0] = h;
  f[1] = m;
  f[2] = (bf16)(r1 - (float)m);
}

__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ out,
                                                            const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                            bf16* __restrict__ qs, bf16* __restrict__ frag, int B,
                                                            int N, int H, float scale_log2, int write_qs) {
  const int64_t rows = (int64_t)B * N * H;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int part = threadIdx.x & 7;
  if (i >= rows) return;  // whole 8-lane groups leave together
  const int hd = (int)(i % H);
  const int64_t bq = i / H;
  const int q = (int)(bq % N), b = (int)(bq / N);
  const bf16x8 o = *reinterpret_cast<const bf16x8*>(out + i * D + part * 8);
  const bf16x8 g = *reinterpret_cast<const bf16x8*>(dout + i * D + part * 8);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s = fmaf((float)o[j], (float)g[j], s);
  if (write_qs) {  // (skipped when the forward wrote Q': mia_attn_fwd_save_q)
    const bf16x8 qv = *reinterpret_cast<const bf16x8*>(qkv + (bq * 3 * H + hd) * D + part * 8);
    bf16x8 qsc;
#pragma unroll
    for (int j = 0; j < 8; ++j) qsc[j] = (bf16)((float)qv[j] * scale_log2);
    *reinterpret_cast<bf16x8*>(qs + i * D + part * 8) = qsc;
  }
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  s += __shfl_xor(s, 4);
  if (part < 2) {
    const int64_t bhh = (int64_t)b * H + hd;
    const float x = part == 0 ? -lse[bhh * N + q] * LOG2E : -s;
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (bf16)0.f;
    split3(x, f);
    *reinterpret_cast<bf16x8*>(frag + ((bhh * 2 + part) * N + q) * 8) = f;
  }
}

// ones fragment for the fifth k-step: elements 0..2 of the low lane half = 1
__device__ __forceinline__ bf16x8 ones3(int lane) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)0.f;
  if (lane < 32) { f[0] = (bf16)1.f; f[1] = (bf16)1.f; f[2] = (bf16)1.f; }
  return f;
}

// The fragment rows of 64 queries by LDS-DMA into [part][64][8]: waves 0 and 1 issue part 0 / 1
// (1 KB each, 16-B rows: the per-lane row reads are conflict-free).  Past the sequence end part 0
// reads part 1's rows (finite; those queries are masked) and part 1 reads zeros.
struct FragDMA {
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned part_bytes;
  __device__ __forceinline__ void init(const bf16* g, int N) {
    part_bytes = (unsigned)N * 16;
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g, 0, (int)(2 * part_bytes), 0x00020000);
  }
  __device__ __forceinline__ void issue(bf16* tile, unsigned row0, int wave, int lane) const {
    if (wave < 2) lds_dma16(rsrc, tile + wave * 512, (unsigned)wave * part_bytes + lane * 16, row0 * 16);
  }
};

// A fifth-k-step fragment row read by every lane: the high lane half carries k = 8..15, which meet
// the zero half of the ones fragment, so its (finite) copy of the row contributes nothing.
__device__ __forceinline__ bf16x8 row_frag(const bf16* row) { return *reinterpret_cast<const bf16x8*>(row); }

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned fb_ld_flag(const unsigned* p) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ void fb_st_flag(unsigned* p, unsigned v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}


}  // namespace
