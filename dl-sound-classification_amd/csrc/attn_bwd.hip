// One-pass bf16 attention backward for training (mia_attn_bwd_onepass), gfx950: S, dP and dS computed once
// per tile, dV / dK accumulated in registers, dQ = dS K summed over the key blocks of each (b, h) by an ordered
// hand-off of running f32 sums (bit-reproducible).  Replaces the backward of F.scaled_dot_product_attention
// inside timm's Attention (reference src/models/ast.py:60-61).  The two-pass backward (attention.hip) remains
// the AST default while it is the faster of the two (attention backward).
// Compiled without -amdgpu-mfma-vgpr-form (see the Makefile): its dK / dV sums live in the AGPR half of
// the register file.
//
// One 4-wave workgroup per (b, h, 256-key block) and CU, one wave per SIMD with up to 512 registers; each wave
// owns 64 keys (two 32-key halves, key on the lane) and keeps their K / V fragments in registers, the block's
// 256 keys also as an LDS image (K^T fragments for dQ).  Per 64-query tile each wave computes S' and dP' ONCE
// (Q' and dO row fragments from LDS against its K / V rows, the row constants -L2 and -delta as a fifth
// k-step), P = exp2(S') and dS = P dP', accumulates dV^T += dO^T P and dK^T += Q'^T dS and writes dS^T (bf16)
// into a double-buffered LDS image; the dQ^T sub-tile of wave w (d half w & 1, query half w >> 1) of the
// PREVIOUS tile is computed over the block's 256 keys during this tile's work: 5 GEMM units per tile, no
// recompute.  Each query half runs as a software pipeline in four stages (cb2_half_staged).
//
// dQ sums over the key blocks of one (b, h) by an ORDERED HAND-OFF of running f32 sums (no float atomics:
// bit-reproducible).  Block kb walks the query tiles rotated by lag * kb; a tile's contributions are added
// in the order of the steps at which the blocks reach it; the first stores its partial, the last writes bf16
// dQ.  Each wave owns its sub-tile's link: its `sc1` stores of the running sum (16 B per lane) are published
// by an `sc1` flag store in the MIDDLE of the next step, behind a vmcnt wait that the step's own loads need
// anyway (no wait for the store acknowledgement on the critical path); the successor block polls the flag
// with an `sc1` load issued with its tile DMA at the start of the step that needs the sum, checks it in the
// middle of that step and loads the sum (`sc1`, to registers) for the link after the second half
// (MI355X_MICROARCH.md, visibility table row 1: one storing wave per flag, every byte stored and loaded
// `sc1`, the store drained before its flag).  With a lag of >= 2 steps between consecutive contributions
// the sum is published a step before it is polled; at a lag of 1 (sequence lengths where 2 does not fit) the
// successor waits about half a step.  A block only waits for a contribution made at an earlier step (the
// first contribution of a tile is made at the step where it has no predecessor), the blocks of one (b, h)
// are consecutive work items of one XCD and the workgroups are dispatched in order, so a wait always ends;
// it is bounded anyway (CB_SPIN_TICKS of the 100 MHz counter): a timeout sets the caller's sticky error word
// and every later wait of any call gives up at once instead of hanging the GPU.
// Rows past the sequence end read as zeros everywhere (K / V / Q' / dO by the descriptors' ranges, the row
// constants per part): such a key meets K = V = 0, such a query p = 1 and dP' = 0, so dS = 0 there, nothing
// is masked and nothing past the end is stored.
#include "attn_common.h"

namespace {

constexpr int CB_SUB = 4096;                   // one 32 x 32 f32 dQ^T sub-tile in register order
constexpr int CB_TILE = 4 * CB_SUB;            // the four sub-tiles of a 64-query tile
constexpr unsigned long long CB_SPIN_TICKS = 20000000ull;  // 200 ms at 100 MHz

// the row-constant fragments of 64 queries by LDS-DMA, one descriptor per part (rows past N read zeros in
// both parts): waves 0 / 1 issue part 0 / 1
struct FragDMA2 {
  __amdgpu_buffer_rsrc_t rsrc;
  __device__ __forceinline__ void init(const bf16* g, int N, int wave) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(g + (int64_t)(wave & 1) * N * 8), 0, N * 16, 0x00020000);
  }
  __device__ __forceinline__ void issue(bf16* tile, unsigned row0, int wave, int lane) const {
    if (wave < 2) lds_dma16(rsrc, tile + wave * 512, lane * 16, row0 * 16);
  }
};

// The tile order of block kb: step j processes tile (j - LAG kb) mod nt (one modulo at the start, then +1 with
// a wrap); a tile's chain position = the number of blocks that reach it at an earlier step, in closed form:
// blocks k >= z = ceil((nt - T) / LAG) wrap past nt (step T + LAG k - nt < T) and come first, in k order,
// then k < z (LAG (nkb - 1) < nt: at most one wrap).  LAG is a compile-time constant, so a step's order
// bookkeeping is a handful of scalar instructions (the search over the blocks with run-time modulos it
// replaced was ~500 scalar instructions per step).
template <int LAG>
struct CbOrder {
  int nt, nkb, kb;
  __device__ __forceinline__ int first() const { return (nt - (LAG * kb) % nt) % nt; }
  __device__ __forceinline__ int next(int T) const { return T + 1 == nt ? 0 : T + 1; }
  __device__ __forceinline__ int pos(int T) const {
    const int z = min(nkb, (nt - T + LAG - 1) / LAG);
    return kb >= z ? kb - z : nkb - z + kb;
  }
};

__device__ __forceinline__ unsigned cb_load_flag(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, 0, off, 16);  // sc1
}

// wave-uniform, bounded: until flag == want (a timeout, or an earlier one of any call, sets / reads *err)
__device__ __forceinline__ void cb_spin(const unsigned* flag, unsigned want, unsigned* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (fb_ld_flag(flag) == want) return;
    if (fb_ld_flag(err) != 0u) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > CB_SPIN_TICKS) {
      fb_st_flag(err, 1u);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

constexpr int CB2_K = 256;
constexpr int CB2L_Q = 0;                        // [2][64][64] bf16 Q' tiles (sw_off)
constexpr int CB2L_G = CB2L_Q + 2 * 8192;        // [2][64][64] bf16 dO tiles (sw_off)
constexpr int CB2L_F = CB2L_G + 2 * 8192;        // [2][2 parts][64][8] bf16 fifth-k-step rows
constexpr int CB2L_S = CB2L_F + 2 * 2048;        // [2][256][64] bf16 dS^T (sw_off)
constexpr int CB2L_K = CB2L_S + 2 * 32768;       // [256][64] bf16 the block's keys (sw_off): K rows and K^T
constexpr int CB2L_BYTES = CB2L_K + 32768;       // 135 168 B: one workgroup per CU

// The same half as a software pipeline in four stages separated by sched_barriers (one wave per SIMD has no
// partner to hide latency behind, so the MFMA chains of one unit issue while the VALU of the previous one
// runs): A = S / dP of key half 0 (their operand reads issued first) with the dV / dK transposed fragments and
// the first dQ fragments requested under it; B = S / dP of key half 1 under the softmax of half 0 (exp, dS,
// the bf16 operands, the dS^T image writes); C = dV / dK of half 0 and four k-steps of the previous tile's dQ
// under the softmax of half 1; D = dV / dK of half 1 and four more dQ k-steps.  sched_group_barrier lays one
// MFMA and its share of the stage's other instructions into each MFMA gap.  dq: k-steps kq0 .. kq0 + 7 of the
// previous tile's dQ^T (A = K^T from the block's image Kt, B = that tile's dS^T image dsP), DQ: any at all.
#ifndef CB_LEAD
#define CB_LEAD 3  // MFMAs issued at the head of stages B and C before any VALU
#endif
#ifndef CB_PREF
#define CB_PREF true  // read query half 1's S / dP operands during half 0's last stage
#endif
// The S / dP row operands of a query half (Q' and dO row fragments, the two row-constant fragments)
struct HalfOps {
  bf16x8 qa[4], ga[4], fl, fd;
  __device__ __forceinline__ void load(const bf16* Q_, const bf16* G_, const bf16* F_, int sq, int lane) {
    const int qr = sq * 32 + (lane & 31);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qa[ks] = frag_row_sw(Q_, qr, ks, lane);
      ga[ks] = frag_row_sw(G_, qr, ks, lane);
    }
    fl = row_frag(F_ + qr * 8);
    fd = row_frag(F_ + 512 + qr * 8);
  }
};

// PRE: op already holds this half's operands (read during the previous half); NEXT: read query half 1's
// operands into op during stage D (the S / dP MFMAs that used op are done by then), so half 1 starts on
// operands that are already in registers instead of waiting out the LDS latency
template <bool DQ, bool PRE, bool NEXT>
__device__ __forceinline__ void cb2_half_staged(f32x16 (&dk)[2][2], f32x16 (&dv)[2][2], f32x16& dq, HalfOps& op,
                                                const bf16* Q_, const bf16* G_, const bf16* F_, bf16* dsT,
                                                const bf16* Kt, const bf16* dsP, int kq0, int dhw, int qhw,
                                                const bf16x8 (&kf)[2][4], const bf16x8 (&vf)[2][4], bf16x8 one,
                                                int sq, int wave, int lane) {
  if constexpr (!PRE) op.load(Q_, G_, F_, sq, lane);
  const bf16x8 (&qa)[4] = op.qa;
  const bf16x8 (&ga)[4] = op.ga;
  const bf16x8 fl = op.fl, fd = op.fd;
  __builtin_amdgcn_sched_barrier(0);
  // ---- A
  f32x16 sc[2], dp[2];
  auto sdp = [&](int kk) __attribute__((always_inline)) {
    sc[kk] = mfma(qa[0], kf[kk][0], zero16());
    dp[kk] = mfma(ga[0], vf[kk][0], zero16());
#pragma unroll
    for (int ks = 1; ks < 4; ++ks) {
      sc[kk] = mfma(qa[ks], kf[kk][ks], sc[kk]);
      dp[kk] = mfma(ga[ks], vf[kk][ks], dp[kk]);
    }
    sc[kk] = mfma(fl, one, sc[kk]);
    dp[kk] = mfma(fd, one, dp[kk]);
  };
  sdp(0);
  bf16x8 gt[2][2], qt[2][2];
#pragma unroll
  for (int sk = 0; sk < 2; ++sk)
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      gt[sk][dh] = frag_tr_sw(G_, sq * 32 + 16 * sk, 32 * dh, lane);
      qt[sk][dh] = frag_tr_sw(Q_, sq * 32 + 16 * sk, 32 * dh, lane);
    }
  bf16x8 ka[2][4], sf[2][4];
  if constexpr (DQ) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      ka[0][ks] = frag_tr_sw(Kt, 16 * (kq0 + ks), 32 * dhw, lane);
      sf[0][ks] = frag_tr_sw(dsP, 16 * (kq0 + ks), 32 * qhw, lane);
    }
  }
#pragma unroll
  for (int g = 0; g < 10; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, DQ ? 3 : 2, 0);  // DS read
  }
  __builtin_amdgcn_sched_barrier(0);
  // ---- B
  bf16x8 pf[2][2], df[2][2];
  auto softmax = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(sc[kk][r]);
      sc[kk][r] = p;
      dp[kk][r] *= p;
    }
    const int krow = 64 * wave + 32 * kk + (lane & 31);
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      pf[kk][sk] = acc_frag(sc[kk], sk);
      df[kk][sk] = acc_frag(dp[kk], sk);
      const int qa4 = sq * 32 + 16 * sk + 4 * (lane >> 5);
      const bf16x8 d = df[kk][sk];
      *reinterpret_cast<bf16x4*>(dsT + sw_off(krow, qa4)) = bf16x4{d[0], d[1], d[2], d[3]};
      *reinterpret_cast<bf16x4*>(dsT + sw_off(krow, qa4 + 8)) = bf16x4{d[4], d[5], d[6], d[7]};
    }
  };
  sdp(1);
  softmax(0);
  // the first MFMAs go out alone: half 0's S / dP chains (stage A's last MFMAs) complete under them before
  // the first exp needs them (in-order issue: a stalled VALU would hold every MFMA behind it)
  __builtin_amdgcn_sched_group_barrier(0x008, CB_LEAD, 1);
#pragma unroll
  for (int g = 0; g < 10 - CB_LEAD; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 7, 1);  // VALU
    if (g & 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 1);  // DS write
  }
  __builtin_amdgcn_sched_group_barrier(0x002, 64, 1);  // the rest of the VALU
  __builtin_amdgcn_sched_group_barrier(0x200, 8, 1);
  __builtin_amdgcn_sched_barrier(0);
  // ---- C
  auto dvdk = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
    for (int sk = 0; sk < 2; ++sk)
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        dv[kk][dh] = mfma(gt[sk][dh], pf[kk][sk], dv[kk][dh]);
        dk[kk][dh] = mfma(qt[sk][dh], df[kk][sk], dk[kk][dh]);
      }
  };
  dvdk(0);
  if constexpr (DQ) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) dq = mfma(ka[0][ks], sf[0][ks], dq);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      ka[1][ks] = frag_tr_sw(Kt, 16 * (kq0 + 4 + ks), 32 * dhw, lane);
      sf[1][ks] = frag_tr_sw(dsP, 16 * (kq0 + 4 + ks), 32 * qhw, lane);
    }
  }
  softmax(1);
  __builtin_amdgcn_sched_group_barrier(0x008, CB_LEAD, 2);  // as in B: half 1's S / dP complete first
#pragma unroll
  for (int g = 0; g < (DQ ? 12 : 8) - CB_LEAD; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, 6, 2);  // VALU
    if (DQ) __builtin_amdgcn_sched_group_barrier(0x100, 1, 2);  // DS read
    if (g & 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 2);  // DS write
  }
  __builtin_amdgcn_sched_group_barrier(0x002, 64, 2);
  __builtin_amdgcn_sched_group_barrier(0x100, 8, 2);
  __builtin_amdgcn_sched_group_barrier(0x200, 8, 2);
  __builtin_amdgcn_sched_barrier(0);
  // ---- D: the dQ k-steps (independent of softmax(1)) first, while its last bf16 operands settle
  if constexpr (DQ) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) dq = mfma(ka[1][ks], sf[1][ks], dq);
  }
  dvdk(1);
  if constexpr (NEXT) {
    op.load(Q_, G_, F_, 1, lane);
#pragma unroll
    for (int g = 0; g < 10; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 3);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 3);  // DS read
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int LAG>
__global__ __launch_bounds__(256, 1) void attn_bwd_chain2_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const bf16* __restrict__ qs,
                                                                 const bf16* __restrict__ frag,
                                                                 bf16* __restrict__ dqkv, float* chain,
                                                                 unsigned* flags, unsigned* err, int N, int H,
                                                                 int nkb, float scale, float dk_scale) {
  __shared__ __attribute__((aligned(1024))) char lds[CB2L_BYTES];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int w = xcd_work_item(blockIdx.x, gridDim.x);  // the key blocks of one (b, h): consecutive, one XCD
  const int bh = w / nkb, kb = w - bh * nkb, b = bh / H, hd = bh % H;
  const int nt = (N + 63) / 64;
  const int64_t ldt = (int64_t)3 * H * D, ldo = (int64_t)H * D;
  const bf16* base = qkv + (int64_t)b * N * ldt + hd * D;
  const unsigned tile_bytes = (unsigned)(64 * ldo * 2);
  bf16* const Kt = reinterpret_cast<bf16*>(lds + CB2L_K);
  {  // the block's 256 keys -> Kt: wave w loads its own 64 keys as 8 pieces of 8 rows; keys past N read zeros
    const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(base + H * D), 0, (int)(((int64_t)(N - 1) * ldt + 64) * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rl = 64 * wave + 8 * i + (lane >> 3);
      const unsigned vo = (unsigned)(((lane >> 3) * (int)ldt + ((lane & 7) ^ swz(rl)) * 8) * 2);
      lds_dma16(kr, Kt + (8 * wave + i) * 512, vo, (unsigned)((int64_t)(kb * CB2_K + 64 * wave + 8 * i) * ldt * 2));
    }
  }
  TileDMA qd, gd;
  FragDMA2 fd;
  qd.init(qs + (int64_t)b * N * ldo + hd * D, ldo, N, wave, lane);
  gd.init(dout + (int64_t)b * N * ldo + hd * D, ldo, N, wave, lane);
  fd.init(frag + (int64_t)bh * 2 * N * 8, N, wave);
  auto Qb = [&](int P) { return reinterpret_cast<bf16*>(lds + CB2L_Q + P * 8192); };
  auto Gb = [&](int P) { return reinterpret_cast<bf16*>(lds + CB2L_G + P * 8192); };
  auto Fb = [&](int P) { return reinterpret_cast<bf16*>(lds + CB2L_F + P * 2048); };
  auto Sb = [&](int P) { return reinterpret_cast<bf16*>(lds + CB2L_S + P * 32768); };
  const CbOrder<LAG> ord{nt, nkb, kb};
  int T = ord.first();     // the tile of the current step
  int Tp = 0, pp = 0;      // the previous step's tile and its chain position (its dQ link is due)
  qd.issue(Qb(0), (unsigned)T * tile_bytes, wave);
  gd.issue(Gb(0), (unsigned)T * tile_bytes, wave);
  fd.issue(Fb(0), (unsigned)T * 64u, wave, lane);
  bf16x8 vf[2][4];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int key = kb * CB2_K + 64 * wave + 32 * kk + (lane & 31);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      vf[kk][ks] = load_frag_global(base + (int64_t)key * ldt + 2 * H * D, ks, lane, key < N);
    settle(vf[kk]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // K and tile 0 in LDS
  const int dhw = wave & 1, qhw = wave >> 1;  // this wave's dQ^T sub-tile
  bf16x8 kf[2][4];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[kk][ks] = frag_row_sw(Kt, 64 * wave + 32 * kk + (lane & 31), ks, lane);
  const bf16x8 one = ones3(lane);
  f32x16 dk[2][2], dv[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) { dk[kk][dh] = zero16(); dv[kk][dh] = zero16(); }
  unsigned* const fl = flags + (int64_t)bh * nt * 4;
  const __amdgpu_buffer_rsrc_t flr = __builtin_amdgcn_make_buffer_rsrc((void*)fl, 0, nt * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(chain + (int64_t)bh * nt * (CB_TILE / 4)), 0, nt * CB_TILE, 0x00020000);
  const int last = nkb - 1;
  bool pub = false;  // a running sum stored this step: its flag goes out in the middle of the step
  int pub_T = 0;
  unsigned pub_val = 0;
  u32x4 run[4];      // the running sum of the previous step's tile (loaded in the middle of that step)
#ifdef CB_STAMP  // timing builds only (tools/attn_bwd_stamps.py): s_memtime per step segment
  unsigned long long* const stamps =
      reinterpret_cast<unsigned long long*>(chain + (int64_t)(gridDim.x / nkb) * nt * (CB_TILE / 4));
  unsigned long long ts[16] = {};
#define CB_TS(k) ts[k] = __builtin_amdgcn_s_memtime()
#else
#define CB_TS(k)
#endif
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // K fragments in registers before slot 1 is reused
  // dQ of the tile of step jp (image slot SP), its running sum added, handed on or written as bf16
  // dQ^T of the previous step's tile from dS^T image SP (16 MFMAs over the block's 256 keys)
  auto dq_mfma = [&](int SP) __attribute__((always_inline)) {
    const bf16* dsT = Sb(SP);
    f32x16 dq = zero16();
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // 8 k-steps' fragments requested, then their 8 MFMAs
      bf16x8 ka[8], sf[8];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        ka[ks] = frag_tr_sw(Kt, 16 * (8 * h + ks), 32 * dhw, lane);
        sf[ks] = frag_tr_sw(dsT, 16 * (8 * h + ks), 32 * qhw, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) dq = mfma(ka[ks], sf[ks], dq);
    }
    return dq;
  };
  // mid-step: the running-sum stores of the previous step are done (the tile DMA needs this wait anyway):
  // publish them; then the predecessor's running sum of tile Tp into registers
  auto link_fetch = [&](unsigned fv) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CB_TS(7);
    // the flag value into an SGPR BEFORE the publish store: vmcnt counts stores too, and a wait for the
    // flag load placed after the store would wait for the store's acknowledgement (~500 cycles a step)
    const unsigned fs = __builtin_amdgcn_readfirstlane(fv);
    asm volatile("; flag read" ::"s"(fs));
    if (pub && lane == 0) fb_st_flag(fl + pub_T * 4 + wave, pub_val);
    pub = false;
    CB_TS(8);
    if (pp > 0) {
      if (__builtin_expect(fs != (unsigned)pp, 0)) {
        CB_TS(10);
        cb_spin(fl + Tp * 4 + wave, (unsigned)pp, err);
      }
      CB_TS(9);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        run[g] = __builtin_amdgcn_raw_buffer_load_b128(cr, lane * 16, Tp * CB_TILE + wave * CB_SUB + g * 1024, 16);
    }
  };
  // tile Tp's dQ: its running sum added, handed on (published in the middle of the next step) or written
  auto link_store = [&](f32x16 dq) __attribute__((always_inline)) {
    if (pp > 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 r = __builtin_bit_cast(f32x4, run[g]);
#pragma unroll
        for (int i = 0; i < 4; ++i) dq[4 * g + i] += r[i];
      }
    }
    if (pp < last) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]}), cr, lane * 16,
            Tp * CB_TILE + wave * CB_SUB + g * 1024, 16);
      pub = true;
      pub_T = Tp;
      pub_val = (unsigned)(pp + 1);
    } else {
      const int q = Tp * 64 + 32 * qhw + (lane & 31);
      if (q < N) {
        bf16* qrow = dqkv + ((int64_t)b * N + q) * ldt + hd * D + 32 * dhw;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 8 * g4 + 4 * (lane >> 5);
          *reinterpret_cast<bf16x4*>(qrow + d0) =
              bf16x4{(bf16)(dq[4 * g4] * scale), (bf16)(dq[4 * g4 + 1] * scale), (bf16)(dq[4 * g4 + 2] * scale),
                     (bf16)(dq[4 * g4 + 3] * scale)};
        }
      }
    }
  };
  // step j on tile T (image slot P); HP: finish the previous tile's dQ (from slot P ^ 1) in the same step --
  // its MFMAs in the basic block of the first query half, its running sum fetched mid-step, its link after
  // the second half
  auto step = [&](int j, auto par, auto has_prev) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    constexpr bool HP = decltype(has_prev)::value;
    CB_TS(0);
    const int pos = ord.pos(T), T1 = ord.next(T);
    if (j + 1 < nt) {  // buffer P^1 was last read by step j - 1's body, before its barrier
      qd.issue(Qb(P ^ 1), (unsigned)T1 * tile_bytes, wave);
      gd.issue(Gb(P ^ 1), (unsigned)T1 * tile_bytes, wave);
      fd.issue(Fb(P ^ 1), (unsigned)T1 * 64u, wave, lane);
    }
    unsigned fv = 0;
    if (HP && pp > 0) fv = cb_load_flag(flr, (Tp * 4 + wave) * 4);  // Tp's predecessor (checked mid-step)
    f32x16 dq = zero16();  // the previous tile's dQ^T: k-steps 0-7 in this half, 8-15 in the next
    HalfOps op;
    cb2_half_staged<HP, false, CB_PREF>(dk, dv, dq, op, Qb(P), Gb(P), Fb(P), Sb(P), Kt, Sb(P ^ 1), 0, dhw, qhw, kf, vf,
                                     one, 0, wave, lane);
    CB_TS(1);
    if constexpr (HP) link_fetch(fv);
    else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile j + 1 landed
    }
    CB_TS(2);
    cb2_half_staged<HP, CB_PREF, false>(dk, dv, dq, op, Qb(P), Gb(P), Fb(P), Sb(P), Kt, Sb(P ^ 1), 8, dhw, qhw, kf, vf,
                                     one, 1, wave, lane);
    CB_TS(3);
    if constexpr (HP) link_store(dq);
    CB_TS(4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // dS^T written
    CB_TS(5);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#ifdef CB_STAMP
    CB_TS(6);
    if (w < 256 && lane == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) stamps[((int64_t)(w * 4 + wave) * 64 + j) * 16 + k] = ts[k];
#pragma unroll
      for (int k = 0; k < 16; ++k) ts[k] = 0;
    }
#endif
    Tp = T;
    pp = pos;
    T = T1;
  };
  {
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using F = std::false_type;
    using Tr = std::true_type;
    step(0, P0{}, F{});
    int j = 1;
    for (; j + 1 < nt; j += 2) {
      step(j, P1{}, Tr{});
      step(j + 1, P0{}, Tr{});
    }
    if (j < nt) step(j, P1{}, Tr{});
  }
  {  // the last tile's dQ
    const unsigned fv = pp > 0 ? cb_load_flag(flr, (Tp * 4 + wave) * 4) : 0u;
    const f32x16 dq = dq_mfma((nt - 1) & 1);
    link_fetch(fv);
    link_store(dq);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (pub && lane == 0) fb_st_flag(fl + pub_T * 4 + wave, pub_val);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int key = kb * CB2_K + 64 * wave + 32 * kk + (lane & 31);
    if (key >= N) continue;
    bf16* krow = dqkv + ((int64_t)b * N + key) * ldt + H * D + hd * D;
    bf16* vrow = krow + H * D;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 8 * g4 + 4 * (lane >> 5);
      bf16x4 a0, a1, c0, c1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a0[i] = (bf16)(dk[kk][0][4 * g4 + i] * dk_scale);
        a1[i] = (bf16)(dk[kk][1][4 * g4 + i] * dk_scale);
        c0[i] = (bf16)dv[kk][0][4 * g4 + i];
        c1[i] = (bf16)dv[kk][1][4 * g4 + i];
      }
      *reinterpret_cast<bf16x4*>(krow + d0) = a0;
      *reinterpret_cast<bf16x4*>(krow + 32 + d0) = a1;
      *reinterpret_cast<bf16x4*>(vrow + d0) = c0;
      *reinterpret_cast<bf16x4*>(vrow + 32 + d0) = c1;
    }
  }
}

}  // namespace


// ------------------------------------------------------------------------------ one-pass backward: host side
static int64_t cb_flags_bytes(int32_t B, int32_t N, int32_t H) {
  return (((int64_t)B * H * cdiv(N, 64) * 4 * 4) + 255) / 256 * 256;  // [B*H][nt][4 sub-tiles] u32
}
// the largest rotation lag (<= 3) that leaves >= 2 steps between consecutive contributions to every tile, else 1
static int cb_lag(int32_t N, int keys) {
  const int nt = (int)cdiv(N, 64), nkb = (int)cdiv(N, keys);
  if (nkb == 1) return 1;
  for (int L = 3; L >= 2; --L)
    if (nt - L * (nkb - 1) >= 2) return L;
  return 1;
}

extern "C" int64_t mia_attn_bwd_chain_bytes(int32_t B, int32_t N, int32_t H) {
#ifdef CB_STAMP
  return cb_flags_bytes(B, N, H) + (int64_t)B * H * cdiv(N, 64) * CB_TILE + 256 * 4 * 64 * 16 * 8;
#endif
  return cb_flags_bytes(B, N, H) + (int64_t)B * H * cdiv(N, 64) * CB_TILE;
}

extern "C" int mia_attn_bwd_onepass(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                                    void* saved, void* chain, uint32_t* err, int32_t B, int32_t N, int32_t H,
                                    float scale, int32_t q_ready, mia_stream_t stream) {
  MIA_CHECK_ARG(qkv && out && dout && lse && dqkv && saved && chain && err, "attn_bwd_onepass: null pointer");
  MIA_CHECK_ARG(B > 0 && N > 0 && H > 0 && (int64_t)B * H < 65536, "attn_bwd_onepass: bad shape");
  const int64_t rows = (int64_t)B * N * H;
  MIA_CHECK_ARG(rows * 8 < (1ll << 31), "attn_bwd_onepass: B*N*H too large");
  MIA_CHECK_ARG((int64_t)N * 3 * H * D * 2 < (1ll << 31), "attn_bwd_onepass: one sequence must span < 2 GiB");
  MIA_CHECK_ARG((int64_t)cdiv(N, 64) * CB_TILE < (1ll << 31), "attn_bwd_onepass: sequence too long");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(saved) | reinterpret_cast<uintptr_t>(chain)) & 255) == 0,
                "attn_bwd_onepass: saved / chain workspaces must be 256-B aligned");
  hipStream_t s = as_stream(stream);
  bf16* qs = (bf16*)saved;
  bf16* frag = qs + rows * D;
  // Q' (unless the forward wrote it) and the row-constant fragments -L2, -delta
  attn_bwd_prep_kernel<<<(unsigned)cdiv(rows * 8, 256), 256, 0, s>>>((const bf16*)qkv, (const bf16*)out,
                                                                     (const bf16*)dout, lse, qs, frag, B, N, H,
                                                                     scale * LOG2E, q_ready ? 0 : 1);
  MIA_LAUNCH_CHECK("attn_bwd_prep");
  unsigned* flags = reinterpret_cast<unsigned*>(chain);
  float* sums = reinterpret_cast<float*>(reinterpret_cast<char*>(chain) + cb_flags_bytes(B, N, H));
  hipError_t e = hipMemsetAsync(flags, 0, (size_t)cb_flags_bytes(B, N, H), s);
  if (e != hipSuccess) return mia::fail(-(int)e, "attn_bwd_onepass: memset: %s", hipGetErrorString(e));
  const int nkb = (int)cdiv(N, CB2_K), lag = cb_lag(N, CB2_K);
  MIA_CHECK_ARG((int64_t)nkb * B * H < (1ll << 31), "attn_bwd_onepass: grid too large");
  const dim3 grid((unsigned)(nkb * B * H));
  const float dks = 1.f / LOG2E;
#define CB_LAUNCH(KER, L) KER<L><<<grid, 256, 0, s>>>((const bf16*)qkv, (const bf16*)dout, qs, frag, (bf16*)dqkv, \
                                                    sums, flags, err, N, H, nkb, scale, dks)
  if (lag == 3) CB_LAUNCH(attn_bwd_chain2_kernel, 3);
  else if (lag == 2) CB_LAUNCH(attn_bwd_chain2_kernel, 2);
  else CB_LAUNCH(attn_bwd_chain2_kernel, 1);
#undef CB_LAUNCH
  MIA_LAUNCH_CHECK("attn_bwd_chain");
  return 0;
}
