// Dense bf16 GEMM, 256x256x64 tiles, 8 waves, LDS-DMA half-tile stream (gfx950).
// C = A . B^T for bf16 DENSE operands in any KC/RC layout combination: the AST linears (qkv, proj,
// fc1, fc2: fwd, dgrad, wgrad; reference ast.py + timm Block) and the EnvNet-v2 FC layers.
//
// Schedule.  The 256x256 block tile is computed as four 128x128 quadrants, one per PHASE:
//   P0 = A0 x B0, P1 = A0 x B1, P2 = A1 x B1, P3 = A1 x B0     (A0/A1, B0/B1 = 128-row halves)
// Every wave owns a 32x64 piece of each quadrant (8 waves = 4 (M) x 2 (N)), so its fragments are
// reused across phases: A0 is read (ds_read_b128) in P0 and kept for P1, B0 read in P0 and kept
// for P3, B1 read in P1 and kept for P2, A1 read in P2.  Each half-tile (128 x 64 bf16 = 16 KB) is
// therefore read from LDS in exactly one phase, which frees its slot early: the global->LDS
// stream (global_load_lds_dwordx4, 2 per wave per half-tile, one half-tile per phase, in the order
// A0(k) B0(k) B1(k) A1(k)) runs 7 half-tiles ahead of consumption in a 2 x 4-slot ring (128 KB),
// and before each phase only the half-tile that phase needs is waited for: a counted
// s_waitcnt vmcnt(10) leaves 5 half-tiles in flight across the raw s_barrier that ends the phase.
// Slot reuse (WAR): a slot is re-filled one phase after its only reading phase (whose ds_reads
// were retired by lgkmcnt(0) before that phase's MFMAs, and a barrier has passed since).
// LDS images are XOR-swizzled on the SOURCE address (lane-linear DMA destination) exactly as the
// 128x128 kernel's: KC rows permute 16-B chunks by (row & 7), RC k-rows permute 32-B blocks by
// (k & 3).  Blocks are remapped so neighbouring tiles share an XCD (bijective swizzle).
#include <stdlib.h>

#include "gemm_common.h"

namespace mgemm {
namespace {

constexpr int NT8 = 512;
constexpr int HT = 128 * 64 * 2;  // half-tile bytes
constexpr int AHEAD = 7;          // half-tiles issued ahead of the phase counter

typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;
typedef short s16x8 __attribute__((ext_vector_type(8)));

// One half-tile stream: 16 pieces of 1 KB (KC: 8 rows x 128 B; RC: 4 k-rows x 256 B); wave w
// issues pieces 2w and 2w+1.
template <int L>
struct HStream {
  const bf16* src[2];
  int64_t step;
  __device__ __forceinline__ void init(const bf16* base, int64_t ld, int64_t extent, int64_t r0, int64_t kbeg,
                                       int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = wave * 2 + i;
      if constexpr (L == MIA_LAYOUT_KC) {
        const int r = 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        int64_t row = r0 + r;
        if (row >= extent) row = extent - 1;
        src[i] = base + row * ld + kbeg + c * 8;
      } else {
        const int kr = 4 * j + (lane >> 4);
        const int p = lane & 15;
        const int c = 2 * ((p >> 1) ^ (kr & 3)) + (p & 1);
        int64_t col = r0 + c * 8;
        if (col + 8 > extent) col = extent - 8;
        src[i] = base + (kbeg + kr) * ld + col;
      }
    }
    step = L == MIA_LAYOUT_KC ? 64 : 64 * ld;
  }
  // K-tile k (clamped to the last one: the stream runs ahead past the end with harmless re-reads
  // into slots nothing reads any more, so the loop has no branch around its DMA)
  __device__ __forceinline__ void issue(char* slot, int wave, int k, int klast) {
    const int64_t off = (int64_t)(k < klast ? k : klast) * step;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((glb_vp)(src[i] + off), (lds_vp)(slot + (wave * 2 + i) * 1024), 16, 0, 0);
  }
};

// 32-row (KC) / 32-column (RC) operand fragment for k-slice ks (16 deep) of a half-tile image.
template <int L>
__device__ __forceinline__ bf16x8 hfrag(const char* tile, int rbase, int ks, int lane) {
  if constexpr (L == MIA_LAYOUT_KC) {
    const int rr = rbase + (lane & 31);
    const int c = 2 * ks + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(tile + rr * 128 + ((c ^ (rr & 7)) * 16));
  } else {
    const int i16 = lane & 15, gq = lane >> 4;
    const int col = rbase + 16 * (gq & 1) + 4 * (i16 & 3);
    const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
    const char* p0 = tile + kr * 256 + (((col >> 4) ^ (kr & 3)) * 32) + (col & 15) * 2;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * 256));
    const s16x8 cc = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, cc);
  }
}

// s_waitcnt through the builtin (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8]),
// not inline asm: the compiler's own waitcnt insertion then knows these counters were drained and
// does not add a conservative lgkmcnt(0) in front of the MFMAs.
constexpr int wc_vm(int n) { return (n & 0xF) | ((n >> 4) << 14) | 0x70 | 0xF00; }
constexpr int WC_LGKM0 = 0xC07F;
// Phase boundary: a raw s_barrier that the compiler may move neither memory operations nor MFMAs
// across (LDS-DMA completion is ordered only by the counted vmcnt placed before it).
__device__ __forceinline__ void phase_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int LA, int LB>
__global__ __launch_bounds__(NT8) void dgemm256_kernel(DArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[8 * HT];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int nwg = g.nbm * g.nbn;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int bm = g.nfast ? wgid / g.nbn : wgid % g.nbm;
  const int bn = g.nfast ? wgid % g.nbn : wgid / g.nbm;
  const int64_t m0 = (int64_t)bm * 256, n0 = (int64_t)bn * 256;
  const int z = blockIdx.y;
  const int64_t kbeg = (int64_t)z * g.kper;
  int64_t kend = kbeg + g.kper;
  if (kend > g.K) kend = g.K;
  const int nk = kend > kbeg ? (int)((kend - kbeg) / 64) : 0;

  // streams j = 0..3: A0, B0, B1, A1
  HStream<LA> sa0, sa1;
  HStream<LB> sb0, sb1;
  sa0.init(g.a, g.lda, g.M, m0, kbeg, wave, lane);
  sa1.init(g.a, g.lda, g.M, m0 + 128, kbeg, wave, lane);
  sb0.init(g.b, g.ldb, g.N, n0, kbeg, wave, lane);
  sb1.init(g.b, g.ldb, g.N, n0 + 128, kbeg, wave, lane);
  auto slot = [&](int h) __attribute__((always_inline)) { return smem + ((((h >> 2) & 1) * 4) + (h & 3)) * HT; };
  auto issue = [&](int h) __attribute__((always_inline)) {
    switch (h & 3) {  // h & 3 is a compile-time constant at every call site
      case 0: sa0.issue(slot(h), wave, h >> 2, nk - 1); break;
      case 1: sb0.issue(slot(h), wave, h >> 2, nk - 1); break;
      case 2: sb1.issue(slot(h), wave, h >> 2, nk - 1); break;
      default: sa1.issue(slot(h), wave, h >> 2, nk - 1); break;
    }
  };
  // Fragment reads run one phase ahead of their MFMAs (except B0, read at the start of P0):
  //   P0 reads B0(k) [used now] + B1(k) [P1];  P1 reads A1(k) [P2];  P2 reads A0(k+1) [P0 of k+1]
  // so before phase g2 the half-tiles up to need(g2) must have landed (P0: 4k+2, P1: 4k+3,
  // P2: 4k+4; P3 reads nothing).
  // Every phase issues exactly one half-tile (real or past-the-end), so the half-tiles issued after
  // the newest one a phase needs are always 4: a constant vmcnt(8).
  auto wait_for_phase = [&](int g2) __attribute__((always_inline)) {
    if ((g2 & 3) != 3) __builtin_amdgcn_s_waitcnt(wc_vm(8));
  };
  // retire this phase's prefetch reads after its MFMAs were issued (WAR against the DMA that
  // refills their slot in a later phase); the sched_barrier keeps the MFMAs ahead of the wait
  auto lds_done = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(WC_LGKM0);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[q][j][r] = 0.f;

  bf16x8 fa[4], fa2[4], fb0[2][4], fb1[2][4];
  if (nk > 0) {
#pragma unroll
    for (int h = 0; h < AHEAD; ++h) issue(h);
    __builtin_amdgcn_s_waitcnt(wc_vm(8));  // A0(0), B0(0), B1(0) landed (4 newer half-tiles in flight)
    phase_barrier();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fa[ks] = hfrag<LA>(slot(0), 32 * wm, ks, lane);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int g0 = 4 * kt;
    // ---- P0: A0 x B0
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) fb0[j][ks] = hfrag<LB>(slot(g0 + 1), 64 * wn + 32 * j, ks, lane);
    __builtin_amdgcn_sched_barrier(0);  // B0 reads first: the MFMAs below wait for them only
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) fb1[j][ks] = hfrag<LB>(slot(g0 + 2), 64 * wn + 32 * j, ks, lane);
    issue(g0 + 0 + AHEAD);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks], fb0[j][ks], acc[0][j], 0, 0, 0);
    lds_done();
    wait_for_phase(g0 + 1);
    phase_barrier();
    // ---- P1: A0 x B1
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fa2[ks] = hfrag<LA>(slot(g0 + 3), 32 * wm, ks, lane);
    issue(g0 + 1 + AHEAD);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks], fb1[j][ks], acc[1][j], 0, 0, 0);
    lds_done();
    wait_for_phase(g0 + 2);
    phase_barrier();
    // ---- P2: A1 x B1
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fa[ks] = hfrag<LA>(slot(g0 + 4), 32 * wm, ks, lane);  // A0(k+1) (junk past the end)
    issue(g0 + 2 + AHEAD);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa2[ks], fb1[j][ks], acc[2][j], 0, 0, 0);
    lds_done();
    phase_barrier();
    // ---- P3: A1 x B0 (registers only)
    issue(g0 + 3 + AHEAD);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[3][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa2[ks], fb0[j][ks], acc[3][j], 0, 0, 0);
    wait_for_phase(g0 + 4);
    phase_barrier();
  }
  __builtin_amdgcn_s_waitcnt(wc_vm(0));  // past-the-end DMA must land before the LDS is reused
  __syncthreads();

  // epilogue: each wave stages its own 32x32 tiles through a private LDS region
  float* stage = reinterpret_cast<float*>(smem) + wave * (32 * 33);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ah = (q == 0 || q == 1) ? 0 : 1, bh = (q == 0 || q == 3) ? 0 : 1;
#pragma unroll
      // wave-private region: the wave's own LDS accesses complete in order, no barrier needed
      for (int r = 0; r < 16; ++r)
        stage[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = acc[q][j][r];
      const int row = lane >> 1, c0 = (lane & 1) * 16;
      const int64_t m = m0 + 128 * ah + 32 * wm + row;
      const int64_t nb = n0 + 128 * bh + 64 * wn + 32 * j + c0;
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = stage[row * 33 + c0 + c];
      if (m < g.M && nb < g.N) {
        if (g.split > 1) {
          float* dst = g.ws + ((int64_t)z * g.M + m) * g.N + nb;
          if (nb + 16 <= g.N && (g.N & 3) == 0) {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
              reinterpret_cast<float4*>(dst)[qq] = make_float4(v[4 * qq], v[4 * qq + 1], v[4 * qq + 2], v[4 * qq + 3]);
          } else {
            for (int c = 0; c < 16; ++c)
              if (nb + c < g.N) dst[c] = v[c];
          }
        } else {
          epi_store16(g.e, m, nb, g.N, v);
        }
      }
    }
}

template <int LA, int LB>
hipError_t launch(const DArgs& d, hipStream_t s) {
  DArgs e = d;
  e.nbm = (int)cdiv(d.M, 256);
  e.nbn = (int)cdiv(d.N, 256);
  e.nfast = (d.split == 1 && e.nbn <= 16 && e.nbm >= 4 * e.nbn) ? 1 : 0;
  dim3 grid((unsigned)(e.nbm * e.nbn), (unsigned)d.split);
  dgemm256_kernel<LA, LB><<<grid, NT8, 0, s>>>(e);
  return hipGetLastError();
}

}  // namespace

bool dgemm256_pays(int64_t M, int64_t N, int /*split*/) {
  // Opt-in (MIA_DGEMM256=1): on the AST shapes (K = 768..3072, M = 105k tokens) this 1-block-per-CU
  // schedule measured 0.6-1.0x the 128x128 two-blocks-per-CU kernel, so it is not the
  // default.  Read per call so tests and A/B runs can switch it inside one process.
  const char* e = getenv("MIA_DGEMM256");
  if (!e || atoi(e) != 1) return false;
  return M >= 8 && N >= 8;
}

hipError_t dgemm256_launch(const DArgs& d, int la, int lb, hipStream_t s) {
  if (la == MIA_LAYOUT_KC && lb == MIA_LAYOUT_KC) return launch<MIA_LAYOUT_KC, MIA_LAYOUT_KC>(d, s);
  if (la == MIA_LAYOUT_KC) return launch<MIA_LAYOUT_KC, MIA_LAYOUT_RC>(d, s);
  if (lb == MIA_LAYOUT_KC) return launch<MIA_LAYOUT_RC, MIA_LAYOUT_KC>(d, s);
  return launch<MIA_LAYOUT_RC, MIA_LAYOUT_RC>(d, s);
}

}  // namespace mgemm
