// Backward-data of the single-input-channel 8x8 conv (EnvNet-v2 trunk conv3, reference
// src/models/envnet_v2.py:31 Conv2d(1, 32, (8, 8))), bf16 MFMA, gfx950.
//
//   dx[b][y][x] = sum_{ky,kx,co} dy[b][y-ky][x-kx][co] * w[co][0][ky][kx]
//
// With one input channel the contraction has no output-channel axis to put on the MFMA N side, so
// the kernel puts the kernel row ky there instead: for one staged dY row r,
//   Q_r[x][ky] = sum_{kx,co} dy[b][r][x-kx][co] * w[co][ky][kx]        (M = x, N = ky, K = (kx, co) = 256)
// and dx[b][r+ky][x] += Q_r[x][ky].  A block owns one clip and 128 output columns and sweeps every
// dY row once (each dY byte is read from HBM once); the 64 output rows x 128 columns accumulate in
// LDS (f32, one writer per address, program order => deterministic; rows 129 floats apart so a dY row's
// scatter into its 8 output rows is conflict-free: at 128 it was 8-way, 0.48 of the kernel's LDS cycles
// in SQ_LDS_BANK_CONFLICT) and are stored once as bf16.
// dY rows are register-staged two rows ahead (issue early, write late) into a 2-deep LDS ring whose
// pixel stride (80 B) makes every 16-lane ds_read_b128 group conflict-free.  N = 8 of the MFMA's 32
// columns carry data: the op is 58 GFLOP/step of real work, HBM-bound on the dY read either way.
#include "common.h"

namespace {

constexpr int C1_C = 32, C1_K = 8;
constexpr int C1_BW = 128;                 // output columns per block
constexpr int C1_SLOTS = C1_BW + C1_K - 1; // staged dY pixels per row
constexpr int C1_PSB = 80;                 // LDS bytes per staged pixel (64 B data + 16 B skew)
constexpr int C1_HMAX = 64;                // output rows held in LDS
// output row stride in LDS: 129 floats, so the 8 kernel rows ky a dY row scatters into (lanes 0-7 of a
// half wave, same column) fall on 8 different banks (a 128-float stride put all 8 on one bank: 8-way)
constexpr int C1_OLD = C1_BW + 1;
constexpr int C1_LD = (C1_SLOTS * 4 + 255) / 256;  // 16-B chunks per thread per row (3)

struct C1Args {
  const bf16* dy;
  const float* w;
  bf16* dx;
  int n, oh, ow, h, wd, nchunk;
};

__global__ __launch_bounds__(256) void conv1ch_dgrad_kernel(C1Args g) {
  __shared__ __attribute__((aligned(16))) char rows[2][C1_SLOTS * C1_PSB];
  __shared__ __attribute__((aligned(16))) float outs[C1_HMAX * C1_OLD];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / g.nchunk;
  const int w0 = (blockIdx.x - b * g.nchunk) * C1_BW;

  for (int i = t; i < C1_HMAX * C1_OLD; i += 256) outs[i] = 0.f;

  // B fragments (whole K = 256 in registers): lane column n = ky, k = 16 ks + 8 (lane >> 5) + j
  // with kx = ks >> 1, co = 16 (ks & 1) + 8 (lane >> 5) + j.
  bf16x8 bw[16];
  const int ky = lane & 31;
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int kx = ks >> 1, co0 = 16 * (ks & 1) + 8 * (lane >> 5);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      bw[ks][j] = ky < C1_K ? (bf16)g.w[((co0 + j) * C1_K + ky) * C1_K + kx] : (bf16)0.f;
  }

  // thread slot q -> (staged pixel s, 16-B chunk c): each 8-lane group of a ds_write_b128 takes the 4
  // chunks of pixels p and p + 4 (80 B x 4 = 320 B = 16 banks apart: conflict-free; pixels p, p + 1 were
  // 2-way), a wave still loads 16 consecutive pixels
  auto slot_of = [](int q, int& s, int& c) __attribute__((always_inline)) {
    const int gq = q >> 3, j = q & 7;
    s = (gq >> 2) * 8 + (gq & 3) + 4 * (j >> 2);
    c = j & 3;
  };
  const bf16* dyb = g.dy + (int64_t)b * g.oh * g.ow * C1_C;
  auto load_row = [&](int r, uint4 (&reg)[C1_LD]) __attribute__((always_inline)) {
    const bf16* src = dyb + (int64_t)r * g.ow * C1_C;
#pragma unroll
    for (int i = 0; i < C1_LD; ++i) {
      int s, c;
      slot_of(t + 256 * i, s, c);
      const int px = w0 - (C1_K - 1) + s;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < g.oh && s < C1_SLOTS && px >= 0 && px < g.ow)
        v = *reinterpret_cast<const uint4*>(src + px * C1_C + c * 8);
      reg[i] = v;
    }
  };
  auto store_row = [&](char* dst, const uint4 (&reg)[C1_LD]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < C1_LD; ++i) {
      int s, c;
      slot_of(t + 256 * i, s, c);
      if (s < C1_SLOTS) *reinterpret_cast<uint4*>(dst + s * C1_PSB + c * 16) = reg[i];
    }
  };
  const int m = lane & 31, half = lane >> 5;
  // one dY row: MFMAs on the staged row r, then scatter Q_r into the LDS output rows r..r+7
  auto compute_row = [&](int r) __attribute__((always_inline)) {
    const char* cur = rows[r & 1];
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int slot = 32 * wave + m - (ks >> 1) + (C1_K - 1);
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(cur + slot * C1_PSB + (16 * (ks & 1) + 8 * half) * 2);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bw[ks], acc, 0, 0, 0);
    }
    if (ky < C1_K) {
      float* o = outs + (r + ky) * C1_OLD + 32 * wave + 4 * half;
#pragma unroll
      for (int i = 0; i < 16; ++i) o[(i & 3) + 8 * (i >> 2)] += acc[i];
    }
  };

  // rows are loaded two ahead into alternating register sets (the HBM latency spans two rows of
  // MFMA work) and written to the LDS ring one row ahead
  uint4 ra[C1_LD], rb[C1_LD];
  load_row(0, ra);
  load_row(1, rb);
  store_row(rows[0], ra);
  __syncthreads();
  for (int r = 0; r < g.oh; r += 2) {
    load_row(r + 2, ra);
    compute_row(r);
    store_row(rows[(r + 1) & 1], rb);
    __syncthreads();
    if (r + 1 >= g.oh) break;
    load_row(r + 3, rb);
    compute_row(r + 1);
    store_row(rows[r & 1], ra);
    __syncthreads();
  }

  // store rows of 128 columns as bf16, 4 columns (8 B) per thread-step
  bf16* dxb = g.dx + (int64_t)b * g.h * g.wd;
  for (int q = t; q < g.h * (C1_BW / 4); q += 256) {
    const int y = q / (C1_BW / 4), x4 = (q - y * (C1_BW / 4)) * 4;
    const int x = w0 + x4;
    if (x >= g.wd) continue;
    const float* o = outs + y * C1_OLD + x4;
    if (x + 4 <= g.wd) {
      bf16x4 v = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      *reinterpret_cast<bf16x4*>(dxb + (int64_t)y * g.wd + x) = v;
    } else {
      for (int i = 0; x + i < g.wd; ++i) dxb[(int64_t)y * g.wd + x + i] = (bf16)o[i];
    }
  }
}

}  // namespace

extern "C" int mia_conv1ch_dgrad(const void* dy, const float* w, void* dx, int32_t n, int32_t oh, int32_t ow,
                                 mia_stream_t stream) {
  MIA_CHECK_ARG(dy && w && dx && n > 0 && oh > 0 && ow > 0, "conv1ch_dgrad: bad arguments");
  const int h = oh + C1_K - 1, wd = ow + C1_K - 1;
  MIA_CHECK_ARG(h <= C1_HMAX, "conv1ch_dgrad: at most %d output rows (got %d)", C1_HMAX, h);
  MIA_CHECK_ARG(wd % 4 == 0, "conv1ch_dgrad: output width must be a multiple of 4 (got %d)", wd);
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dx)) % 16 == 0,
                "conv1ch_dgrad: dy/dx must be 16-byte aligned");
  MIA_CHECK_ARG((int64_t)oh * ow * C1_C < (1ll << 31), "conv1ch_dgrad: clip too large for 32-bit indexing");
  C1Args a{reinterpret_cast<const bf16*>(dy), w, reinterpret_cast<bf16*>(dx), n, oh, ow, h, wd,
           (int)cdiv(wd, C1_BW)};
  const int64_t blocks = (int64_t)n * a.nchunk;
  MIA_CHECK_ARG(blocks < (1ll << 31), "conv1ch_dgrad: grid too large");
  conv1ch_dgrad_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(a);
  MIA_LAUNCH_CHECK("conv1ch_dgrad");
  return 0;
}
