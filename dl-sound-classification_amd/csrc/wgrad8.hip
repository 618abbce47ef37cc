// Weight gradient of the EnvNet-v2 trunk 8x8 conv (reference src/models/envnet_v2.py:34
// Conv2d(32, 32, (8, 8)), input = relu(bn(previous conv)) ), bf16 MFMA, gfx950.
//
//   dW[co][ky][kx][ci] = sum_{b, oy, ox} dY[b][oy][ox][co] * relu(bn(x))[b][oy+ky][ox+kx][ci]
//
// Rolling-window schedule: a block owns (clip, 128-column chunk) items and walks the output rows
// of an item top to bottom.  The 8 input rows an output row needs stay in a 9-slot LDS ring, so
// every input row is staged (and BN+ReLU'd) ONCE per item instead of once per kernel row, and
// every dY row once: HBM reads ~ x + dY instead of ~8x + 2 dY for a ky-partitioned grid.
// Wave w owns kernel row ky = w: its 8 accumulator tiles are dW[:, w, kx, :] (32 co x 32 ci) for
// kx = 0..7 (128 registers), kept across all items; each block writes one f32 slab and the
// split-K reducer sums the slabs.  Operands are transposed LDS reads (ds_read_b64_tr_b16) of the
// [px][32 ch] images, exactly as the row-window wgrad kernel.  Rows for step s+1 are loaded raw
// into registers while step s computes (issue early, convert + write late).
#include "gemm_common.h"

namespace mgemm {
namespace {

constexpr int W8_NT = 512;
constexpr int W8_BP = 128;                  // output columns per item
constexpr int W8_WPX = W8_BP + 7;           // staged input columns
constexpr int W8_XROW = W8_WPX * 64;        // bytes per staged input row (32 ch bf16)
constexpr int W8_RING = 9;                  // 8 rows in use + the one being written
constexpr int W8_DROW = W8_BP * 64;         // bytes per staged dY row
constexpr int W8_XCH = (W8_WPX * 4 + W8_NT - 1) / W8_NT;  // 16-B chunks per thread per input row (2)

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 tr_frag(const char* p0, int stride) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MIA_LDS s16x4*)(p0 + 4 * stride));
  const s16x8 c = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, c);
}

__device__ __forceinline__ u32x4 bn_relu_pack(u32x4 u, bool ok, const float* sc, const float* sh) {
  if (!ok) return u32x4{0u, 0u, 0u, 0u};
  uint32_t w4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = fmaxf(fmaf(__uint_as_float(u[i] << 16), sc[2 * i], sh[2 * i]), 0.f);
    const float hi = fmaxf(fmaf(__uint_as_float(u[i] & 0xffff0000u), sc[2 * i + 1], sh[2 * i + 1]), 0.f);
    w4[i] = pk_bf16(lo, hi);
  }
  return u32x4{w4[0], w4[1], w4[2], w4[3]};
}

__global__ __launch_bounds__(W8_NT) void wgrad8_kernel(W8Args g) {
  __shared__ __attribute__((aligned(16))) char smem[W8_RING * W8_XROW + 2 * W8_DROW];
  char* ring = smem;
  char* dys = smem + W8_RING * W8_XROW;
  const int t = threadIdx.x, lane = t & 63;
  const int ky = __builtin_amdgcn_readfirstlane(t >> 6);
  const int i16 = lane & 15, gq = lane >> 4;
  const int cg = t & 3;  // this thread's 8-channel group in every staged 16-B chunk
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sc[i] = g.ps[cg * 8 + i]; sh[i] = g.pt[cg * 8 + i]; }

  f32x16 acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;

  const int nchunk = (g.ow + W8_BP - 1) / W8_BP;
  const int items = g.n * nchunk;
  u32x4 xr[W8_XCH], dr;
  uint32_t xok = 0;
  bool dok = false;
  const u32x4* xs = reinterpret_cast<const u32x4*>(g.x);
  const u32x4* ds = reinterpret_cast<const u32x4*>(g.dy);

  for (int item = blockIdx.x; item < items; item += gridDim.x) {
    const int b = item / nchunk;
    const int x0 = (item - b * nchunk) * W8_BP;
    // raw loads of input row iy / dY row oy (16-B chunk = 8 channels), unconditional addresses
    auto load_x = [&](int iy) __attribute__((always_inline)) {
      xok = 0;
#pragma unroll
      for (int i = 0; i < W8_XCH; ++i) {
        const int q = t + W8_NT * i;
        const int px = x0 + (q >> 2);
        const bool ok = (q >> 2) < W8_WPX && px < g.w && iy < g.h;
        const int64_t off = ok ? ((((int64_t)b * g.h + iy) * g.w + px) * 4 + (q & 3)) : 0;
        xr[i] = xs[off];
        xok |= (uint32_t)ok << i;
      }
    };
    auto load_dy = [&](int oy) __attribute__((always_inline)) {
      const int px = x0 + (t >> 2);
      dok = oy >= 0 && oy < g.oh && px < g.ow;
      const int64_t off = dok ? ((((int64_t)b * g.oh + oy) * g.ow + px) * 4 + (t & 3)) : 0;
      dr = ds[off];
    };
    auto store_x = [&](int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < W8_XCH; ++i) {
        const int q = t + W8_NT * i;
        if ((q >> 2) < W8_WPX)
          *reinterpret_cast<u32x4*>(ring + slot * W8_XROW + q * 16) = bn_relu_pack(xr[i], (xok >> i) & 1u, sc, sh);
      }
    };
    auto store_dy = [&](int buf) __attribute__((always_inline)) {
      *reinterpret_cast<u32x4*>(dys + buf * W8_DROW + t * 16) = dok ? dr : u32x4{0u, 0u, 0u, 0u};
    };

    load_x(0);
    store_x(0);
    __syncthreads();
    for (int s = 0; s < g.h; ++s) {
      // stage s+1 in flight while step s computes
      load_x(s + 1);
      load_dy(s - 6);
      const int oy = s - 7;
      if (oy >= 0) {
        const char* xrow = ring + ((oy + ky) % W8_RING) * W8_XROW;
        const char* drow = dys + (oy & 1) * W8_DROW;
#pragma unroll
        for (int ks = 0; ks < W8_BP / 16; ++ks) {
          const int kr = ks * 16 + 8 * (gq >> 1) + (i16 >> 2);
          const int c4 = 16 * (gq & 1) + 4 * (i16 & 3);
          const bf16x8 fa = tr_frag(drow + kr * 64 + c4 * 2, 64);
#pragma unroll
          for (int kx = 0; kx < 8; ++kx) {
            const bf16x8 fb = tr_frag(xrow + (kr + kx) * 64 + c4 * 2, 64);
            acc[kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[kx], 0, 0, 0);
          }
        }
      }
      if (s + 1 < g.h) store_x((s + 1) % W8_RING);
      if (s - 6 >= 0 && s - 6 < g.oh) store_dy((s - 6) & 1);
      __syncthreads();
    }
  }

  // slab: ws[block][co][ky*256 + kx*32 + ci]
  float* dst = g.ws + (int64_t)blockIdx.x * 32 * 2048 + ky * 256;
#pragma unroll
  for (int kx = 0; kx < 8; ++kx)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      dst[(int64_t)co * 2048 + kx * 32 + (lane & 31)] = acc[kx][r];
    }
}

}  // namespace

hipError_t wgrad8_launch(const W8Args& a, hipStream_t s) {
  wgrad8_kernel<<<a.nblk, W8_NT, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace mgemm
