// EnvNet-v2 trunk 1x2 convolutions (reference src/models/envnet_v2.py:38-49, blocks 3 and 4:
// Conv2d(c, c', (1, 2)) x 2 per block) -- weight gradient as ONE dense GEMM.
//
// For a (1, 2) kernel, stride 1, no padding, on an input of width W (output width W-1):
//   dW[co][kx][ci] = sum_{b,y,x<W-1} dY[b][y][x][co] * a[b][y][x+kx][ci]
//                  = sum_{input pixels q} Ashift[q][co*2 + kx] * a[q][ci]
// with Ashift[b][y][x][co*2 + kx] = dY[b][y][x-kx][co] (zero where x-kx is outside [0, W-1)).
// The forward over every input pixel q (the last column of each row is computed and dropped) is
//   y[q][co] = sum_{kx,ci} W[co][kx][ci] * a[q + kx][ci] = a_view[q][kx*Cin + ci] . W^T
// with a_view the map itself read with row stride Cin and row length 2 Cin (overlapping rows), and
// the input gradient is dX[q][ci] = sum_{co,kx} Ashift[q][co*2 + kx] * W[co][kx][ci]: all three
// are dense GEMMs on the LDS-DMA kernel.
// So the weight gradient is a plain (2 Cout) x Cin x (pixels) GEMM of two dense K-major operands,
// whose output rows (co*2 + kx) are already the OHWI gradient layout.  The two helpers below build
// Ashift (one pass over dY) and the BN+ReLU'd input a = bf16(relu(x*scale + shift)) (one pass over
// x) -- the same rounding as the pre-op the implicit GEMM applies while staging -- and the GEMM
// runs on the dense LDS-DMA kernel at MFMA rate instead of the gathered implicit GEMM.
#include "common.h"

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk(float lo, float hi) { return pk_bf16(lo, hi); }

// out = bf16(relu(x * scale + shift)), 8 channels per thread
__global__ __launch_bounds__(256) void bn_relu_apply_kernel(const bf16* __restrict__ x, int64_t P, int C,
                                                            const float* __restrict__ sc,
                                                            const float* __restrict__ sh, bf16* __restrict__ out) {
  const int G = C / 8;
  const int64_t total = P * G;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c0 = (int)(i % G) * 8;
    const u32x4 v = reinterpret_cast<const u32x4*>(x)[i];
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float lo = fmaxf(fmaf(__uint_as_float(v[q] << 16), sc[c0 + 2 * q], sh[c0 + 2 * q]), 0.f);
      const float hi = fmaxf(fmaf(__uint_as_float(v[q] & 0xffff0000u), sc[c0 + 2 * q + 1], sh[c0 + 2 * q + 1]), 0.f);
      o[q] = pk(lo, hi);
    }
    reinterpret_cast<u32x4*>(out)[i] = o;
  }
}

// Ashift[r][x][2c + kx] = dy[r][x - kx][c] for 0 <= x - kx < W - 1, else 0 (r = b*H + y).
// One thread: one (r, x) pixel and 8 channels -> 16 interleaved outputs (two 16-B stores).
__global__ __launch_bounds__(256) void shift_pad2_kernel(const bf16* __restrict__ dy, int64_t rows, int W, int C,
                                                         bf16* __restrict__ out) {
  const int G = C / 8, Wo = W - 1;
  const int64_t total = rows * W * G;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int g = (int)(i % G);
    const int64_t pix = i / G;
    const int x = (int)(pix % W);
    const int64_t r = pix / W;
    u32x4 d0 = {0u, 0u, 0u, 0u}, d1 = {0u, 0u, 0u, 0u};
    if (x < Wo) d0 = *reinterpret_cast<const u32x4*>(dy + ((r * Wo + x) * C + g * 8));
    if (x >= 1) d1 = *reinterpret_cast<const u32x4*>(dy + ((r * Wo + x - 1) * C + g * 8));
    // interleave: element c*2 + kx; channel pair (2q, 2q+1) of d0/d1 -> four bf16
    u32x4 o0, o1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t a = d0[q], b = d1[q];
      const uint32_t lo = (a & 0xffffu) | (b << 16);          // c = 2q:   kx 0, kx 1
      const uint32_t hi = (a >> 16) | (b & 0xffff0000u);      // c = 2q+1: kx 0, kx 1
      if (q < 2) { o0[2 * q] = lo; o0[2 * q + 1] = hi; }
      else { o1[2 * (q - 2)] = lo; o1[2 * (q - 2) + 1] = hi; }
    }
    bf16* dst = out + pix * 2 * C + g * 16;
    reinterpret_cast<u32x4*>(dst)[0] = o0;
    reinterpret_cast<u32x4*>(dst)[1] = o1;
  }
}

// dst = [one zero pixel] + dy re-laid on the input grid: dst[1 + r*w + x] = dy[r*(w-1) + x] for x < w-1, zero
// at x = w-1 (one 16-B piece per thread); the optional `zp` (zc bf16) is zeroed too -- the pad pixel after the
// forward input, which the weight-gradient view reads against a zero gradient and so must be finite
__global__ __launch_bounds__(256) void pad_w2_kernel(const u32x4* __restrict__ dy, int64_t rows, int w, int c16,
                                                     u32x4* __restrict__ dst, u32x4* __restrict__ zp, int zc16) {
  const int64_t total = (1 + rows * w) * c16;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / c16;
    const int k = (int)(i - pix * c16);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (pix > 0) {
      const int64_t q = pix - 1, r = q / w;
      const int x = (int)(q - r * w);
      if (x < w - 1) v = dy[(r * (w - 1) + x) * c16 + k];
    }
    dst[i] = v;
    if (zp && i < zc16) zp[i] = u32x4{0u, 0u, 0u, 0u};
  }
}

// dst[r][x] = src[r][x] for x < w-1 (drops the padded last column of a (1, 2)-conv forward
// computed over every input pixel), 16 B per thread
__global__ __launch_bounds__(256) void drop_last_col_kernel(const u32x4* __restrict__ src, int64_t rows, int w,
                                                            int c16, u32x4* __restrict__ dst) {
  const int64_t total = rows * (w - 1) * c16;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t pix = i / c16;
    const int k = (int)(i - pix * c16);
    const int64_t r = pix / (w - 1);
    const int x = (int)(pix - r * (w - 1));
    dst[i] = src[(r * w + x) * c16 + k];
  }
}

int grid_for(int64_t work) {
  const int64_t b = (work + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int mia_bn_relu_apply(const void* x, int64_t P, int32_t C, const float* scale, const float* shift,
                                 void* out, mia_stream_t stream) {
  MIA_CHECK_ARG(x && scale && shift && out && P > 0 && C > 0 && C % 8 == 0, "bn_relu_apply: bad arguments");
  MIA_CHECK_ARG(al16(x) && al16(out), "bn_relu_apply: x / out must be 16-byte aligned");
  bn_relu_apply_kernel<<<grid_for(P * (C / 8)), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const bf16*>(x), P, C, scale, shift, reinterpret_cast<bf16*>(out));
  MIA_LAUNCH_CHECK("bn_relu_apply");
  return 0;
}

extern "C" int mia_shift_pad_w2(const void* dy, int64_t rows, int32_t w, int32_t c, void* out, mia_stream_t stream) {
  MIA_CHECK_ARG(dy && out && rows > 0 && w >= 2 && c > 0 && c % 8 == 0, "shift_pad_w2: bad arguments");
  MIA_CHECK_ARG(al16(dy) && al16(out), "shift_pad_w2: dy / out must be 16-byte aligned");
  shift_pad2_kernel<<<grid_for(rows * w * (c / 8)), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const bf16*>(dy), rows, w, c, reinterpret_cast<bf16*>(out));
  MIA_LAUNCH_CHECK("shift_pad_w2");
  return 0;
}

extern "C" int mia_pad_w2(const void* dy, int64_t rows, int32_t w, int32_t c, void* dst, void* zero_pixel,
                          int32_t zc, mia_stream_t stream) {
  MIA_CHECK_ARG(dy && dst && rows > 0 && w >= 2 && c > 0 && c % 8 == 0 && zc % 8 == 0 && (zc == 0 || zero_pixel),
                "pad_w2: bad arguments");
  MIA_CHECK_ARG(al16(dy) && al16(dst) && (!zero_pixel || al16(zero_pixel)), "pad_w2: 16-byte aligned pointers");
  pad_w2_kernel<<<grid_for((1 + rows * w) * (c / 8)), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const u32x4*>(dy), rows, w, c / 8, reinterpret_cast<u32x4*>(dst),
      reinterpret_cast<u32x4*>(zero_pixel), zc / 8);
  MIA_LAUNCH_CHECK("pad_w2");
  return 0;
}

extern "C" int mia_drop_last_col(const void* src, int64_t rows, int32_t w, int32_t c, void* dst, mia_stream_t stream) {
  MIA_CHECK_ARG(src && dst && rows > 0 && w >= 2 && c > 0 && c % 8 == 0, "drop_last_col: bad arguments");
  MIA_CHECK_ARG(al16(src) && al16(dst), "drop_last_col: src / dst must be 16-byte aligned");
  drop_last_col_kernel<<<grid_for(rows * (w - 1) * (c / 8)), 256, 0, as_stream(stream)>>>(
      reinterpret_cast<const u32x4*>(src), rows, w, c / 8, reinterpret_cast<u32x4*>(dst));
  MIA_LAUNCH_CHECK("drop_last_col");
  return 0;
}
