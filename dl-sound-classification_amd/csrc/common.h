// Shared device/host helpers for libmiaudio (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>

#include "../../include/miaudio.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2_cvt __attribute__((ext_vector_type(2)));

// two floats -> two bf16 (round to nearest even, as the (bf16) cast) packed lo | hi << 16: one v_cvt_pk_bf16_f32
// (the two casts and the shift-or were four VALU instructions)
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_cvt{lo, hi}, bf16x2));
}
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define MIA_LDS __attribute__((address_space(3)))

// ---------------------------------------------------------------- error handling
namespace mia {
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int cu_count();  // compute units of the current device (cached; 256 on MI355X)
}  // namespace mia

#define MIA_CHECK_ARG(cond, ...)                       \
  do {                                                 \
    if (!(cond)) return mia::fail(-22, __VA_ARGS__);   \
  } while (0)

#define MIA_LAUNCH_CHECK(what)                                                   \
  do {                                                                           \
    hipError_t e__ = hipGetLastError();                                          \
    if (e__ != hipSuccess)                                                       \
      return mia::fail(-(int)e__, "%s: launch failed: %s", what, hipGetErrorString(e__)); \
  } while (0)

static inline hipStream_t as_stream(mia_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// Lanes of ONE wave exchanging data through LDS with no s_barrier.  The hardware runs a wave's LDS
// instructions in order, but the compiler reasons per lane: another lane's store is a data race to
// it, so without this fence it may reuse a load from the previous iteration or move loads/stores
// across the exchange (seen: eval-mode fe_conv3 read stale B fragments in its second pipeline half).
// Place it between the writes and the other lanes' reads, and between those reads and the next writes.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <typename T> __device__ __forceinline__ float to_f(T x);
template <> __device__ __forceinline__ float to_f<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f<bf16>(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// dtype-dispatched scalar load/store on raw pointers
__device__ __forceinline__ float ld_elem(const void* p, int dtype, int64_t i) {
  return dtype == MIA_F32 ? ((const float*)p)[i] : (float)((const bf16*)p)[i];
}
__device__ __forceinline__ void st_elem(void* p, int dtype, int64_t i, float v) {
  if (dtype == MIA_F32) ((float*)p)[i] = v;
  else ((bf16*)p)[i] = (bf16)v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// LDS-only workgroup barrier: this wave's LDS operations complete, then s_barrier; the "memory" clobber keeps the
// compiler from moving memory operations across it, and no vmcnt wait is implied (global loads / stores and LDS-DMA
// stay in flight, unlike __syncthreads)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Deterministic block-wide sum (blockDim.x == 256) of p[k * stride] over k < n, in double.
// Fixed per-thread strided order + fixed tree: bit-identical across runs.
__device__ __forceinline__ double block_sum_strided(const float* __restrict__ p, int n, int64_t stride) {
  __shared__ double red_bss[256];
  double s = 0.0;
  for (int k = threadIdx.x; k < n; k += 256) s += (double)p[(int64_t)k * stride];
  red_bss[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red_bss[threadIdx.x] += red_bss[threadIdx.x + w];
    __syncthreads();
  }
  const double r = red_bss[0];
  __syncthreads();
  return r;
}

// Coalesced deterministic column sums of a row-major f32 matrix p[rows][cols] (ld = row stride),
// the per-block partial rows of the fixed-order reductions: pass 1, block (x, y) = 64 columns of
// row slice y; its 4 waves sum rows g, g + 4, ... of the slice (lane = column, 256-B row segments,
// in double) and are combined in a fixed order -> part2[y][cols]; colsum_slices() then adds the
// slices in order.  Replaces one-column-per-block strided walks (one 4-B read per line).
constexpr int COLSUM_SLICES = 16;
inline int64_t colsum_part2_bytes(int cols) { return (int64_t)COLSUM_SLICES * cols * 8; }
static __global__ __launch_bounds__(256) void colsum_pass1_kernel(const float* __restrict__ p, int64_t rows, int cols,
                                                                  int64_t ld, double* __restrict__ part2) {
  __shared__ double red_cp[4][64];
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l;
  const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = r0 + per < rows ? r0 + per : rows;
  double s = 0.0;
  if (c < cols) {
#pragma unroll 8
    for (int64_t r = r0 + g; r < r1; r += 4) s += (double)p[r * ld + c];
  }
  red_cp[g][l] = s;
  __syncthreads();
  if (g == 0 && c < cols)
    part2[(int64_t)blockIdx.y * cols + c] = ((red_cp[0][l] + red_cp[1][l]) + red_cp[2][l]) + red_cp[3][l];
}
inline void colsum_pass1(const float* p, int64_t rows, int cols, int64_t ld, double* part2, hipStream_t s) {
  colsum_pass1_kernel<<<dim3((unsigned)((cols + 63) / 64), COLSUM_SLICES), 256, 0, s>>>(p, rows, cols, ld, part2);
}
__device__ __forceinline__ double colsum_slices(const double* __restrict__ part2, int cols, int c) {
  double v = 0.0;
#pragma unroll
  for (int y = 0; y < COLSUM_SLICES; ++y) v += part2[(int64_t)y * cols + c];
  return v;
}

// ---------------------------------------------------------------- OCP MX-fp8 (see mia_mx_quantize)
// shared exponent of a 32-element block from its amax: floor(log2(amax)) - 8 (e4m3 emax), clamped to
// [-127, 127]; a zero / subnormal amax takes -127 (scale byte 0)
__device__ __forceinline__ int mx_exponent(float amax) {
  const int be = (int)((__float_as_uint(amax) >> 23) & 0xff);
  const int e = be == 0 ? -127 : be - 127 - 8;
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}
// 8 values -> 8 e4m3fn bytes of x * 2^-e (v_ldexp_f32: exact, subnormal results included), saturated
// to +-448 (v_med3_f32), round-to-nearest-even (v_cvt_pk_fp8_f32, OCP format on gfx950)
__device__ __forceinline__ uint2 mx_pack8(const float* v, int e) {
  float y[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) y[k] = __builtin_amdgcn_fmed3f(__builtin_amdgcn_ldexpf(v[k], -e), -448.f, 448.f);
  int p0 = 0, p1 = 0;
  p0 = __builtin_amdgcn_cvt_pk_fp8_f32(y[0], y[1], p0, false);
  p0 = __builtin_amdgcn_cvt_pk_fp8_f32(y[2], y[3], p0, true);
  p1 = __builtin_amdgcn_cvt_pk_fp8_f32(y[4], y[5], p1, false);
  p1 = __builtin_amdgcn_cvt_pk_fp8_f32(y[6], y[7], p1, true);
  return make_uint2((uint32_t)p0, (uint32_t)p1);
}
// 8 consecutive values held by each of 4 adjacent lanes (lane & 3 = quarter of the block): the block's
// exponent from the 4 lanes' amax (every lane of the wave must execute this)
// (the exchanges are DPP quad permutations -- lane ^ 1, lane ^ 2 inside each group of 4 -- VALU moves instead
// of the two LDS-crossbar ds_bpermute round trips __shfl_xor compiles to)
__device__ __forceinline__ int mx_exponent_4lanes(const float* v) {
  float am = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) am = fmaxf(am, fabsf(v[k]));
  constexpr int XOR1 = 1 | (0 << 2) | (3 << 4) | (2 << 6);  // quad_perm [1, 0, 3, 2]
  constexpr int XOR2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // quad_perm [2, 3, 0, 1]
#ifdef MIA_MX_SHFL  // A/B build: the ds_bpermute form
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
#else
  am = fmaxf(am, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(am), XOR1, 0xf, 0xf, false)));
  am = fmaxf(am, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(am), XOR2, 0xf, 0xf, false)));
#endif
  return mx_exponent(am);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// splitmix64 counter hash -> uniform [0,1) (dropout masks; same recipe as oracle/synth.py)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float hash_u01(uint64_t seed, uint64_t idx) {
  uint64_t z = splitmix64(idx ^ (seed * 0xD1B54A32D192ED03ull));
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// 8 consecutive elements (16 B bf16 / 32 B f32, aligned) <-> 8 floats
__device__ __forceinline__ void load8(const void* p, int dtype, int64_t off, float (&f)[8]) {
  if (dtype == MIA_BF16) {
    uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p) + off);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    const float4* q = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + off);
    float4 a = q[0], b = q[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
}
__device__ __forceinline__ void store8(void* p, int dtype, int64_t off, const float (&f)[8]) {
  if (dtype == MIA_BF16) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = pk_bf16(f[2 * i], f[2 * i + 1]);
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p) + off) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float4* q = reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + off);
    q[0] = make_float4(f[0], f[1], f[2], f[3]);
    q[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
}

