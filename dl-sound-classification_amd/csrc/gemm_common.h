// Shared pieces of the GEMM kernels (gemm.hip and its callers): the epilogue descriptor and its
// vectorised store path, and the dense bf16 GEMM argument block.
#pragma once
#include "common.h"

namespace mgemm {

struct EpiDev {
  char* ptr;
  int dtype, act, accumulate, aux_dtype;
  int64_t ldc, rm_inner, rm_outer, rm_istride, rm_offset;
  const float* bias;
  const char* aux;
  int64_t ldaux;
  float alpha, act_scale;
  double* sqsum;  // per-tile sum of squares of the stored output (see MiaEpilogue), or null
};

struct DArgs {
  const bf16* a;
  const bf16* b;
  int64_t lda, ldb, M, N, K, kper;
  int split, nbm, nbn;
  int nfast;  // 1: tall GEMM (AST linears: M = tokens, few column tiles): grouped tile order, see gm
  int gm;     // row blocks per group in the grouped order: within a group the column tiles are walked
              // slowest, so the group's A rows (gm x 128 x K) stay in the XCD's L2 across all column
              // tiles while each B column tile serves gm consecutive blocks; sized so gm A row blocks
              // fit ~2 MB.  (A pure N-fastest walk re-fetched all of B from the Infinity Cache once per
              // row block per XCD: ~8-11 GB per AST launch.)
  float* ws;
  EpiDev e;
  // 0: store through e; 1: only the per-tile sums of squares of the f32 product (e.sqsum), nothing
  // stored; 2: no store either -- the product is a weight gradient and the epilogue applies the Adam
  // update of `adam` to the parameter it belongs to (full 128 x 128 tiles, split 1)
  int mode;
  struct AdamEpi {
    float* p;
    float* m;
    float* v;
    bf16* shadow;        // bf16 operand copy of p, rewritten (or null)
    const float* coef;   // device clip coefficient (mia_clip_adam's)
    float lr_over_bc1, bc2_sqrt, beta1, beta2, eps, wd;
    int64_t ld;          // row stride of p / m / v / shadow (elements)
  } adam;
};

// -------------------------------------------------------------------------- epilogue
static __device__ __forceinline__ void epi_store(const EpiDev& e, int64_t m, int64_t n, float acc) {
  float v = acc * e.alpha;
  if (e.bias) v += e.bias[n];
  switch (e.act) {
    case MIA_ACT_RELU: v = fmaxf(v, 0.f); break;
    case MIA_ACT_GELU: v = gelu_erf(v); break;
    case MIA_DACT_NZ: {
      const float a = ld_elem(e.aux, e.aux_dtype, m * e.ldaux + n);
      v = a != 0.f ? v * e.act_scale : 0.f;
      break;
    }
    case MIA_DACT_GELU: v *= gelu_erf_grad(ld_elem(e.aux, e.aux_dtype, m * e.ldaux + n)); break;
    case MIA_ACT_ADD_AUX: v += ld_elem(e.aux, e.aux_dtype, m * e.ldaux + n); break;
    case MIA_ACT_GELU_SAVE:
      st_elem(const_cast<char*>(e.aux), e.aux_dtype, m * e.ldaux + n, v);
      v = gelu_erf(v);
      break;
    case MIA_ACT_GELU_SAVE_D:
      st_elem(const_cast<char*>(e.aux), e.aux_dtype, m * e.ldaux + n, gelu_erf_grad(v));
      v = gelu_erf(v);
      break;
    case MIA_DACT_MUL: v *= ld_elem(e.aux, e.aux_dtype, m * e.ldaux + n); break;
    default: break;
  }
  int64_t prow = m;
  if (e.rm_inner) {
    if (e.rm_offset == MIA_RM_DROP) {  // drop mode: the last row of every rm_inner group is not stored
      const int64_t x = m % e.rm_inner;
      if (x >= e.rm_outer) return;
      prow = (m / e.rm_inner) * e.rm_outer + x;
    } else {
      prow = (m / e.rm_inner) * e.rm_outer + (m % e.rm_inner) * e.rm_istride + e.rm_offset;
    }
  }
  const int64_t idx = prow * e.ldc + n;
  if (e.accumulate) v += ld_elem(e.ptr, e.dtype, idx);
  st_elem(e.ptr, e.dtype, idx, v);
}

static __device__ __forceinline__ void ld16(const void* p, int dtype, int64_t idx, float* f) {
  if (dtype == MIA_BF16) {
    const uint4* q = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(p) + idx);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4 u = q[h];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[8 * h + 2 * i] = __uint_as_float(w[i] << 16);
        f[8 * h + 2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    }
  } else {
    const float4* q = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + idx);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const float4 u = q[h];
      f[4 * h] = u.x; f[4 * h + 1] = u.y; f[4 * h + 2] = u.z; f[4 * h + 3] = u.w;
    }
  }
}

static __device__ __forceinline__ void st16(void* p, int dtype, int64_t idx, const float* o) {
  if (dtype == MIA_BF16) {
    uint32_t w[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      w[c] = pk_bf16(o[2 * c], o[2 * c + 1]);
    }
    uint4* d = reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(p) + idx);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
  } else {
    float4* d = reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + idx);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
}

// 16 contiguous outputs (m, n0..n0+15) of one row.  Fast path (no accumulate, 16-B aligned output
// and aux rows): bias as float4, aux read/written with 16-B accesses, 16-B stores.  Otherwise per
// element.
static __device__ __forceinline__ void epi_store16(const EpiDev& e, int64_t m, int64_t n0, int64_t N, const float* v) {
  int64_t prow = m;
  if (e.rm_inner) {
    if (e.rm_offset == MIA_RM_DROP) {
      const int64_t x = m % e.rm_inner;
      if (x >= e.rm_outer) return;
      prow = (m / e.rm_inner) * e.rm_outer + x;
    } else {
      prow = (m / e.rm_inner) * e.rm_outer + (m % e.rm_inner) * e.rm_istride + e.rm_offset;
    }
  }
  const int64_t idx = prow * e.ldc + n0;
  const bool uses_aux = e.act == MIA_DACT_NZ || e.act == MIA_DACT_GELU || e.act == MIA_ACT_ADD_AUX ||
                        e.act == MIA_ACT_GELU_SAVE || e.act == MIA_ACT_GELU_SAVE_D || e.act == MIA_DACT_MUL;
  const int64_t aidx = m * e.ldaux + n0;
  const bool fast = n0 + 16 <= N && !e.accumulate &&
                    ((idx * (e.dtype == MIA_BF16 ? 2 : 4)) & 15) == 0 &&
                    ((reinterpret_cast<uintptr_t>(e.ptr)) & 15) == 0 &&
                    (!uses_aux || (((aidx * (e.aux_dtype == MIA_BF16 ? 2 : 4)) & 15) == 0 &&
                                   ((reinterpret_cast<uintptr_t>(e.aux)) & 15) == 0));
  if (!fast) {
    for (int c = 0; c < 16; ++c)
      if (n0 + c < N) epi_store(e, m, n0 + c, v[c]);
    return;
  }
  float o[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) o[c] = v[c] * e.alpha;
  if (e.bias) {
    const float4* b4 = reinterpret_cast<const float4*>(e.bias + n0);
    const bool ba = ((reinterpret_cast<uintptr_t>(e.bias + n0)) & 15) == 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 bb;
      if (ba) bb = b4[q];
      else bb = make_float4(e.bias[n0 + 4 * q], e.bias[n0 + 4 * q + 1], e.bias[n0 + 4 * q + 2], e.bias[n0 + 4 * q + 3]);
      o[4 * q] += bb.x; o[4 * q + 1] += bb.y; o[4 * q + 2] += bb.z; o[4 * q + 3] += bb.w;
    }
  }
  if (e.act == MIA_ACT_RELU) {
#pragma unroll
    for (int c = 0; c < 16; ++c) o[c] = fmaxf(o[c], 0.f);
  } else if (e.act == MIA_ACT_GELU) {
#pragma unroll
    for (int c = 0; c < 16; ++c) o[c] = gelu_erf(o[c]);
  } else if (e.act == MIA_ACT_GELU_SAVE) {
    st16(const_cast<char*>(e.aux), e.aux_dtype, aidx, o);
#pragma unroll
    for (int c = 0; c < 16; ++c) o[c] = gelu_erf(o[c]);
  } else if (e.act == MIA_ACT_GELU_SAVE_D) {
    float d[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) d[c] = gelu_erf_grad(o[c]);
    st16(const_cast<char*>(e.aux), e.aux_dtype, aidx, d);
#pragma unroll
    for (int c = 0; c < 16; ++c) o[c] = gelu_erf(o[c]);
  } else if (uses_aux) {
    float a[16];
    ld16(e.aux, e.aux_dtype, aidx, a);
    if (e.act == MIA_DACT_NZ) {
#pragma unroll
      for (int c = 0; c < 16; ++c) o[c] = a[c] != 0.f ? o[c] * e.act_scale : 0.f;
    } else if (e.act == MIA_DACT_GELU) {
#pragma unroll
      for (int c = 0; c < 16; ++c) o[c] *= gelu_erf_grad(a[c]);
    } else if (e.act == MIA_DACT_MUL) {
#pragma unroll
      for (int c = 0; c < 16; ++c) o[c] *= a[c];
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) o[c] += a[c];
    }
  }
  st16(e.ptr, e.dtype, idx, o);
}


// Rolling-window weight gradient of the 8x8, 32 -> 32 channel valid conv with a BN+ReLU pre-op
// (wgrad8.hip): bf16 NHWC x (n, oh+7, ow+7, 32) raw, dy (n, oh, ow, 32); writes nblk f32 slabs
// ws[nblk][32][2048] (OHWI columns) for the split-K reducer.
struct W8Args {
  const bf16* x;
  const bf16* dy;
  const float* ps;
  const float* pt;
  int n, h, w, oh, ow;
  int nblk;
  float* ws;
};
hipError_t wgrad8_launch(const W8Args& a, hipStream_t s);

// 256 x 256 dense bf16 GEMM of the AST linears (mgemm.hip): eligibility, workspace, launch
bool mg_ok(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
           int compute);
int mg_split(int64_t M, int64_t N, int64_t K);
int64_t mg_workspace_bytes(int64_t M, int64_t N, int64_t K, int colsum, int a_colsum = 0);
int mg_run(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
           void* workspace, hipStream_t s);



}  // namespace mgemm
