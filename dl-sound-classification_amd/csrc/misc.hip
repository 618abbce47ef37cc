// Small kernels of the training step: weight repacking, soft-label loss, grad-norm clip + Adam,
// dropout, AST token assembly, on-GPU BC mixing / SpecAugment+Mixup, casts (gfx950).
#include "common.h"

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------------ weight repacking
__global__ void pack_weight_kernel(const float* __restrict__ src, void* dst, int dtype, int cout, int cin, int kh,
                                   int kw, int mode) {
  const int64_t total = (int64_t)cout * cin * kh * kw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (mode == 0) {  // dst (co, ky, kx, ci) <- src (co, ci, ky, kx)
      const int ci = (int)(i % cin); int64_t q = i / cin;
      const int kx = (int)(q % kw); q /= kw;
      const int ky = (int)(q % kh); const int co = (int)(q / kh);
      st_elem(dst, dtype, i, src[(((int64_t)co * cin + ci) * kh + ky) * kw + kx]);
    } else if (mode == 1) {  // dst (ci, ky, kx, co) <- src (co, ci, kh-1-ky, kw-1-kx)
      const int co = (int)(i % cout); int64_t q = i / cout;
      const int kx = (int)(q % kw); q /= kw;
      const int ky = (int)(q % kh); const int ci = (int)(q / kh);
      st_elem(dst, dtype, i, src[(((int64_t)co * cin + ci) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)]);
    } else if (mode == 2) {  // dst (p, ci, j, co) <- src (co, ci, 0, 2*(kw/2-1-j)+p), kh == 1
      const int half = kw / 2;
      const int co = (int)(i % cout); int64_t q = i / cout;
      const int j = (int)(q % half); q /= half;
      const int ci = (int)(q % cin); const int p = (int)(q / cin);
      st_elem(dst, dtype, i, src[((int64_t)co * cin + ci) * kw + 2 * (half - 1 - j) + p]);
    } else if (mode == 3) {  // dst (ky, j, co) <- src (co, 0, ky, kw-1-j), cin == 1
      const int co = (int)(i % cout); int64_t q = i / cout;
      const int j = (int)(q % kw); const int ky = (int)(q / kw);
      st_elem(dst, dtype, i, src[((int64_t)co * kh + ky) * kw + (kw - 1 - j)]);
    } else {  // mode 4: dst (co, ci, ky, kx) <- src (co, ky, kx, ci), f32
      const int kx = (int)(i % kw); int64_t q = i / kw;
      const int ky = (int)(q % kh); q /= kh;
      const int ci = (int)(q % cin); const int co = (int)(q / cin);
      st_elem(dst, dtype, i, src[(((int64_t)co * kh + ky) * kw + kx) * cin + ci]);
    }
  }
}

// The same repacking for up to MIA_PACK_BATCH weights in one launch (a training step's per-step bf16 packs
// are each a few thousand to 131 072 elements: launch-bound, ~4.7 us apiece as separate kernels).  Job j
// covers the flat range [begin_j, begin_j + total_j); a thread finds its job by a scan of the <= 16 ranges.
struct PackBatch {
  MiaPackJob job[MIA_PACK_BATCH];
  int64_t begin[MIA_PACK_BATCH + 1];
  int n;
};
__global__ void pack_weight_batch_kernel(PackBatch b) {
  const int64_t total = b.begin[b.n];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int j = 0;
    while (j + 1 < b.n && i >= b.begin[j + 1]) ++j;
    const MiaPackJob& J = b.job[j];
    const int64_t e = i - b.begin[j];
    const int cout = J.cout, cin = J.cin, kh = J.kh, kw = J.kw;
    const float* src = J.src;
    float v;
    if (J.mode == 0) {
      const int ci = (int)(e % cin); int64_t q = e / cin;
      const int kx = (int)(q % kw); q /= kw;
      const int ky = (int)(q % kh); const int co = (int)(q / kh);
      v = src[(((int64_t)co * cin + ci) * kh + ky) * kw + kx];
    } else if (J.mode == 1) {
      const int co = (int)(e % cout); int64_t q = e / cout;
      const int kx = (int)(q % kw); q /= kw;
      const int ky = (int)(q % kh); const int ci = (int)(q / kh);
      v = src[(((int64_t)co * cin + ci) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)];
    } else if (J.mode == 2) {
      const int half = kw / 2;
      const int co = (int)(e % cout); int64_t q = e / cout;
      const int jj = (int)(q % half); q /= half;
      const int ci = (int)(q % cin); const int p = (int)(q / cin);
      v = src[((int64_t)co * cin + ci) * kw + 2 * (half - 1 - jj) + p];
    } else {  // mode 3
      const int co = (int)(e % cout); int64_t q = e / cout;
      const int jj = (int)(q % kw); const int ky = (int)(q / kw);
      v = src[((int64_t)co * kh + ky) * kw + (kw - 1 - jj)];
    }
    st_elem(J.dst, J.dtype, e, v);
  }
}

// ------------------------------------------------------------------ soft-label CE
// One block; wave w handles rows w, w+4, ...
constexpr int CE_NT = 1024;
__global__ __launch_bounds__(CE_NT) void soft_ce_kernel(const float* __restrict__ logits, const float* __restrict__ y,
                                                        int B, int C, int input_sigmoid, float* loss_out,
                                                        float* __restrict__ dlogits, int* correct_out) {
  __shared__ double wl[CE_NT / 64];
  __shared__ int wc[CE_NT / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double lsum = 0.0;
  int hits = 0;
  const float invB = 1.f / (float)B;
  for (int b = wave; b < B; b += CE_NT / 64) {
    const float* zr = logits + (int64_t)b * C;
    const float* yr = y + (int64_t)b * C;
    // pass 1: max of z (z = sigmoid(logit) if requested), argmax of logits and of y
    float mx = -INFINITY, bestz = -INFINITY, besty = -INFINITY;
    int az = 1 << 30, ay = 1 << 30;
    for (int c = lane; c < C; c += 64) {
      const float l = zr[c];
      const float z = input_sigmoid ? 1.f / (1.f + __expf(-l)) : l;
      mx = fmaxf(mx, z);
      if (l > bestz) { bestz = l; az = c; }
      if (yr[c] > besty) { besty = yr[c]; ay = c; }
    }
    mx = wave_max(mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float bz = __shfl_xor(bestz, o, 64); const int iz = __shfl_xor(az, o, 64);
      if (bz > bestz || (bz == bestz && iz < az)) { bestz = bz; az = iz; }
      const float by = __shfl_xor(besty, o, 64); const int iy = __shfl_xor(ay, o, 64);
      if (by > besty || (by == besty && iy < ay)) { besty = by; ay = iy; }
    }
    float se = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float l = zr[c];
      const float z = input_sigmoid ? 1.f / (1.f + __expf(-l)) : l;
      se += expf(z - mx);
    }
    se = wave_sum(se);
    // pass 2: loss and R = sum_c y_c p_c / (p_c + eps)
    float lrow = 0.f, R = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float l = zr[c];
      const float z = input_sigmoid ? 1.f / (1.f + __expf(-l)) : l;
      const float p = expf(z - mx) / se;
      lrow += yr[c] * logf(p + 1e-8f);
      R += yr[c] * p / (p + 1e-8f);
    }
    lrow = wave_sum(lrow);
    R = wave_sum(R);
    for (int c = lane; c < C; c += 64) {
      const float l = zr[c];
      const float s = input_sigmoid ? 1.f / (1.f + __expf(-l)) : l;
      const float p = expf(s - mx) / se;
      float g = (p * R - yr[c] * p / (p + 1e-8f)) * invB;
      if (input_sigmoid) g *= s * (1.f - s);
      dlogits[(int64_t)b * C + c] = g;
    }
    if (lane == 0) { lsum += -(double)lrow; hits += (az == ay); }
  }
  if (lane == 0) { wl[wave] = lsum; wc[wave] = hits; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tl = 0.0;
    int tc = 0;
    for (int w = 0; w < CE_NT / 64; ++w) { tl += wl[w]; tc += wc[w]; }
    loss_out[0] = (float)(tl / (double)B);
    if (correct_out) correct_out[0] = tc;
  }
}

// ------------------------------------------------------------------ clip + Adam
constexpr int ADAM_PARTS = 1024;
constexpr int NF_NT = 1024;

// Squared L2 norm partials of every gradient tensor: 16-B loads (tensor storage is 16-B aligned
// torch allocations; a misaligned one takes the scalar path), f32 accumulation flushed to double.
// A tensor with precomputed partials (pre_sq[tsr], e.g. the sqsum slots of the GEMM epilogue that
// wrote it) is not re-read: its partials are summed instead, in the same fixed grid-stride order.
__global__ __launch_bounds__(NT) void sqnorm_kernel(void* const* __restrict__ grads, const int64_t* __restrict__ sizes,
                                                    const void* const* __restrict__ pre_sq,
                                                    const int64_t* __restrict__ pre_n, float* __restrict__ ws) {
  const int tsr = blockIdx.y;
  const float* g = reinterpret_cast<const float*>(grads[tsr]);
  const int64_t n = sizes[tsr];
  const int64_t tid = (int64_t)blockIdx.x * NT + threadIdx.x, nthr = (int64_t)gridDim.x * NT;
  const double* pre = pre_sq ? reinterpret_cast<const double*>(pre_sq[tsr]) : nullptr;
  double s = 0.0;
  float fs = 0.f;
  int cnt = 0;
  if (pre) {
    for (int64_t i = tid; i < pre_n[tsr]; i += nthr) s += pre[i];
  } else if ((reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    const int64_t n4 = n >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = tid; i < n4; i += nthr) {
      const float4 v = g4[i];
      fs = fmaf(v.x, v.x, fs); fs = fmaf(v.y, v.y, fs); fs = fmaf(v.z, v.z, fs); fs = fmaf(v.w, v.w, fs);
      if (++cnt == 64) { s += fs; fs = 0.f; cnt = 0; }
    }
    for (int64_t i = (n4 << 2) + tid; i < n; i += nthr) fs = fmaf(g[i], g[i], fs);
  } else {
    for (int64_t i = tid; i < n; i += nthr) {
      fs = fmaf(g[i], g[i], fs);
      if (++cnt == 256) { s += fs; fs = 0.f; cnt = 0; }
    }
  }
  s += fs;
  s = wave_sum_d(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0)
    reinterpret_cast<double*>(ws)[(int64_t)tsr * ADAM_PARTS + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ws layout (doubles): [ntensors][ADAM_PARTS] partials, then [0] = coef (float in double slot)
__global__ __launch_bounds__(NF_NT) void norm_final_kernel(double* ws, int ntensors, int nparts, float clip,
                                                           float* total_out, float* coef_out) {
  double s = 0.0;
  const int total = ntensors * nparts;
  for (int i = threadIdx.x; i < total; i += NF_NT) {  // fixed order: deterministic
    const int tsr = i / nparts, p = i % nparts;
    s += ws[(int64_t)tsr * ADAM_PARTS + p];
  }
  s = wave_sum_d(s);
  __shared__ double red[NF_NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;
    for (int w = 0; w < NF_NT / 64; ++w) acc += red[w];
    const double tot = sqrt(acc);
    const float totalf = (float)tot;
    float coef = 1.f;
    if (clip > 0.f) {
      coef = clip / (totalf + 1e-6f);
      if (coef > 1.f) coef = 1.f;
    }
    if (total_out) total_out[0] = totalf;
    coef_out[0] = coef;
  }
}

__global__ __launch_bounds__(NT) void adam_kernel(void* const* __restrict__ params, void* const* __restrict__ grads,
                                                  void* const* __restrict__ m1, void* const* __restrict__ m2,
                                                  void* const* __restrict__ shadow,
                                                  const int64_t* __restrict__ sizes, const float* __restrict__ coef_p,
                                                  float lr_over_bc1, float bc2_sqrt, float beta1, float beta2, float eps,
                                                  float wd, const int32_t* __restrict__ steps, float lr) {
  const int tsr = blockIdx.y;
  if (!grads[tsr]) return;  // a deferred weight gradient: its update runs in its GEMM (mia_gemm_adam)
  if (steps) {  // per-tensor step counts (a parameter that missed gradients keeps its own count, as torch's Adam)
    const double st = (double)steps[tsr];
    lr_over_bc1 = (float)(lr / (1.0 - pow((double)beta1, st)));
    bc2_sqrt = (float)sqrt(1.0 - pow((double)beta2, st));
  }
  float* p = reinterpret_cast<float*>(params[tsr]);
  const float* g = reinterpret_cast<const float*>(grads[tsr]);
  float* m = reinterpret_cast<float*>(m1[tsr]);
  float* v = reinterpret_cast<float*>(m2[tsr]);
  bf16* sw = shadow ? reinterpret_cast<bf16*>(shadow[tsr]) : nullptr;  // bf16 operand copy of p (or none)
  const int64_t n = sizes[tsr];
  const float coef = coef_p[0];
  auto upd = [&](float pv, float gv, float& mv, float& vv) {
    gv = fmaf(wd, pv, gv * coef);
    mv = mv + (1.f - beta1) * (gv - mv);           // exp_avg.lerp_(grad, 1 - beta1)
    vv = fmaf((1.f - beta2) * gv, gv, vv * beta2);  // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1-beta2)
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    return pv - lr_over_bc1 * (mv / denom);
  };
  const int64_t tid = (int64_t)blockIdx.x * NT + threadIdx.x, nthr = (int64_t)gridDim.x * NT;
  const bool al = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                    reinterpret_cast<uintptr_t>(v)) & 15) == 0 && (reinterpret_cast<uintptr_t>(sw) & 7) == 0;
  int64_t done = 0;
  if (al) {
    // four float4 groups per iteration, all 16 loads issued before any use (one HBM round trip per
    // 4 groups); every byte is touched once, so loads and stores are non-temporal (no L2/MALL
    // allocation for a 10 GB once-through stream)
    const int64_t n4 = n >> 2;
    constexpr int U = 4;
    f32x4* p4 = reinterpret_cast<f32x4*>(p);
    const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
    f32x4* m4 = reinterpret_cast<f32x4*>(m);
    f32x4* v4 = reinterpret_cast<f32x4*>(v);
    auto step4 = [&](int64_t i, f32x4 pv, f32x4 gv, f32x4 mv, f32x4 vv) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = mv[e], b = vv[e];
        pv[e] = upd(pv[e], gv[e], a, b);
        mv[e] = a;
        vv[e] = b;
      }
      __builtin_nontemporal_store(pv, p4 + i);
      __builtin_nontemporal_store(mv, m4 + i);
      __builtin_nontemporal_store(vv, v4 + i);
      if (sw) {
        const bf16x4 b4 = {(bf16)pv[0], (bf16)pv[1], (bf16)pv[2], (bf16)pv[3]};
        __builtin_nontemporal_store(b4, reinterpret_cast<bf16x4*>(sw) + i);
      }
    };
    int64_t i = tid;
    for (; i + (U - 1) * nthr < n4; i += U * nthr) {
      f32x4 pv[U], gv[U], mv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = i + u * nthr;
        pv[u] = __builtin_nontemporal_load(p4 + j);
        gv[u] = __builtin_nontemporal_load(g4 + j);
        mv[u] = __builtin_nontemporal_load(m4 + j);
        vv[u] = __builtin_nontemporal_load(v4 + j);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) step4(i + u * nthr, pv[u], gv[u], mv[u], vv[u]);
    }
    for (; i < n4; i += nthr) step4(i, p4[i], g4[i], m4[i], v4[i]);
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += nthr) {
    float mv = m[i], vv = v[i];
    p[i] = upd(p[i], g[i], mv, vv);
    m[i] = mv;
    v[i] = vv;
    if (sw) sw[i] = (bf16)p[i];
  }
}

// ------------------------------------------------------------------ dropout / casts
__global__ void dropout_kernel(void* x, int dtype, int64_t n, float p, uint64_t seed) {
  const float scale = 1.f / (1.f - p);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float u = hash_u01(seed, (uint64_t)i);
    const float v = u >= p ? ld_elem(x, dtype, i) * scale : 0.f;
    st_elem(x, dtype, i, v);
  }
}

__global__ void cast_kernel(const void* src, int sd, void* dst, int dd, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    st_elem(dst, dd, i, ld_elem(src, sd, i));
}

__global__ void add_inplace_kernel(float* x, const void* y, int yd, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] += ld_elem(y, yd, i);
}

// ------------------------------------------------------------------ AST tokens
__global__ void tokens_fwd_kernel(const float* __restrict__ patches, const float* __restrict__ cls,
                                  const float* __restrict__ pos, float* __restrict__ out, int B, int Np, int D) {
  const int64_t total = (int64_t)B * (Np + 1) * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int64_t q = i / D;
    const int tkn = (int)(q % (Np + 1));
    const int b = (int)(q / (Np + 1));
    const float base = tkn == 0 ? cls[d] : patches[((int64_t)b * Np + tkn - 1) * D + d];
    out[i] = base + pos[(int64_t)tkn * D + d];
  }
}

// bf16 mode: the patch GEMM wrote token rows (x[b][t] = bias + patch t-1 of clip b . W for t >= 1, the
// cls rows hold the bias of a zero patch); add the positional rows, cls token at t = 0, in place
__global__ void tokens_fwd_inplace_kernel(float4* __restrict__ x, const float4* __restrict__ cls,
                                          const float4* __restrict__ pos, int N, int D4) {
  const int64_t row = blockIdx.x;  // one token row per block, D4 threads
  const int tkn = (int)(row % N), d = threadIdx.x;
  const float4 p = pos[(int64_t)tkn * D4 + d];
  float4 v = tkn == 0 ? cls[d] : x[row * D4 + d];
  v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
  x[row * D4 + d] = v;
}

// The patch matrix of the AST patch embedding (Conv2d(1, D, ps, stride st) over the (B, Fm, Tf)
// spectrogram, reference src/models/ast.py:38 PatchEmbed) in token order: row b*N + t holds patch t-1
// of clip b as bf16 (k = ky*ps + kx, the order of the flattened OIHW weight), row b*N (the cls slot) is
// zero.  8 consecutive k per thread, one 16-B store.
__global__ void ast_patches_kernel(const float* __restrict__ spec, int B, int Fm, int Tf, int ps, int st, int gw,
                                   int N, uint4* __restrict__ out) {
  const int k8 = ps * ps / 8;
  const int64_t total = (int64_t)B * N * k8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % k8);
    const int64_t row = i / k8;
    const int tkn = (int)(row % N);
    const int b = (int)(row / N);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (tkn > 0) {
      const int p = tkn - 1, gy = p / gw, gx = p - gy * gw;
      const int k0 = 8 * c, ky = k0 / ps, kx = k0 - ky * ps;
      const float* src = spec + ((int64_t)b * Fm + gy * st + ky) * Tf + gx * st + kx;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[j] = pk_bf16(src[2 * j], src[2 * j + 1]);
      }
    }
    out[i] = uint4{w[0], w[1], w[2], w[3]};
  }
}

// dpos[t][d] = sum_b dout[b][t][d]; dcls = dpos[0]; dpatches[b][p] = dout[b][1+p]
__global__ void tokens_bwd_kernel(const float* __restrict__ dout, float* __restrict__ dpatches, float* __restrict__ dcls,
                                  float* __restrict__ dpos, int B, int Np, int D) {
  const int64_t total = (int64_t)(Np + 1) * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int tkn = (int)(i / D);
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
      const float v = dout[((int64_t)b * (Np + 1) + tkn) * D + d];
      s += v;
      if (tkn > 0 && dpatches) dpatches[((int64_t)b * Np + tkn - 1) * D + d] = v;
    }
    if (dpos) dpos[i] = s;
    if (tkn == 0 && dcls) dcls[d] = s;
  }
}

// the same with 16-B accesses (4 consecutive d per thread; the per-element sums keep their order over b)
__global__ void tokens_bwd_vec_kernel(const float4* __restrict__ dout, float4* __restrict__ dpatches,
                                      float4* __restrict__ dcls, float4* __restrict__ dpos, int B, int Np, int D4) {
  const int64_t total = (int64_t)(Np + 1) * D4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D4);
    const int tkn = (int)(i / D4);
    float4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int b = 0; b < B; ++b) {
      const float4 v = dout[((int64_t)b * (Np + 1) + tkn) * D4 + d];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      if (tkn > 0 && dpatches) dpatches[((int64_t)b * Np + tkn - 1) * D4 + d] = v;
    }
    if (dpos) dpos[i] = s;
    if (tkn == 0 && dcls) dcls[d] = s;
  }
}

// ------------------------------------------------------------------ BC mixing
// mean square of row idx[blockIdx.x] (or blockIdx.x) of x
constexpr int MS_NT = 1024;
__global__ __launch_bounds__(MS_NT) void clip_ms_kernel(const float* __restrict__ x, int64_t T, const int* __restrict__ idx,
                                                        float* __restrict__ ms) {
  int row = blockIdx.x;
  if (idx) {
    row = idx[blockIdx.x];
    if (row < 0) { if (threadIdx.x == 0) ms[blockIdx.x] = 0.f; return; }
  }
  const float* r = x + (int64_t)row * T;
  float fs = 0.f;
  if ((reinterpret_cast<uintptr_t>(r) & 15) == 0) {
    const int64_t n4 = T >> 2;
    for (int64_t i = threadIdx.x; i < n4; i += MS_NT) {
      const float4 v = reinterpret_cast<const float4*>(r)[i];
      fs = fmaf(v.x, v.x, fs); fs = fmaf(v.y, v.y, fs); fs = fmaf(v.z, v.z, fs); fs = fmaf(v.w, v.w, fs);
    }
    for (int64_t i = (n4 << 2) + threadIdx.x; i < T; i += MS_NT) fs = fmaf(r[i], r[i], fs);
  } else {
    for (int64_t i = threadIdx.x; i < T; i += MS_NT) fs = fmaf(r[i], r[i], fs);
  }
  double s = wave_sum_d((double)fs);
  __shared__ double red[MS_NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < MS_NT / 64; ++w) t += red[w];
    ms[blockIdx.x] = (float)(t / (double)T);
  }
}

__device__ __forceinline__ float spl_db(float ms) {  // BCMixingUtils.a_weighted_spl (preprocessing.py:395-415)
  const float rms = __fsqrt_rn(ms);
  return rms > 0.f ? __fadd_rn(__fmul_rn(20.f, log10f(rms)), 94.f) : -80.f;
}

// one thread per clip: ms[b] (own clip) and msq[b] (partner) -> p, soft labels
__global__ void bc_coef_kernel(const float* __restrict__ ms, const float* __restrict__ msq,
                               const int* __restrict__ partner, const float* __restrict__ r,
                               const int64_t* __restrict__ labels, const int64_t* __restrict__ pool_labels, int B,
                               int C, float* __restrict__ p_out, float* __restrict__ yout) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int q = partner[b];
  const float rr = r[b];
  float p = 1.f;
  if (q >= 0) {
    // perceptual_mixing_coefficient (preprocessing.py:421-447): f32 SPLs, Python-double arithmetic,
    // f32 clamp
    const double d = (double)spl_db(ms[b]) - (double)spl_db(msq[b]);
    double pd = (double)rr;
    if (fabs(d) > 10.0) {
      const double adj = fmin(fabs(d) / 40.0, 0.3);
      pd = d > 0.0 ? pd * (1.0 - adj) : pd * (1.0 + adj);
    }
    p = fminf(fmaxf((float)pd, 0.f), 1.f);
  }
  p_out[b] = p;
  if (yout) {
    for (int c = 0; c < C; ++c) yout[(int64_t)b * C + c] = 0.f;
    if (q >= 0) {
      yout[(int64_t)b * C + labels[b]] = rr;                   // create_soft_labels: uses r, not p
      yout[(int64_t)b * C + pool_labels[q]] = 1.f - rr;
    } else {
      yout[(int64_t)b * C + labels[b]] = 1.f;
    }
  }
}

__global__ void bc_mix_kernel(const float* __restrict__ x, const float* __restrict__ pool, int64_t T, int B,
                              const int* __restrict__ partner, const float* __restrict__ p_in, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int q = partner[b];
  const float p = p_in[b];
  // mix_waveforms (preprocessing.py:468-471) rounded op by op like the reference: p*x1 and (1-p)*x2
  // in f32, their sum, then / f32(sqrt(f32(p^2 + (1-p)^2))) with the sum of squares in double
  const double pd = (double)p;
  const float norm = __fsqrt_rn((float)(pd * pd + (1.0 - pd) * (1.0 - pd)));
  const float q1 = 1.f - p;
  const float* xa = x + (int64_t)b * T;
  const float* xb = pool + (int64_t)(q >= 0 ? q : 0) * T;
  float* o = out + (int64_t)b * T;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = q >= 0 ? __fdiv_rn(__fadd_rn(__fmul_rn(p, xa[i]), __fmul_rn(q1, xb[i])), norm) : xa[i];
}

// Partner draw of apply_bc_mixing (preprocessing.py:584-591): uniform among the pool clips of a
// different class.  One workgroup per clip: pass 1 counts the n_diff candidates, k = min(floor(u *
// n_diff), n_diff - 1), pass 2 finds the k-th candidate in pool order with a chunked block scan
// (ballot + popcount).  Exact (no rejection rounds); -1 when the pool holds no other class.
constexpr int PT_NT = 256;
__global__ __launch_bounds__(PT_NT) void bc_partner_kernel(const int64_t* __restrict__ labels,
                                                           const int64_t* __restrict__ pool_labels, int N,
                                                           const float* __restrict__ u, int* __restrict__ partner) {
  __shared__ int wcnt[PT_NT / 64];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t l = labels[b];
  int ndiff = 0;
  for (int c = 0; c < N; c += PT_NT) {
    const int i = c + threadIdx.x;
    ndiff += __syncthreads_count(i < N && pool_labels[i] != l);
  }
  if (ndiff == 0) {
    if (threadIdx.x == 0) partner[b] = -1;
    return;
  }
  const int k = min((int)floorf(u[b] * (float)ndiff), ndiff - 1);
  int base = 0;  // candidates before this chunk (uniform across the block)
  for (int c = 0; c < N; c += PT_NT) {
    const int i = c + threadIdx.x;
    const bool f = i < N && pool_labels[i] != l;
    const uint64_t m = __ballot(f);
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int before = base;
    for (int w = 0; w < wave; ++w) before += wcnt[w];
    const int rank = before + __popcll(m & ((1ull << lane) - 1ull));
    if (f && rank == k) partner[b] = i;
    int tot = 0;
    for (int w = 0; w < PT_NT / 64; ++w) tot += wcnt[w];
    base += tot;
    __syncthreads();
    if (base > k) break;
  }
}

// Time stretch + gain of EnvNetPreprocessor.apply_augmentation (preprocessing.py:886-925): clip b is
// resampled to m = int(T / factor[b]) samples with torch's linear, align_corners=False rule
// (src = (T/m)(i + 0.5) - 0.5 clamped at 0, i0 = floor(src), i1 = min(i0 + 1, T - 1)) and scaled by
// gain[b]; factor <= 0 means no stretch.  The result is written into the T-sample window (stretched
// clips cropped to T, shortened clips zero-filled past m), so the batch keeps one shape.
__global__ void stretch_gain_kernel(const float* __restrict__ x, int64_t T, const double* __restrict__ factor,
                                    const float* __restrict__ gain, float* __restrict__ out) {
  const int b = blockIdx.y;
  const double fac = factor ? factor[b] : 0.0;
  const int64_t m = fac > 0.0 ? (int64_t)((double)T / fac) : T;
  const float g = gain ? gain[b] : 1.f;
  const float scale = (float)T / (float)m;
  const float* xr = x + (int64_t)b * T;
  float* o = out + (int64_t)b * T;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if (i >= m) {
      v = 0.f;
    } else if (m == T) {
      v = xr[i];
    } else {
      float src = __fsub_rn(__fmul_rn(scale, (float)i + 0.5f), 0.5f);
      src = src < 0.f ? 0.f : src;
      const int64_t i0 = min((int64_t)floorf(src), T - 1);
      const float l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
      const float l0 = 1.f - l1;
      const int64_t i1 = i0 + (i0 < T - 1 ? 1 : 0);
      v = __fadd_rn(__fmul_rn(xr[i0], l0), __fmul_rn(xr[i1], l1));
    }
    o[i] = gain ? __fmul_rn(v, g) : v;
  }
}

// ------------------------------------------------------------------ SpecAugment + Mixup
__global__ void specaug_mixup_kernel(const float* __restrict__ spec, const float* __restrict__ pool,
                                     float* __restrict__ out, int B, int F, int T, const int* t0, const int* tl,
                                     const int* f0, const int* fl, const int* partner, const float* lam) {
  const int b = blockIdx.y;
  const int64_t per = (int64_t)F * T;
  const int q = partner ? partner[b] : -1;
  const float l = (lam && q >= 0) ? lam[b] : 1.f;
  const int ts = t0 ? t0[b] : 0, te = ts + (tl ? tl[b] : 0);
  const int fs = f0 ? f0[b] : 0, fe = fs + (fl ? fl[b] : 0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < per; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i % T), f = (int)(i / T);
    float v = spec[(int64_t)b * per + i];
    if ((t >= ts && t < te) || (f >= fs && f < fe)) v = 0.f;
    if (q >= 0) v = __fadd_rn(__fmul_rn(l, v), __fmul_rn(1.f - l, pool[(int64_t)q * per + i]));  // preprocessing.py:961, op by op
    out[(int64_t)b * per + i] = v;
  }
}

int blocks_for(int64_t n, int per = 256, int cap = 16384) {
  int64_t b = cdiv(n, per);
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" int mia_pack_weight(const float* src, void* dst, int32_t dtype, int32_t cout, int32_t cin, int32_t kh,
                               int32_t kw, int32_t mode, mia_stream_t stream) {
  MIA_CHECK_ARG(src && dst && cout > 0 && cin > 0 && kh > 0 && kw > 0 && mode >= 0 && mode <= 4, "pack_weight: args");
  if (mode == 2) MIA_CHECK_ARG(kh == 1 && kw % 2 == 0, "pack_weight: parity mode needs kh == 1 and even kw");
  if (mode == 3) MIA_CHECK_ARG(cin == 1, "pack_weight: row-split mode needs cin == 1");
  const int64_t total = (int64_t)cout * cin * kh * kw;
  pack_weight_kernel<<<blocks_for(total), 256, 0, as_stream(stream)>>>(src, dst, dtype, cout, cin, kh, kw, mode);
  MIA_LAUNCH_CHECK("pack_weight");
  return 0;
}

extern "C" int mia_pack_weights(const MiaPackJob* jobs, int32_t n, mia_stream_t stream) {
  MIA_CHECK_ARG(jobs && n > 0 && n <= MIA_PACK_BATCH, "pack_weights: 1..%d jobs", MIA_PACK_BATCH);
  PackBatch b;
  memset(&b, 0, sizeof(b));
  b.n = n;
  b.begin[0] = 0;
  for (int j = 0; j < n; ++j) {
    const MiaPackJob& J = jobs[j];
    MIA_CHECK_ARG(J.src && J.dst && J.cout > 0 && J.cin > 0 && J.kh > 0 && J.kw > 0 && J.mode >= 0 && J.mode <= 3 &&
                      (J.dtype == MIA_BF16 || J.dtype == MIA_F32),
                  "pack_weights: job %d: bad arguments (modes 0-3, bf16 / f32)", j);
    if (J.mode == 2) MIA_CHECK_ARG(J.kh == 1 && J.kw % 2 == 0, "pack_weights: job %d: parity mode needs kh == 1, even kw", j);
    if (J.mode == 3) MIA_CHECK_ARG(J.cin == 1, "pack_weights: job %d: row-split mode needs cin == 1", j);
    b.job[j] = J;
    b.begin[j + 1] = b.begin[j] + (int64_t)J.cout * J.cin * J.kh * J.kw;
  }
  pack_weight_batch_kernel<<<blocks_for(b.begin[n]), 256, 0, as_stream(stream)>>>(b);
  MIA_LAUNCH_CHECK("pack_weights");
  return 0;
}

extern "C" int mia_soft_ce(const float* logits, const float* y, int32_t B, int32_t C, int32_t input_sigmoid, float* loss,
                           float* dlogits, int32_t* correct, mia_stream_t stream) {
  MIA_CHECK_ARG(logits && y && loss && dlogits && B > 0 && C > 0, "soft_ce: args");
  soft_ce_kernel<<<1, CE_NT, 0, as_stream(stream)>>>(logits, y, B, C, input_sigmoid, loss, dlogits, correct);
  MIA_LAUNCH_CHECK("soft_ce");
  return 0;
}

extern "C" int64_t mia_adam_workspace_bytes(int32_t ntensors) {
  return ((int64_t)ntensors * ADAM_PARTS + 2) * 8;
}

// byte offset of the clip coefficient (f32) inside mia_clip_adam's workspace
extern "C" int64_t mia_adam_coef_offset(int32_t ntensors) { return (int64_t)ntensors * ADAM_PARTS * 8; }

extern "C" int mia_clip_adam(void* const* params, void* const* grads, void* const* exp_avg, void* const* exp_avg_sq,
                             void* const* shadow_bf16, const int64_t* sizes, int32_t ntensors, int64_t max_numel,
                             int64_t max_norm_numel, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int32_t step, float clip,
                             float* total_norm_out, void* sqnorm_ws, const void* const* pre_sq,
                             const int64_t* pre_n, const int32_t* steps, mia_stream_t stream) {
  MIA_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && sizes && sqnorm_ws, "clip_adam: null table");
  MIA_CHECK_ARG(ntensors > 0 && ntensors < 65536 && step >= 1, "clip_adam: ntensors/step");
  MIA_CHECK_ARG(!pre_sq || pre_n, "clip_adam: pre_sq needs pre_n");
  hipStream_t s = as_stream(stream);
  double* ws = reinterpret_cast<double*>(sqnorm_ws);
  float* coef = reinterpret_cast<float*>(ws + (int64_t)ntensors * ADAM_PARTS);
  const int parts = (int)std::min<int64_t>(ADAM_PARTS, std::max<int64_t>(1, cdiv(max_norm_numel, 256 * 256)));
  sqnorm_kernel<<<dim3(parts, ntensors), NT, 0, s>>>(grads, sizes, pre_sq, pre_n, reinterpret_cast<float*>(ws));
  MIA_LAUNCH_CHECK("sqnorm");
  norm_final_kernel<<<1, NF_NT, 0, s>>>(ws, ntensors, parts, clip, total_norm_out, coef);
  MIA_LAUNCH_CHECK("norm_final");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const int ablocks = (int)std::min<int64_t>(8192, std::max<int64_t>(1, cdiv(max_numel, 256 * 32)));
  adam_kernel<<<dim3(ablocks, ntensors), NT, 0, s>>>(params, grads, exp_avg, exp_avg_sq, shadow_bf16, sizes, coef,
                                                     (float)(lr / bc1), (float)sqrt(bc2), beta1, beta2, eps,
                                                     weight_decay, steps, lr);
  MIA_LAUNCH_CHECK("adam");
  return 0;
}

extern "C" int mia_dropout(void* x, int32_t dtype, int64_t numel, float p, uint64_t seed, mia_stream_t stream) {
  MIA_CHECK_ARG(x && p >= 0.f && p < 1.f, "dropout: args");
  if (p == 0.f || numel == 0) return 0;
  dropout_kernel<<<blocks_for(numel), 256, 0, as_stream(stream)>>>(x, dtype, numel, p, seed);
  MIA_LAUNCH_CHECK("dropout");
  return 0;
}

extern "C" int mia_cast(const void* src, int32_t sdtype, void* dst, int32_t ddtype, int64_t numel, mia_stream_t stream) {
  MIA_CHECK_ARG(src && dst, "cast: null");
  if (numel == 0) return 0;
  cast_kernel<<<blocks_for(numel), 256, 0, as_stream(stream)>>>(src, sdtype, dst, ddtype, numel);
  MIA_LAUNCH_CHECK("cast");
  return 0;
}

extern "C" int mia_add_inplace(float* x, const void* y, int32_t ydtype, int64_t numel, mia_stream_t stream) {
  MIA_CHECK_ARG(x && y, "add_inplace: null");
  if (numel == 0) return 0;
  add_inplace_kernel<<<blocks_for(numel), 256, 0, as_stream(stream)>>>(x, y, ydtype, numel);
  MIA_LAUNCH_CHECK("add_inplace");
  return 0;
}

extern "C" int mia_tokens_fwd(const float* patches, const float* cls, const float* pos, float* out, int32_t B,
                              int32_t Np, int32_t D, mia_stream_t stream) {
  MIA_CHECK_ARG(patches && cls && pos && out && B > 0 && Np > 0 && D > 0, "tokens_fwd: args");
  tokens_fwd_kernel<<<blocks_for((int64_t)B * (Np + 1) * D), 256, 0, as_stream(stream)>>>(patches, cls, pos, out, B, Np, D);
  MIA_LAUNCH_CHECK("tokens_fwd");
  return 0;
}

extern "C" int mia_tokens_fwd_inplace(float* x, const float* cls, const float* pos, int32_t B, int32_t N, int32_t D,
                                      mia_stream_t stream) {
  MIA_CHECK_ARG(x && cls && pos && B > 0 && N > 1 && D > 0 && D % 4 == 0, "tokens_fwd_inplace: args");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(cls) | reinterpret_cast<uintptr_t>(pos)) & 15) == 0,
                "tokens_fwd_inplace: x / cls / pos must be 16-byte aligned");
  MIA_CHECK_ARG(D / 4 <= 1024 && (int64_t)B * N < (1ll << 31), "tokens_fwd_inplace: D <= 4096, B*N < 2^31");
  tokens_fwd_inplace_kernel<<<(unsigned)((int64_t)B * N), D / 4, 0, as_stream(stream)>>>(
      reinterpret_cast<float4*>(x), reinterpret_cast<const float4*>(cls), reinterpret_cast<const float4*>(pos), N, D / 4);
  MIA_LAUNCH_CHECK("tokens_fwd_inplace");
  return 0;
}

extern "C" int mia_ast_patches(const float* spec, int32_t B, int32_t Fm, int32_t Tf, int32_t ps, int32_t st, void* out,
                               mia_stream_t stream) {
  // each thread's 8 consecutive k stay in one patch row (k0 = 8c, kx = k0 mod ps): ps % 8 == 0
  MIA_CHECK_ARG(spec && out && B > 0 && ps > 0 && st > 0 && Fm >= ps && Tf >= ps && ps % 8 == 0,
                "ast_patches: args (ps must be a multiple of 8)");
  MIA_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "ast_patches: out must be 16-byte aligned");
  const int gh = (Fm - ps) / st + 1, gw = (Tf - ps) / st + 1, N = gh * gw + 1;
  ast_patches_kernel<<<blocks_for((int64_t)B * N * (ps * ps / 8)), 256, 0, as_stream(stream)>>>(
      spec, B, Fm, Tf, ps, st, gw, N, reinterpret_cast<uint4*>(out));
  MIA_LAUNCH_CHECK("ast_patches");
  return 0;
}

extern "C" int mia_tokens_bwd(const float* dout, float* dpatches, float* dcls, float* dpos, int32_t B, int32_t Np,
                              int32_t D, mia_stream_t stream) {
  MIA_CHECK_ARG(dout && B > 0 && Np > 0 && D > 0, "tokens_bwd: args");
  const bool vec = D % 4 == 0 && ((reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dpatches) |
                                   reinterpret_cast<uintptr_t>(dpos) | reinterpret_cast<uintptr_t>(dcls)) & 15) == 0;
  if (vec)
    tokens_bwd_vec_kernel<<<blocks_for((int64_t)(Np + 1) * (D / 4)), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(dout), reinterpret_cast<float4*>(dpatches), reinterpret_cast<float4*>(dcls),
        reinterpret_cast<float4*>(dpos), B, Np, D / 4);
  else
    tokens_bwd_kernel<<<blocks_for((int64_t)(Np + 1) * D), 256, 0, as_stream(stream)>>>(dout, dpatches, dcls, dpos, B, Np, D);
  MIA_LAUNCH_CHECK("tokens_bwd");
  return 0;
}

extern "C" int mia_bc_mix(const float* x, const float* pool, int64_t T, int32_t B, const int32_t* partner,
                          const float* r, const int64_t* labels, const int64_t* pool_labels, int32_t num_classes,
                          float* out, float* yout, float* p_out, void* workspace, mia_stream_t stream) {
  MIA_CHECK_ARG(x && pool && partner && r && labels && pool_labels && out && p_out && workspace && B > 0 && T > 0,
                "bc_mix: args");
  MIA_CHECK_ARG(out != x && out != pool, "bc_mix: out must not alias the inputs");
  hipStream_t s = as_stream(stream);
  float* ms = reinterpret_cast<float*>(workspace);
  float* msq = ms + B;
  clip_ms_kernel<<<B, MS_NT, 0, s>>>(x, T, nullptr, ms);
  MIA_LAUNCH_CHECK("clip_ms");
  clip_ms_kernel<<<B, MS_NT, 0, s>>>(pool, T, partner, msq);
  MIA_LAUNCH_CHECK("clip_ms(partner)");
  bc_coef_kernel<<<(unsigned)cdiv(B, 256), 256, 0, s>>>(ms, msq, partner, r, labels, pool_labels, B, num_classes,
                                                        p_out, yout);
  MIA_LAUNCH_CHECK("bc_coef");
  bc_mix_kernel<<<dim3((unsigned)std::min<int64_t>(cdiv(T, 256), 512), B), 256, 0, s>>>(x, pool, T, B, partner, p_out,
                                                                                      out);
  MIA_LAUNCH_CHECK("bc_mix");
  return 0;
}

extern "C" int mia_bc_partner(const int64_t* labels, int32_t B, const int64_t* pool_labels, int32_t N, const float* u,
                              int32_t* partner, mia_stream_t stream) {
  MIA_CHECK_ARG(labels && pool_labels && u && partner && B > 0 && N > 0, "bc_partner: args");
  bc_partner_kernel<<<B, PT_NT, 0, as_stream(stream)>>>(labels, pool_labels, N, u, partner);
  MIA_LAUNCH_CHECK("bc_partner");
  return 0;
}

extern "C" int mia_stretch_gain(const float* x, int64_t T, int32_t B, const double* factor, const float* gain,
                                float* out, mia_stream_t stream) {
  MIA_CHECK_ARG(x && out && B > 0 && T > 0 && out != x, "stretch_gain: args");
  stretch_gain_kernel<<<dim3((unsigned)std::min<int64_t>(cdiv(T, 256), 512), B), 256, 0, as_stream(stream)>>>(
      x, T, factor, gain, out);
  MIA_LAUNCH_CHECK("stretch_gain");
  return 0;
}

extern "C" int mia_spec_augment_mixup(const float* spec, const float* pool, float* out, int32_t B, int32_t F,
                                      int32_t T, const int32_t* t0, const int32_t* tlen, const int32_t* f0,
                                      const int32_t* flen, const int32_t* partner, const float* lam,
                                      mia_stream_t stream) {
  MIA_CHECK_ARG(spec && out && B > 0 && F > 0 && T > 0, "spec_augment_mixup: args");
  MIA_CHECK_ARG(!partner || (pool && pool != out), "spec_augment_mixup: mixup needs a pool distinct from out");
  specaug_mixup_kernel<<<dim3((unsigned)std::min<int64_t>(cdiv((int64_t)F * T, 256), 512), B), 256, 0,
                         as_stream(stream)>>>(spec, pool ? pool : spec, out, B, F, T, t0, tlen, f0, flen, partner, lam);
  MIA_LAUNCH_CHECK("spec_augment_mixup");
  return 0;
}

// ------------------------------------------------------------------------------ box calibration
// Streaming copy dst <- src of n16 16-B groups (bench.py's same-process HBM calibration: the rate this box's
// HBM reaches for a plain read + write stream, next to which a kernel's achieved GB/s is judged).  Four
// groups in flight per thread, non-temporal loads and stores (the stream is touched once), grid-stride.
__global__ __launch_bounds__(256) void stream_copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                          int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) v[u] = __builtin_nontemporal_load(src + i + 256 * u);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) __builtin_nontemporal_store(v[u], dst + i + 256 * u);
  }
}

extern "C" int mia_stream_copy(const void* src, void* dst, int64_t bytes, mia_stream_t stream) {
  MIA_CHECK_ARG(src && dst && bytes > 0 && bytes % 16 == 0, "stream_copy: bytes must be a positive multiple of 16");
  MIA_CHECK_ARG(((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0,
                "stream_copy: 16-B aligned pointers");
  const int64_t n16 = bytes / 16;
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(n16, 1024), (int64_t)mia::cu_count() * 16);
  stream_copy_kernel<<<grid, 256, 0, as_stream(stream)>>>((const f32x4*)src, (f32x4*)dst, n16);
  MIA_LAUNCH_CHECK("stream_copy");
  return 0;
}

// Back-to-back bf16 MFMAs (bench.py's same-process MFMA calibration: the v_mfma_f32_16x16x32_bf16 rate this box
// holds with every SIMD busy on random operands -- the DVFS clock under an MFMA load differs box to box, so an
// MFMA-bound kernel's TFLOP/s is also read against this rate).  Each wave keeps 4 independent accumulators
// (the dependent-issue latency hidden), operands are per-lane pseudo-random bf16 (the clock held on zeros is
// higher), and the accumulators are written out at the end so nothing is dead.
__global__ __launch_bounds__(256) void mfma_rate_kernel(int iters, uint32_t seed, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  uint32_t h = seed ^ (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h = h * 1664525u + 1013904223u;
    a[i] = (bf16)((float)(int)(h >> 16 & 0xff) * (1.f / 128.f) - 1.f);
    b[i] = (bf16)((float)(int)(h >> 24) * (1.f / 128.f) - 1.f);
  }
  f32x4 acc[4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[q], 0, 0, 0);
  }
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) v += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  sink[blockIdx.x * 256 + threadIdx.x] = v + (float)lane * 0.f;
}

extern "C" int64_t mia_mfma_rate_sink_floats(int32_t waves_per_simd) {
  return (int64_t)mia::cu_count() * (waves_per_simd > 0 ? waves_per_simd : 1) * 256;
}

extern "C" int mia_mfma_rate(float* sink, int32_t iters, int32_t waves_per_simd, mia_stream_t stream) {
  MIA_CHECK_ARG(sink && iters > 0 && waves_per_simd > 0 && waves_per_simd <= 8, "mfma_rate: bad arguments");
  const unsigned grid = (unsigned)(mia::cu_count() * waves_per_simd);  // 4 waves per block: one per SIMD
  mfma_rate_kernel<<<grid, 256, 0, as_stream(stream)>>>(iters, 0x9e3779b9u, sink);
  MIA_LAUNCH_CHECK("mfma_rate");
  return 0;
}
