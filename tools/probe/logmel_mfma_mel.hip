// Fused batched log-mel for gfx950: ASTPreprocessor.preprocess (preprocessing.py:1013-1039).
//
// Per frame f (hop 160): the 400 windowed samples x[f*160-200+u]*hann[u] (reflect padding at the
// clip edges, = torch.stft center=True with the 400-tap window centred in n_fft=1024) are packed as
// 200 complex points z[n] = x[2n] + i x[2n+1], transformed by a 512-point Stockham radix-8 FFT in
// LDS (one wave per frame, 3 passes in one in-place buffer per wave), split into the 513 real-FFT
// bins, squared, projected onto the 128 htk mel bands by f32 MFMA (below), and converted to dB
// (10 log10 = 10 log10(2) * v_log_f32).
// Complex values are float2 vectors: every complex add is one v_pk_add_f32, every twiddle
// multiply one v_pk_mul_f32 + one v_pk_fma_f32 (op_sel swizzles, no moves); the Stockham buffer is
// XOR-swizzled (first-pass writes 1-2-way instead of 8-way bank conflicts).
// Persistent 4-wave workgroups (three per CU) walk (clip, 16-frame chunk) items: the 2,800-sample
// input segment of the NEXT chunk is loaded into registers (coalesced, reflect-padded) while this
// chunk's 16 frames are computed (4 per wave), then committed to LDS; window taps and the twiddles of
// the three passes are read once per workgroup (the real-split twiddles derived per frame from one per
// lane).
// Mel projection: each wave keeps the power spectra of its 4 frames in LDS and runs them through
// v_mfma_f32_4x4x1_16b_f32 (16 independent 4 x 4 x 1 blocks per instruction; layout measured by
// tools/probe/mfma4x4_layout.cpp: lane 4b + j supplies B column j and receives D[0..3][j] of block b,
// lane 4b + i supplies A row i): block b of set s owns mels 64 s + 4 b .. + 3 (the 4 lanes' B operands
// = their weights) and the 4 frames (rows), and steps through the block's own bins from its 4-aligned
// first bin, one bin per instruction, so every block walks only its own band (block-sparse: 84
// instructions for 4 frames x 128 mels at 44.1 kHz instead of 4 x 129 x 2 dense).  An f32 MFMA is
// bit-for-bit an f32 fmaf chain in k order and a zero weight is an exact no-op on the finite power, so
// each band's sum is the same ordered chain over its bins as the per-band FMA loop this replaces
// (bit-identical output).  The weights are pre-interleaved once per call by mel_mfma_table_kernel into
// [set][4-bin step][lane] f32x4 rows in the workspace (one global 16-B load per lane per 4 MFMAs),
// the power spectrum is read with one ds_read_b128 per 4 MFMAs.  The dB values go straight from the
// accumulators to global memory (lane = mel, 4 frames).
// Per-clip top_db clamp + mean / unbiased-std normalisation need the clip max first, so two light
// passes follow (stats over the dB tensor, which stays in the 256 MB Infinity Cache at batch 256,
// then an in-place normalise).
#include "common.h"

namespace {

constexpr int FB = 16;          // frames per chunk (LW waves x 4)
constexpr int LW = 4;           // waves per workgroup
constexpr int LNT = 64 * LW;
constexpr int NFFT = 1024;
constexpr int NC = 512;         // complex FFT size
constexpr int HOP = 160;
constexpr int WIN = 400;
constexpr int NMEL_MAX = 128;
constexpr int SEG = (FB - 1) * HOP + WIN;  // 5360 samples
constexpr int SPT = (SEG + LNT - 1) / LNT;  // segment samples per thread

typedef float f2 __attribute__((ext_vector_type(2)));

struct MelTables {
  const float* window;   // [WIN]
  const f2* tw512;       // [512] exp(-2 pi i q / 512)
  const f2* tw1024;      // [513] exp(-2 pi i k / 1024)
  const int* band_start; // [n_mels]
  const int* band_len;   // [n_mels]
  const int* band_off;   // [n_mels] offset into band_w
  const float* band_w;   // [nnz]
};

__device__ __forceinline__ f2 cmul(f2 a, f2 b) { return __builtin_elementwise_fma(a.yy, b.yx * f2{-1.f, 1.f}, a.xx * b); }
__device__ __forceinline__ f2 mul_mi(f2 a) { return a.yx * f2{1.f, -1.f}; }  // a * (-i)

// In-register DFT8 (natural-order output), W8 = exp(-2 pi i / 8).
__device__ __forceinline__ void dft8(f2 (&v)[8]) {
  const float s = 0.70710678118654752f;
  const f2 a0 = v[0] + v[4], a4 = v[0] - v[4];
  const f2 a1 = v[1] + v[5], t5 = v[1] - v[5];
  const f2 a2 = v[2] + v[6], t6 = v[2] - v[6];
  const f2 a3 = v[3] + v[7], t7 = v[3] - v[7];
  const f2 a5 = s * (t5 + t5.yx * f2{1.f, -1.f});   // * W8^1 = s(1 - i)
  const f2 a6 = mul_mi(t6);                         // * W8^2 = -i
  const f2 a7 = s * (t7.yx * f2{1.f, -1.f} - t7);   // * W8^3 = s(-1 - i)
  const f2 b0 = a0 + a2, b2 = a0 - a2;
  const f2 b1 = a1 + a3, b3 = mul_mi(a1 - a3);
  const f2 b4 = a4 + a6, b6 = a4 - a6;
  const f2 b5 = a5 + a7, b7 = mul_mi(a5 - a7);
  v[0] = b0 + b1; v[4] = b0 - b1;
  v[2] = b2 + b3; v[6] = b2 - b3;
  v[1] = b4 + b5; v[5] = b4 - b5;
  v[3] = b6 + b7; v[7] = b6 - b7;
}

// Stockham buffer swizzle: entry i at i ^ ((i >> 3) & 7).  The reads (lane + 64 r) stay one contiguous
// 256-entry span per half wave (conflict-free ds_read_b64); the first pass's writes (8 consecutive
// entries per lane) spread over 16 banks pairs instead of 2 (1- to 2-way instead of 8-way).
__device__ __forceinline__ int swz(int i) { return i ^ ((i >> 3) & 7); }


__device__ __forceinline__ int reflect_idx(int n, int T) {
  if (n < 0) n = -n;
  if (n >= T) n = 2 * (T - 1) - n;
  return n;
}

constexpr int QMAX = (NC + 1 + 3) / 4 + 1;  // 4-bin steps per set, upper bound (513 bins from any 4-aligned start)
#ifndef LM_WR
#define LM_WR 8
#endif
constexpr int WR = LM_WR;                     // weight steps in flight per lane (mel projection)
constexpr int PST = 520;                     // floats per saved power spectrum (513 bins + zero pad, 16-B rows)
constexpr float DB_PER_LOG2 = 3.0102999566398120f;  // 10 log10(2)
// W16^q = exp(-2 pi i q / 16)
__constant__ const f2 W16[8] = {{1.f, 0.f},
                                {0.92387953251128674f, -0.38268343236508977f},
                                {0.70710678118654752f, -0.70710678118654752f},
                                {0.38268343236508977f, -0.92387953251128674f},
                                {0.f, -1.f},
                                {-0.38268343236508977f, -0.92387953251128674f},
                                {-0.70710678118654752f, -0.70710678118654752f},
                                {-0.92387953251128674f, -0.38268343236508977f}};

// The mel projection's operand tables, once per call (one workgroup): per set s (mels 64 s .. 64 s + 63)
// the number of 4-bin steps nq[s] = the widest block's span, per lane the 4-aligned first bin of its
// block (moved left where needed so every block's nq[s] steps stay inside the PST-float spectrum row:
// the extra steps have zero weights), and the weights as [set][step][lane] f32x4.
// hdr = {nq[0], nq[1], start[2][64]}.
__global__ __launch_bounds__(128) void mel_mfma_table_kernel(MelTables tb, int n_mels, int* __restrict__ hdr,
                                                             f32x4* __restrict__ tab) {
  __shared__ int gs[32], ge[32], nq[2];
  const int t = threadIdx.x;
  if (t < 32) {
    int lo = 1 << 30, hi = -1;
    for (int m = 4 * t; m < 4 * t + 4 && m < n_mels; ++m) {
      const int len = tb.band_len[m];
      if (len <= 0) continue;
      lo = min(lo, tb.band_start[m]);
      hi = max(hi, tb.band_start[m] + len - 1);
    }
    if (hi < 0) lo = 0, hi = -1;  // no bins: zero steps of its own
    gs[t] = lo & ~3;
    ge[t] = hi;
  }
  __syncthreads();
  if (t < 2) {
    int q = 0;
    for (int g = 16 * t; g < 16 * t + 16; ++g) q = max(q, (ge[g] - gs[g] + 1 + 3) >> 2);
    nq[t] = q;
    hdr[t] = q;
  }
  __syncthreads();
  const int st = t >> 6, lane = t & 63, g = 16 * st + (lane >> 2), m = 64 * st + lane;
  const int a = min(gs[g], PST - 4 * nq[st]);  // PST, gs multiples of 4; 4 nq <= 4 (QMAX - 1) <= PST
  hdr[2 + t] = a;
  const bool has = m < n_mels;
  const int ks = has ? tb.band_start[m] : 0, len = has ? tb.band_len[m] : 0, off = has ? tb.band_off[m] : 0;
  for (int q = 0; q < nq[st]; ++q) {
    f32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = a + 4 * q + j;
      w[j] = (k >= ks && k < ks + len) ? tb.band_w[off + k - ks] : 0.f;
    }
    tab[(st * QMAX + q) * 64 + lane] = w;
  }
}

#ifndef LM_OCC
#define LM_OCC 3
#endif
#ifndef LM_TILE
#define LM_TILE 1
#endif
#ifndef LM_WLDS
#define LM_WLDS 0
#endif
constexpr int WLMAX = 24;  // weight steps (both sets) staged in LDS when LM_WLDS
__global__ __launch_bounds__(LNT) __attribute__((amdgpu_waves_per_eu(LM_OCC, LM_OCC))) void fft_mel_db_kernel(const float* __restrict__ wav, int64_t ld, int T,
                                                            int frames, int nbm, int nitems, int n_mels,
                                                            MelTables tb, const int* __restrict__ mhdr,
                                                            const f32x4* __restrict__ mtab,
                                                            float* __restrict__ out,
                                                            float* __restrict__ blockmax) {
  __shared__ float seg[SEG];
  __shared__ f2 buf[LW][NC];             // one in-place Stockham buffer per wave
  __shared__ float pw[LW][3][PST];    // power spectra of frames 0-2 of each wave (frame 3 stays in buf)
#if LM_WLDS
  __shared__ f32x4 wl[WLMAX * 64];
#endif
  __shared__ float redmax[LW];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

  // loop-invariant per-lane constants: window taps, stage twiddles, real-split twiddles
  f2 win[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = 2 * (lane + 64 * r);
    win[r] = u < WIN ? f2{tb.window[u], tb.window[u + 1]} : f2{0.f, 0.f};
  }
  f2 tw1[8], tw2[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    tw1[r] = tb.tw512[((lane % 8) * (NC / 64) * r) & (NC - 1)];
    tw2[r] = tb.tw512[(lane * (NC / 512) * r) & (NC - 1)];
  }
  // real-split twiddles W1024^(lane + 64 q) = W1024^lane * W16^q (one per lane in registers)
  f2 tws0 = tb.tw1024[lane];

#if LM_WLDS
  const int nq0 = mhdr[0], nq1 = mhdr[1];
  const bool wlds = nq0 + nq1 <= WLMAX;
  if (wlds) {
    for (int i = t; i < nq0 * 64; i += LNT) wl[i] = mtab[i];
    for (int i = t; i < nq1 * 64; i += LNT) wl[nq0 * 64 + i] = mtab[QMAX * 64 + i];
  }
#endif
  // the reflect-padded input segment of chunk `it` into registers (coalesced 4-B loads)
  auto seg_load = [&](int it, float (&r)[SPT]) __attribute__((always_inline)) {
    const int b = it / nbm;
    const int s0 = (it - b * nbm) * FB * HOP - WIN / 2;
    const float* x = wav + (int64_t)b * ld;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int i = t + LNT * j;
      const int n = s0 + i;
#ifdef LM_NOLOAD
      r[j] = (float)(i & 7) * 0.01f + (float)n * 1e-6f;
#else
      r[j] = (i < SEG && n >= -(NFFT / 2) && n < T + NFFT / 2) ? x[reflect_idx(n, T)] : 0.f;  // T > 512
#endif
    }
  };

  f2* d = buf[wave];
  float pre[SPT];
  int it = blockIdx.x;
  if (it < nitems) seg_load(it, pre);
  for (; it < nitems; it += gridDim.x) {
    __syncthreads();  // the previous chunk's segment and tile reads are done (tables visible, 1st pass)
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int i = t + LNT * j;
      if (i < SEG) seg[i] = pre[j];
    }
    __syncthreads();
    if (it + (int)gridDim.x < nitems) seg_load(it + gridDim.x, pre);  // in flight under this chunk
    const int b = it / nbm;
    const int f0 = (it - b * nbm) * FB;
    float lmax = -INFINITY;
    int nf_w = 0;  // frames this wave computed in this chunk (wave-uniform)
#pragma unroll 1
    for (int k = 0; k < FB / LW; ++k) {
      const int fi = wave * (FB / LW) + k;
      if (f0 + fi >= frames) break;  // wave-uniform
      // stage 0 (Ns = 1) reads z[j + 64 r] straight from the segment, z[n] = 0 for n >= 200
      {
        f2 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int n = lane + 64 * r;
          if (r < 4 && n < WIN / 2)
            v[r] = *reinterpret_cast<const f2*>(&seg[fi * HOP + 2 * n]) * win[r];
          else
            v[r] = f2{0.f, 0.f};
        }
        dft8(v);
#pragma unroll
        for (int r = 0; r < 8; ++r) d[swz(lane * 8 + r)] = v[r];
      }
      wave_sync();
      // stages 1 (Ns = 8) and 2 (Ns = 64), in place: every lane's reads land before any lane's writes
      // (one wave, program order), so the single buffer needs no ping-pong
#ifdef LM_SKIPFFT
#pragma unroll
      for (int st = 1; st < 1; ++st) {
#else
#pragma unroll
      for (int st = 1; st < 3; ++st) {
#endif
        const int Ns = st == 1 ? 8 : 64;
        f2 v[8];
        const int jm = lane % Ns;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const f2 a = d[swz(lane + 64 * r)];
          v[r] = r ? cmul(a, st == 1 ? tw1[r] : tw2[r]) : a;
        }
        dft8(v);
        wave_sync();
        const int idxD = (lane / Ns) * Ns * 8 + jm;
#pragma unroll
        for (int r = 0; r < 8; ++r) d[swz(idxD + r * Ns)] = v[r];
        wave_sync();
      }
      // Z in d (natural order). Real-FFT split -> power P[k] (k = 0..512), kept in registers, then
      // written over the (consumed) spectrum as floats.  X[k] = 0.5 (e - i W^k o) with
      // e = Z[k] + conj(Z[N-k]), o = Z[k] - conj(Z[N-k]); |X|^2 = 0.25 |e - i W^k o|^2.
      float pk[8];
      asm volatile("" : "+v"(tws0));  // derived per frame (not hoisted: registers)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = lane + 64 * q;
        const f2 zk = d[swz(k)];
        const f2 zc = d[swz((NC - k) & (NC - 1))] * f2{1.f, -1.f};
        const f2 tq = q ? cmul(tws0, W16[q]) : tws0;
        const f2 wo = cmul(tq, zk - zc);
        const f2 X = (zk + zc) - wo.yx * f2{-1.f, 1.f};  // e - i wo = (e.x + wo.y, e.y - wo.x)
        pk[q] = 0.25f * (X.x * X.x + X.y * X.y);
      }
      float pn = 0.f;
      if (lane == 0) {
        const f2 z0 = d[0];
        const float xn = z0.x - z0.y;  // X[512]
        pn = xn * xn;
      }
      wave_sync();  // every lane's spectrum reads are done (frame 3's spectrum goes over its FFT buffer)
      float* P = k < 3 ? pw[wave][k] : reinterpret_cast<float*>(d);
#pragma unroll
      for (int q = 0; q < 8; ++q) P[lane + 64 * q] = pk[q];
      if (lane < PST - NC) P[NC + lane] = lane == 0 ? pn : 0.f;  // bin 512 + zero pad (read with zero weights)
      ++nf_w;
    }
    wave_sync();
#if LM_TILE
    f32x4 dv0, dv1;
#endif
    // mel projection of the wave's nf_w frames: lane supplies A = P[frame lane & 3][block's bins] and
    // B = the weights of mel 64 s + lane; accumulator r of lane 4 b + j = mel 64 s + 4 b + j, frame r
    {
      const float* Pi = (lane & 3) < 3 ? pw[wave][lane & 3] : reinterpret_cast<const float*>(d);
      const int fb0 = f0 + wave * (FB / LW);
#pragma unroll 1
      for (int st = 0; st < 2; ++st) {
#ifdef LM_SKIPMEL
        const int nq = 0;
#else
        const int nq = mhdr[st];  // uniform
#endif
        const float* pa = Pi + mhdr[2 + 64 * st + lane];
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#if LM_WLDS
        if (wlds) {
          const f32x4* wt = wl + (st ? nq0 * 64 : 0) + lane;
#pragma unroll 4
          for (int q = 0; q < nq; ++q) {
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(pa + 4 * q);
            const f32x4 w4 = wt[q * 64];
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[0], w4[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[1], w4[1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[2], w4[2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[3], w4[3], acc, 0, 0, 0);
          }
        } else
#endif
        {
        int lo = lane;
        asm volatile("" : "+v"(lo));  // per chunk: keeps the (loop-invariant) ring loads from being hoisted
        const f32x4* wt = mtab + st * QMAX * 64 + lo;
        // weights: a ring of WR steps in flight from L2 (the FFT's registers are dead here)
        f32x4 wr[WR];
#pragma unroll
        for (int j = 0; j < WR; ++j)
          if (j < nq) wr[j] = wt[j * 64];
#pragma unroll 1
        for (int q0 = 0; q0 < nq; q0 += WR) {
#pragma unroll
          for (int j = 0; j < WR; ++j) {
            const int q = q0 + j;
            if (q >= nq) break;
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(pa + 4 * q);
            const f32x4 w4 = wr[j];
            if (q + WR < nq) wr[j] = wt[(q + WR) * 64];
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[0], w4[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[1], w4[1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[2], w4[2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a4[3], w4[3], acc, 0, 0, 0);
          }
        }
        }
#if LM_TILE
        if (st == 0) dv0 = acc; else dv1 = acc;
      }
    }
    // dB values through a 128 x 16 tile (aliasing the spectra, free once every wave's MFMAs are done)
    // so the output rows are written as 16 contiguous frames
    __syncthreads();
    {
      float (*tile)[FB + 1] = reinterpret_cast<float (*)[FB + 1]>(&pw[0][0][0]);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int m = 64 * st + lane;
        if (m < n_mels) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (r >= nf_w) break;
            // AmplitudeToDB (multiplier 10, amin 1e-10): the floor is the exact torch value (-100.0f), so
            // an all-silent clip stays constant (std 0: no normalisation)
            const float a = st ? dv1[r] : dv0[r];
            const float db = a <= 1e-10f ? -100.f : DB_PER_LOG2 * __builtin_amdgcn_logf(a);
            tile[m][wave * (FB / LW) + r] = db;
            lmax = fmaxf(lmax, db);
          }
        }
      }
    }
#else
        const int m = 64 * st + lane;
        if (m < n_mels) {
          float* om = out + ((int64_t)b * n_mels + m) * frames + fb0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (r >= nf_w) break;
            // AmplitudeToDB (multiplier 10, amin 1e-10): the floor is the exact torch value (-100.0f), so
            // an all-silent clip stays constant (std 0: no normalisation)
            const float a = acc[r];
            const float db = a <= 1e-10f ? -100.f : DB_PER_LOG2 * __builtin_amdgcn_logf(a);
            om[r] = db;
            lmax = fmaxf(lmax, db);
          }
        }
      }
    }
#endif
    lmax = wave_max(lmax);
    if (lane == 0) redmax[wave] = lmax;
    __syncthreads();
    if (t == 0) {
      float mx = redmax[0];
#pragma unroll
      for (int w = 1; w < LW; ++w) mx = fmaxf(mx, redmax[w]);
      blockmax[it] = mx;  // it = b * nbm + chunk
    }
#if LM_TILE
    {
      const float (*tile)[FB + 1] = reinterpret_cast<const float (*)[FB + 1]>(&pw[0][0][0]);
      const int nf = min(FB, frames - f0);
      float* ob = out + (int64_t)b * n_mels * frames + f0;
      for (int i = t; i < n_mels * FB; i += LNT) {
        const int m = i / FB, fi = i % FB;
#ifdef LM_NOSTORE
        if (fi < nf && tile[m][fi] == 12345.f) ob[(int64_t)m * frames + fi] = tile[m][fi];
#else
        if (fi < nf) ob[(int64_t)m * frames + fi] = tile[m][fi];
#endif
      }
    }
#endif
  }
}

// Pass 2: per clip slice -> partial (sum, sumsq) of the clamped dB values, in double.
__global__ __launch_bounds__(256) void clip_stats_kernel(const float* __restrict__ out, int64_t per_clip,
                                                         const float* __restrict__ blockmax, int nbm,
                                                         float top_db, double* __restrict__ partial) {
  const int b = blockIdx.y;
  __shared__ float smax;
  __shared__ double red[2][4];
  const int t = threadIdx.x;
  if (t < 64) {
    float m = -INFINITY;
    for (int i = t; i < nbm; i += 64) m = fmaxf(m, blockmax[(int64_t)b * nbm + i]);
    m = wave_max(m);
    if (t == 0) smax = m;
  }
  __syncthreads();
  const float floor_v = smax - top_db;
  const float* x = out + (int64_t)b * per_clip;
  double s = 0.0, ss = 0.0;  // sums of (v - amax): exact zero variance for a constant clip
  const bool vec = ((per_clip & 3) == 0);  // 16-B aligned clip rows (the B x 128 x 1379 case)
  const int64_t n4 = vec ? per_clip >> 2 : 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + t; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 q = reinterpret_cast<const float4*>(x)[i];
    const float e[4] = {q.x, q.y, q.z, q.w};
    float fs = 0.f, fss = 0.f;  // 4 terms in f32 (|v - amax| <= top_db), flushed to double
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = fmaxf(e[j], floor_v) - smax;
      fs += v;
      fss = fmaf(v, v, fss);
    }
    s += (double)fs;
    ss += (double)fss;
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + t; i < per_clip; i += (int64_t)gridDim.x * 256) {
    const double v = (double)fmaxf(x[i], floor_v) - (double)smax;
    s += v;
    ss += v * v;
  }
  s = wave_sum_d(s);
  ss = wave_sum_d(ss);
  if ((t & 63) == 0) { red[0][t >> 6] = s; red[1][t >> 6] = ss; }
  __syncthreads();
  if (t == 0) {
    partial[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    partial[((int64_t)b * gridDim.x + blockIdx.x) * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// Pass 3: clamp + (x - mean) / std_unbiased * target_std + target_mean, in place.
__global__ __launch_bounds__(256) void clip_norm_kernel(float* __restrict__ out, int64_t per_clip,
                                                        const float* __restrict__ blockmax, int nbm,
                                                        const double* __restrict__ partial, int nparts,
                                                        float top_db, int normalize, float tmean,
                                                        float tstd) {
  const int b = blockIdx.y;
  __shared__ float sp[3];
  const int t = threadIdx.x;
  if (t < 64) {
    float m = -INFINITY;
    for (int i = t; i < nbm; i += 64) m = fmaxf(m, blockmax[(int64_t)b * nbm + i]);
    m = wave_max(m);
    double s = 0.0, ss = 0.0;
    if (normalize) {
      for (int i = t; i < nparts; i += 64) {
        s += partial[((int64_t)b * nparts + i) * 2];
        ss += partial[((int64_t)b * nparts + i) * 2 + 1];
      }
      s = wave_sum_d(s);
      ss = wave_sum_d(ss);
    }
    if (t == 0) {
      sp[0] = m - top_db;
      const double n = (double)per_clip;
      const double dm = s / n;
      double var = (ss - n * dm * dm) / (n - 1.0);
      if (var < 0) var = 0;
      sp[1] = (float)((double)m + dm);
      sp[2] = (float)sqrt(var);
    }
  }
  __syncthreads();
  const float fl = sp[0], mean = sp[1], sd = sp[2];
  const bool do_norm = normalize && sd > 0.f;
  float* x = out + (int64_t)b * per_clip;
  const int64_t n4 = ((per_clip & 3) == 0) ? per_clip >> 2 : 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + t; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 q = reinterpret_cast<float4*>(x)[i];
    float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = fmaxf(e[j], fl);
      if (do_norm) v = (v - mean) / sd * tstd + tmean;
      e[j] = v;
    }
    reinterpret_cast<float4*>(x)[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + t; i < per_clip; i += (int64_t)gridDim.x * 256) {
    float v = fmaxf(x[i], fl);
    if (do_norm) v = (v - mean) / sd * tstd + tmean;
    x[i] = v;
  }
}

constexpr int NPARTS = 16;

}  // namespace

constexpr int64_t MEL_HDR_BYTES = 1024;                        // {nq[2], start[128]} (520 B) rounded
constexpr int64_t MEL_TAB_BYTES = (int64_t)2 * QMAX * 64 * 16;  // [2][QMAX][64] f32x4

extern "C" int64_t mia_logmel_workspace_bytes(int64_t B, int64_t frames) {
  const int64_t nbm = cdiv(frames, FB);
  return cdiv(B * nbm * 4, 16) * 16 + B * NPARTS * 2 * 8 + MEL_HDR_BYTES + MEL_TAB_BYTES + 16;
}

extern "C" int mia_logmel_fwd(const float* wav, int64_t B, int64_t T, int64_t ld_wav,
                              const MiaMelCfg* cfg, const float* window, const void* tw512,
                              const void* tw1024, const int32_t* band_start,
                              const int32_t* band_len, const int32_t* band_off,
                              const float* band_w, float* out, void* workspace,
                              mia_stream_t stream) {
  MIA_CHECK_ARG(wav && cfg && window && tw512 && tw1024 && band_start && band_len && band_off &&
                    band_w && out && workspace,
                "logmel: null pointer");
  MIA_CHECK_ARG(cfg->n_fft == NFFT && cfg->hop == HOP && cfg->win_length == WIN,
                "logmel: kernel is specialised for n_fft=1024, hop=160, win=400 (got %d/%d/%d)",
                cfg->n_fft, cfg->hop, cfg->win_length);
  MIA_CHECK_ARG(cfg->n_mels > 0 && cfg->n_mels <= NMEL_MAX, "logmel: n_mels must be in 1..128");
  MIA_CHECK_ARG(T > NFFT / 2 && T < (1ll << 30) && B > 0 && B < 65536 && ld_wav >= T,
                "logmel: bad shape B=%lld T=%lld", (long long)B, (long long)T);
  const int frames = (int)(1 + T / HOP);
  const int nbm = (int)cdiv(frames, FB);
  const int64_t nitems = B * nbm;
  MIA_CHECK_ARG(nitems < (1ll << 31), "logmel: too many frame chunks");
  float* blockmax = reinterpret_cast<float*>(workspace);
  double* partial = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + cdiv(B * nbm * 4, 16) * 16);
  int* mhdr = reinterpret_cast<int*>(partial + B * NPARTS * 2);
  f32x4* mtab = reinterpret_cast<f32x4*>(reinterpret_cast<char*>(mhdr) + MEL_HDR_BYTES);
  MelTables tb{window, reinterpret_cast<const f2*>(tw512), reinterpret_cast<const f2*>(tw1024),
               band_start, band_len, band_off, band_w};
  hipStream_t s = as_stream(stream);
  // three 4-wave workgroups per CU, persistent over the (clip, chunk) items
  const unsigned grid = (unsigned)std::min<int64_t>(nitems, LM_OCC * mia::cu_count());
  mel_mfma_table_kernel<<<1, 128, 0, s>>>(tb, cfg->n_mels, mhdr, mtab);
  MIA_LAUNCH_CHECK("mel_mfma_table");
  fft_mel_db_kernel<<<grid, LNT, 0, s>>>(wav, ld_wav, (int)T, frames, nbm, (int)nitems, cfg->n_mels, tb, mhdr, mtab,
                                        out, blockmax);
  MIA_LAUNCH_CHECK("fft_mel_db");
  const int64_t per_clip = (int64_t)cfg->n_mels * frames;
  if (cfg->normalize) {
    clip_stats_kernel<<<dim3(NPARTS, (unsigned)B), 256, 0, s>>>(out, per_clip, blockmax, nbm, cfg->top_db, partial);
    MIA_LAUNCH_CHECK("clip_stats");
  }
  clip_norm_kernel<<<dim3(NPARTS * 4, (unsigned)B), 256, 0, s>>>(out, per_clip, blockmax, nbm, partial, NPARTS,
                                                               cfg->top_db, cfg->normalize, cfg->target_mean,
                                                               cfg->target_std);
  MIA_LAUNCH_CHECK("clip_norm");
  return 0;
}
