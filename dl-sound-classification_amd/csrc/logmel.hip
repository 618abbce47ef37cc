// Fused batched log-mel for gfx950: ASTPreprocessor.preprocess (preprocessing.py:1013-1039).
//
// Per frame f (hop 160): the 400 windowed samples x[f*160-200+u]*hann[u] (reflect padding at the
// clip edges, = torch.stft center=True with the 400-tap window centred in n_fft=1024) are packed as
// 200 complex points z[n] = x[2n] + i x[2n+1], transformed by a 512-point Stockham radix-8 FFT in
// LDS (one wave per frame, 3 passes in one in-place buffer per wave), split into the 513 real-FFT
// bins, squared, reduced into the 128 htk mel bands (sparse band table staged in LDS:
// start/len/offset/weights), and converted to dB (10 log10 = 10 log10(2) * v_log_f32).
// Complex values are float2 vectors: every complex add is one v_pk_add_f32, every twiddle
// multiply one v_pk_mul_f32 + one v_pk_fma_f32 (op_sel swizzles, no moves); the Stockham buffer is
// XOR-swizzled (first-pass writes 1-2-way instead of 8-way bank conflicts).
// Persistent 4-wave workgroups (three per CU: 46 KB LDS, <= 168 VGPRs) walk (clip, 16-frame chunk)
// items: the 2,800-sample input segment of the NEXT chunk is loaded into registers (coalesced,
// reflect-padded) while this chunk's 16 frames are computed (4 per wave), then committed to LDS
// behind the chunk's tile store; the mel table, window taps and the twiddles of the three passes are
// read once per workgroup (the real-split twiddles derived per frame from one per lane).  Each mel
// band is widened to whole 16-B aligned groups of 4 bins with zero weights, so the band loop reads 4
// bins and 4 weights with one ds_read_b128 each; the weights sit in LDS interleaved by lane (row =
// group index, column = the lane's band), so a weight read is 64 consecutive 16-B chunks: the
// per-band layout made them data-dependent and bank-conflicting (fft_mel_db 0.636 -> 0.528 ms, bit-
// identical; padding the power spectrum the same way, or a wider Stockham swizzle: no further gain).
// The 128 x 16 dB tile is written back as 128 rows of 16 contiguous frames.  Measured at B = 256
// (tools/bench_logmel.py, tools/logmel_pmc.sh): ~400 VALU and ~110 LDS instructions per frame.
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
constexpr int SEG = (FB - 1) * HOP + WIN;  // 2800 samples
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


// Hand-off between the FFT stages of one wave through its own LDS buffer: every LDS operation of this wave has
// completed (lgkmcnt(0)) before the next is issued.  One wave's LDS operations execute in order, so the wave
// barrier alone already orders them; the drain makes each hand-off independent of that ordering and of any
// interruption of the wave between a stage's writes and the next stage's reads.
__device__ __forceinline__ void lds_handoff() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Sum over the 64 lanes, the same value in every lane and in every call (fixed order): DPP butterflies inside
// each 16-lane row (xor 1, xor 2, half-row mirror, row mirror), then the four row sums by readlane.
template <int CTRL> __device__ __forceinline__ float dpp_row_add(float v) {
  return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = dpp_row_add<0xB1>(v);   // quad_perm [1,0,3,2]
  v = dpp_row_add<0x4E>(v);   // quad_perm [2,3,0,1]
  v = dpp_row_add<0x141>(v);  // row_half_mirror
  v = dpp_row_add<0x140>(v);  // row_mirror
  const int b = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
  return (r0 + r1) + (r2 + r3);
}

// Per-frame self-check of the FFT (x = the 400 windowed samples at n = 0..399 of the 1024-point frame, X its DFT,
// P_k = |X_k|^2, F = sum_{k<1024} P_k = P_0 + P_512 + 2 sum_{k=1..511} P_k):
//  * Parseval: F = 1024 sum_n x_n^2;
//  * a checksum that must vanish: sum_{k<1024} (-1)^k P_k = 1024 sum_n x_n x_{(n + 512) mod 1024} = 0 (the
//    circular autocorrelation at lag 512 of a frame that is zero past n = 399).
// Both read only the power spectrum the band loop uses, so they cost no registers across the FFT.  f32 rounding
// measured on 2 400 windowed frames (noise, tones, chirps, DC, sparse, 1e4-loud; scipy single precision):
// Parseval <= 3.3e-7 relative, |checksum| <= 1.7e-7 F; the bounds leave two orders of magnitude for the
// radix-8 Stockham's own rounding and still see one typical bin's power move by 1 %.  A frame that fails is recomputed (up to LOGMEL_TRIES times); err words:
// [0] frames still failing, [1..3] the first one (clip + 1, frame, wave), [4] frames that passed on a retry,
// [5..7] the first of those.
constexpr float PARSEVAL_REL = 1e-4f;
constexpr float CHECKSUM_REL = 2e-5f;
constexpr int LOGMEL_TRIES = 3;

__device__ __forceinline__ void logmel_record(uint32_t* err, int slot, int clip, int frame, int wave) {
  atomicAdd(err + slot, 1u);
  if (atomicCAS(err + slot + 1, 0u, (uint32_t)clip + 1u) == 0u) {
    __hip_atomic_store(err + slot + 2, (uint32_t)frame, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(err + slot + 3, (uint32_t)wave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ int reflect_idx(int n, int T) {
  if (n < 0) n = -n;
  if (n >= T) n = 2 * (T - 1) - n;
  return n;
}

constexpr int MAX_WROWS = 12;  // interleaved weight rows staged in LDS (htk, 128 mels at n_fft 1024: 3 + 7)
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

__global__ __launch_bounds__(LNT) __attribute__((amdgpu_waves_per_eu(3, 3))) void fft_mel_db_kernel(const float* __restrict__ wav, int64_t ld, int T,
                                                            int frames, int nbm, int nitems, int n_mels,
                                                            MelTables tb, float* __restrict__ out,
                                                            float* __restrict__ blockmax, uint32_t* __restrict__ err,
                                                            int64_t fault_frame, int fault_tries) {
  __shared__ float seg[SEG];
  __shared__ f2 buf[LW][NC];             // one in-place Stockham buffer per wave
  __shared__ float tile[NMEL_MAX][FB + 1];
  // band weights interleaved by lane: row goff[pass] + i holds group i (4 bins) of band lane + 64 pass
  // for all 64 lanes, so the band loop's weight reads are 64 consecutive 16-B chunks (conflict-free)
  __shared__ f32x4 bwi[MAX_WROWS * 64];
  __shared__ int bs[NMEL_MAX], bl[NMEL_MAX], bo[NMEL_MAX];
  __shared__ int goff[NMEL_MAX / 64 + 1];
  __shared__ float redmax[LW];
  __shared__ f2 tw64[64];
  __shared__ int w_lds_s;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

  // mel band table into LDS (the per-band loops below then touch no global memory), each band widened
  // to whole 16-B aligned groups of 4 bins with zero weights, so the band loop reads 4 bins and their
  // 4 weights with one ds_read_b128 each (a table too large for LDS is read from global memory one
  // weight at a time)
  if (t == 0) {
    int rows = 0;
    for (int p = 0; p * 64 < n_mels; ++p) {
      goff[p] = rows;
      int g = 0;
      for (int m = 64 * p; m < n_mels && m < 64 * (p + 1); ++m) {
        const int ks = tb.band_start[m], len = tb.band_len[m];
        bs[m] = ks & ~3;                                  // 16-B aligned first bin
        bl[m] = ((ks & 3) + len + 3) & ~3;                // whole 4-bin groups
        g = max(g, bl[m] >> 2);
      }
      rows += g;
    }
    w_lds_s = rows <= MAX_WROWS;
  }
  __syncthreads();
  const bool w_lds = w_lds_s;  // block-uniform
  if (w_lds) {
    for (int p = 0; p * 64 < n_mels; ++p) {
      const int m = 64 * p + lane;
      if (m >= n_mels) continue;
      const int lead = tb.band_start[m] & 3, len = tb.band_len[m], src = tb.band_off[m];
      for (int i = wave; 4 * i < bl[m]; i += LW) {
        f32x4 w4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = 4 * i + j;
          w4[j] = (k >= lead && k < lead + len) ? tb.band_w[src + k - lead] : 0.f;
        }
        bwi[(goff[p] + i) * 64 + lane] = w4;
      }
    }
  } else {
    for (int m = t; m < n_mels; m += LNT) {
      bs[m] = tb.band_start[m];
      bl[m] = tb.band_len[m];
      bo[m] = tb.band_off[m];
    }
  }
  // loop-invariant per-lane constants: window taps, stage twiddles, real-split twiddles
  f2 win[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = 2 * (lane + 64 * r);
    win[r] = u < WIN ? f2{tb.window[u], tb.window[u + 1]} : f2{0.f, 0.f};
  }
  // stage-1 twiddles W512^(8 (lane % 8) r) = W64^((lane % 8) r): 64 distinct values, read from LDS (8 addresses
  // per read, broadcast); the stage-2 twiddles W512^(lane r) stay in registers
  if (t < 64) tw64[t] = tb.tw512[(NC / 64) * t];
  f2 tw2[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) tw2[r] = tb.tw512[(lane * (NC / 512) * r) & (NC - 1)];
  // real-split twiddles W1024^(lane + 64 q) = W1024^lane * W16^q (one per lane in registers)
  f2 tws0 = tb.tw1024[lane];

  // the reflect-padded input segment of chunk `it` into registers (coalesced 4-B loads)
  auto seg_load = [&](int it, float (&r)[SPT]) __attribute__((always_inline)) {
    const int b = it / nbm;
    const int s0 = (it - b * nbm) * FB * HOP - WIN / 2;
    const float* x = wav + (int64_t)b * ld;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int i = t + LNT * j;
      const int n = s0 + i;
      r[j] = (i < SEG && n >= -(NFFT / 2) && n < T + NFFT / 2) ? x[reflect_idx(n, T)] : 0.f;  // T > 512
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
    int attempt = 0;  // a frame whose FFT fails its self-check is recomputed (k is not advanced)
#pragma unroll 1
    for (int k = 0; k < FB / LW;) {
      const int fi = wave * (FB / LW) + k;
      if (f0 + fi >= frames) break;  // wave-uniform
      float pk[8];
      float pn = 0.f;
      // stage 0 (Ns = 1) reads z[j + 64 r] straight from the segment, z[n] = 0 for n >= 200
      float et = 0.f;  // this lane's share of sum_n x_n^2 (Parseval)
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
#pragma unroll
        for (int r = 0; r < 4; ++r) et = fmaf(v[r].x, v[r].x, fmaf(v[r].y, v[r].y, et));
        dft8(v);
#pragma unroll
        for (int r = 0; r < 8; ++r) d[swz(lane * 8 + r)] = v[r];
      }
      lds_handoff();
      // stages 1 (Ns = 8) and 2 (Ns = 64), in place: each stage's reads complete before its writes
      // (data dependence through dft8) and its writes complete before the next stage's reads (lds_handoff)
#pragma unroll
      for (int st = 1; st < 3; ++st) {
        const int Ns = st == 1 ? 8 : 64;
        f2 v[8];
        const int jm = lane % Ns;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const f2 a = d[swz(lane + 64 * r)];
          v[r] = r ? cmul(a, st == 1 ? tw64[((lane & 7) * r) & 63] : tw2[r]) : a;
        }
        dft8(v);
        lds_handoff();
        const int idxD = (lane / Ns) * Ns * 8 + jm;
#pragma unroll
        for (int r = 0; r < 8; ++r) d[swz(idxD + r * Ns)] = v[r];
        lds_handoff();
      }
      // test-only fault injection (MIA_LOGMEL_FAULT, see mia_logmel_fwd): one spectrum value of one frame
      // scaled by 1.05 on its first `fault_tries` attempts
      if (fault_tries > attempt && (int64_t)b * frames + f0 + fi == fault_frame) {
        if (lane == 5) d[swz(5 + 64 * 3)] *= 1.05f;
        lds_handoff();
      }
      // Z in d (natural order). Real-FFT split -> power P[k] (k = 0..512), kept in registers, then
      // written over the (consumed) spectrum as floats.  X[k] = 0.5 (e - i W^k o) with
      // e = Z[k] + conj(Z[N-k]), o = Z[k] - conj(Z[N-k]); |X|^2 = 0.25 |e - i W^k o|^2.
      asm volatile("" : "+v"(tws0));  // derived per frame (not hoisted: registers)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int kb = lane + 64 * q;  // bin
        const f2 zk = d[swz(kb)];
        const f2 zc = d[swz((NC - kb) & (NC - 1))] * f2{1.f, -1.f};
        const f2 tq = q ? cmul(tws0, W16[q]) : tws0;
        const f2 wo = cmul(tq, zk - zc);
        const f2 X = (zk + zc) - wo.yx * f2{-1.f, 1.f};  // e - i wo = (e.x + wo.y, e.y - wo.x) = 2 X[k]
        pk[q] = 0.25f * (X.x * X.x + X.y * X.y);
      }
      if (lane == 0) {
        const f2 z0 = d[0];
        const float xn = z0.x - z0.y;  // X[512]
        pn = xn * xn;
      }
      // self-check sums: bins 1..511 count twice (their mirror images 513..1023), bins 0 and 512 once;
      // (-1)^k = (-1)^lane for k = lane + 64 q
      float fs = pn - (lane == 0 ? pk[0] : 0.f);
#pragma unroll
      for (int q = 0; q < 8; ++q) fs = fmaf(2.f, pk[q], fs);
      const float e_t = wave_sum_dpp(et);
      const float e_f = wave_sum_dpp(fs);
      const float chk = wave_sum_dpp((lane & 1) ? -fs : fs);
      // absolute floors: a frame whose whole power is ~1e-20 maps every band below amin = 1e-10 (-100 dB) whatever
      // its rounding, and near-denormal samples (amplitude ~1e-21) must not read as a failed check
      // a non-finite frame (NaN/Inf samples, e_t from the inputs alone) carries NaN to the output as the
      // reference does; it is not a failed transform
      const bool ok = (fabsf(e_f * (1.f / NFFT) - e_t) <= fmaf(PARSEVAL_REL, e_t, 1e-24f) &&
                       fabsf(chk) <= fmaf(CHECKSUM_REL, e_f, 1e-20f)) || !isfinite(e_t);
      lds_handoff();  // the spectrum reads are done (P overwrites it below; a retry rewrites it)
      if (!ok && attempt + 1 < LOGMEL_TRIES) {  // wave-uniform
        ++attempt;
        continue;
      }
      if ((attempt > 0 || !ok) && err && lane == 0) logmel_record(err, ok ? 4 : 0, b, f0 + fi, wave);
      attempt = 0;
      float* P = reinterpret_cast<float*>(d);
#pragma unroll
      for (int q = 0; q < 8; ++q) P[lane + 64 * q] = pk[q];
      if (lane == 0) P[NC] = pn;
      lds_handoff();
      for (int m = lane; m < n_mels; m += 64) {
        const int ks = bs[m], kl = bl[m], off = bo[m];
        float acc = 0.f;
        if (w_lds) {
          const f32x4* wrow = bwi + goff[m >> 6] * 64 + lane;
          for (int i = 0; i < kl; i += 4) {  // zero weights outside the band (P stays finite there)
            const f32x4 w4 = wrow[(i >> 2) * 64];
            const f32x4 p4 = *reinterpret_cast<const f32x4*>(&P[ks + i]);
            acc = fmaf(p4[0], w4[0], acc);
            acc = fmaf(p4[1], w4[1], acc);
            acc = fmaf(p4[2], w4[2], acc);
            acc = fmaf(p4[3], w4[3], acc);
          }
        } else {
          for (int i = 0; i < kl; ++i) acc = fmaf(P[ks + i], tb.band_w[off + i], acc);
        }
        // AmplitudeToDB (multiplier 10, amin 1e-10): the floor is the exact torch value (-100.0f), so
        // an all-silent clip stays constant (std 0: no normalisation)
        const float db = acc <= 1e-10f ? -100.f : DB_PER_LOG2 * __builtin_amdgcn_logf(acc);
        tile[m][fi] = db;
        lmax = fmaxf(lmax, db);
      }
      lds_handoff();
      ++k;
    }
    lmax = wave_max(lmax);
    if (lane == 0) redmax[wave] = lmax;
    __syncthreads();
    if (t == 0) {
      float mx = redmax[0];
#pragma unroll
      for (int w = 1; w < LW; ++w) mx = fmaxf(mx, redmax[w]);
      blockmax[it] = mx;  // it = b * nbm + chunk
    }
    // tile store: rows of FB contiguous frames
    const int nf = min(FB, frames - f0);
    float* ob = out + (int64_t)b * n_mels * frames + f0;
    for (int i = t; i < n_mels * FB; i += LNT) {
      const int m = i / FB, fi = i % FB;
      if (fi < nf) ob[(int64_t)m * frames + fi] = tile[m][fi];
    }
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

extern "C" int64_t mia_logmel_workspace_bytes(int64_t B, int64_t frames) {
  const int64_t nbm = cdiv(frames, FB);
  return B * nbm * 4 + 16 + B * NPARTS * 2 * 8 + 16;
}

extern "C" int mia_logmel_fwd(const float* wav, int64_t B, int64_t T, int64_t ld_wav,
                              const MiaMelCfg* cfg, const float* window, const void* tw512,
                              const void* tw1024, const int32_t* band_start,
                              const int32_t* band_len, const int32_t* band_off,
                              const float* band_w, float* out, void* workspace, uint32_t* err,
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
  MelTables tb{window, reinterpret_cast<const f2*>(tw512), reinterpret_cast<const f2*>(tw1024),
               band_start, band_len, band_off, band_w};
  hipStream_t s = as_stream(stream);
  // Test-only fault injection for the FFT self-check: MIA_LOGMEL_FAULT="<clip>,<frame>,<tries>" corrupts that
  // frame's spectrum on its first <tries> attempts (tests/test_gpu_logmel.py); unset in every product run.
  int64_t fault_frame = -1;
  int fault_tries = 0;
  if (const char* f = getenv("MIA_LOGMEL_FAULT")) {
    long long c = -1, fr = -1;
    int tr = 0;
    if (sscanf(f, "%lld,%lld,%d", &c, &fr, &tr) == 3 && c >= 0 && fr >= 0) {
      fault_frame = c * frames + fr;
      fault_tries = tr;
    }
  }
  // three 4-wave workgroups per CU (LDS 43 KB, 152 VGPRs), persistent over the (clip, chunk) items
  const unsigned grid = (unsigned)std::min<int64_t>(nitems, 3 * mia::cu_count());
  fft_mel_db_kernel<<<grid, LNT, 0, s>>>(wav, ld_wav, (int)T, frames, nbm, (int)nitems, cfg->n_mels, tb, out,
                                        blockmax, err, fault_frame, fault_tries);
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
