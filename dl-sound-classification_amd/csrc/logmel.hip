// Fused batched log-mel for gfx950: ASTPreprocessor.preprocess (preprocessing.py:1013-1039).
//
// Per frame f (hop 160): the 400 windowed samples x[f*160-200+u]*hann[u] (reflect padding at the
// clip edges, = torch.stft center=True with the 400-tap window centred in n_fft=1024) are packed as
// 200 complex points z[n] = x[2n] + i x[2n+1], transformed by a 512-point Stockham radix-8 FFT in
// LDS (one wave per frame, 3 passes in one in-place buffer per wave; window taps and twiddles held in
// registers), split into the 513 real-FFT bins, squared, reduced into the 128 htk mel bands (sparse
// band table staged in LDS: start/len/offset/weights), and converted to dB (f32 log10).
// A block owns 16 consecutive frames of one clip: the 2,800-sample input segment is read from HBM
// once with coalesced loads into LDS, and the 128 x 16 dB tile is written back as 128 rows of
// 16 contiguous frames.  Per-clip top_db clamp + mean / unbiased-std normalisation need the clip
// max first, so two light passes follow (stats over the dB tensor, which stays in the 256 MB
// Infinity Cache at batch 256, then an in-place normalise).
#include "common.h"

namespace {

constexpr int FB = 16;          // frames per block (3 blocks per CU by LDS)
constexpr int NFFT = 1024;
constexpr int NC = 512;         // complex FFT size
constexpr int HOP = 160;
constexpr int WIN = 400;
constexpr int NMEL_MAX = 128;
constexpr int SEG = (FB - 1) * HOP + WIN;  // 2800 samples

struct MelTables {
  const float* window;   // [WIN]
  const float2* tw512;   // [512] exp(-2 pi i q / 512)
  const float2* tw1024;  // [513] exp(-2 pi i k / 1024)
  const int* band_start; // [n_mels]
  const int* band_len;   // [n_mels]
  const int* band_off;   // [n_mels] offset into band_w
  const float* band_w;   // [nnz]
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul_mi(float2 a) { return make_float2(a.y, -a.x); }  // a * (-i)

// In-register DFT8 (natural-order output), W8 = exp(-2 pi i / 8).
__device__ __forceinline__ void dft8(float2 (&v)[8]) {
  const float s = 0.70710678118654752f;
  float2 a0 = cadd(v[0], v[4]), a4 = csub(v[0], v[4]);
  float2 a1 = cadd(v[1], v[5]), t5 = csub(v[1], v[5]);
  float2 a2 = cadd(v[2], v[6]), t6 = csub(v[2], v[6]);
  float2 a3 = cadd(v[3], v[7]), t7 = csub(v[3], v[7]);
  float2 a5 = make_float2(s * (t5.x + t5.y), s * (t5.y - t5.x));    // * W8^1 = s(1 - i)
  float2 a6 = cmul_mi(t6);                                          // * W8^2 = -i
  float2 a7 = make_float2(s * (-t7.x + t7.y), s * (-t7.y - t7.x));  // * W8^3 = s(-1 - i)
  float2 b0 = cadd(a0, a2), b2 = csub(a0, a2);
  float2 b1 = cadd(a1, a3), b3 = cmul_mi(csub(a1, a3));
  float2 b4 = cadd(a4, a6), b6 = csub(a4, a6);
  float2 b5 = cadd(a5, a7), b7 = cmul_mi(csub(a5, a7));
  v[0] = cadd(b0, b1); v[4] = csub(b0, b1);
  v[2] = cadd(b2, b3); v[6] = csub(b2, b3);
  v[1] = cadd(b4, b5); v[5] = csub(b4, b5);
  v[3] = cadd(b6, b7); v[7] = csub(b6, b7);
}

__device__ __forceinline__ int reflect_idx(int n, int T) {
  if (n < 0) n = -n;
  if (n >= T) n = 2 * (T - 1) - n;
  return n;
}

constexpr int MAX_NNZ = 1536;  // band weights staged in LDS (htk, 128 mels at n_fft 1024: 1,008)

__global__ __launch_bounds__(256) void fft_mel_db_kernel(const float* __restrict__ wav, int64_t ld, int T,
                                                         int frames, int n_mels, MelTables tb,
                                                         float* __restrict__ out, float* __restrict__ blockmax) {
  __shared__ float seg[SEG];
  __shared__ float2 buf[4][NC];          // one in-place Stockham buffer per wave
  __shared__ float tile[NMEL_MAX][FB + 1];
  __shared__ float bw[MAX_NNZ];
  __shared__ int bs[NMEL_MAX], bl[NMEL_MAX], bo[NMEL_MAX];
  __shared__ float redmax[4];

  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FB;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float* x = wav + (int64_t)b * ld;

  // mel band table into LDS (the per-band loops below then touch no global memory)
  const int nnz = tb.band_off[n_mels - 1] + tb.band_len[n_mels - 1];
  const bool w_lds = nnz <= MAX_NNZ;  // block-uniform
  if (w_lds)
    for (int i = t; i < nnz; i += 256) bw[i] = tb.band_w[i];
  for (int m = t; m < n_mels; m += 256) { bs[m] = tb.band_start[m]; bl[m] = tb.band_len[m]; bo[m] = tb.band_off[m]; }
  // coalesced segment load with reflect padding
  const int s0 = f0 * HOP - WIN / 2;
  for (int i = t; i < SEG; i += 256) {
    const int n = s0 + i;
    float v = 0.f;
    if (n >= -(NFFT / 2) && n < T + NFFT / 2) v = x[reflect_idx(n, T)];  // valid reflect range (T > 512)
    seg[i] = v;
  }
  // loop-invariant per-lane constants: window taps, stage twiddles, real-split twiddles
  float2 win[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = 2 * (lane + 64 * r);
    win[r] = u < WIN ? make_float2(tb.window[u], tb.window[u + 1]) : make_float2(0.f, 0.f);
  }
  float2 tw1[8], tw2[8], tws[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    tw1[r] = tb.tw512[((lane % 8) * (NC / 64) * r) & (NC - 1)];
    tw2[r] = tb.tw512[(lane * (NC / 512) * r) & (NC - 1)];
    tws[r] = tb.tw1024[lane + 64 * r];
  }
  __syncthreads();

  const float* bwp = w_lds ? bw : tb.band_w;
  float lmax = -INFINITY;
  float2* d = buf[wave];
  for (int fi = wave; fi < FB; fi += 4) {
    const int f = f0 + fi;
    if (f >= frames) break;  // wave-uniform
    // stage 0 (Ns = 1) reads z[j + 64 r] straight from the segment, z[n] = 0 for n >= 200
    {
      float2 v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int n = lane + 64 * r;
        if (r < 4 && n < WIN / 2) {
          const float2 xv = *reinterpret_cast<const float2*>(&seg[fi * HOP + 2 * n]);
          v[r] = make_float2(xv.x * win[r].x, xv.y * win[r].y);
        } else {
          v[r] = make_float2(0.f, 0.f);
        }
      }
      dft8(v);
#pragma unroll
      for (int r = 0; r < 8; ++r) d[lane * 8 + r] = v[r];
    }
    wave_sync();
    // stages 1 (Ns = 8) and 2 (Ns = 64), in place: every lane's reads land before any lane's writes
    // (one wave, program order), so the single buffer needs no ping-pong
#pragma unroll
    for (int st = 1; st < 3; ++st) {
      const int Ns = st == 1 ? 8 : 64;
      float2 v[8];
      const int jm = lane % Ns;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        float2 a = d[lane + 64 * r];
        if (r) a = cmul(a, st == 1 ? tw1[r] : tw2[r]);
        v[r] = a;
      }
      dft8(v);
      wave_sync();
      const int idxD = (lane / Ns) * Ns * 8 + jm;
#pragma unroll
      for (int r = 0; r < 8; ++r) d[idxD + r * Ns] = v[r];
      wave_sync();
    }
    // Z in d (natural order). Real-FFT split -> power P[k] (k = 0..512), kept in registers, then
    // written over the (consumed) spectrum as floats
    float pk[8];
    float pn = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = lane + 64 * q;
      const float2 zk = d[k];
      const float2 zc = d[(NC - k) & (NC - 1)];
      const float2 zcj = make_float2(zc.x, -zc.y);
      const float2 e = cadd(zk, zcj);          // 2 * even part
      const float2 o = csub(zk, zcj);          // 2i * odd part (before twiddle)
      // X[k] = 0.5*(e - i W^k o)
      const float2 wo = cmul(tws[q], o);
      const float2 X = make_float2(0.5f * (e.x + wo.y), 0.5f * (e.y - wo.x));
      pk[q] = X.x * X.x + X.y * X.y;
    }
    if (lane == 0) {
      const float2 z0 = d[0];
      const float xn = z0.x - z0.y;  // X[512]
      pn = xn * xn;
    }
    wave_sync();
    float* P = reinterpret_cast<float*>(d);
#pragma unroll
    for (int q = 0; q < 8; ++q) P[lane + 64 * q] = pk[q];
    if (lane == 0) P[NC] = pn;
    wave_sync();
    for (int m = lane; m < n_mels; m += 64) {
      const int ks = bs[m], kl = bl[m], off = bo[m];
      float acc = 0.f;
      for (int i = 0; i < kl; ++i) acc = fmaf(P[ks + i], bwp[off + i], acc);
      // AmplitudeToDB (multiplier 10, amin 1e-10): the floor is the exact torch value (-100.0f; f32
      // log10f is 1 ulp low there), so an all-silent clip stays constant (std 0: no normalisation)
      const float db = acc <= 1e-10f ? -100.f : 10.f * log10f(acc);
      tile[m][fi] = db;
      lmax = fmaxf(lmax, db);
    }
    wave_sync();
  }
  lmax = wave_max(lmax);
  if (lane == 0) redmax[wave] = lmax;
  __syncthreads();
  if (t == 0) {
    blockmax[(int64_t)b * gridDim.x + blockIdx.x] =
        fmaxf(fmaxf(redmax[0], redmax[1]), fmaxf(redmax[2], redmax[3]));
  }
  // coalesced tile store: rows of FB contiguous frames
  const int nf = min(FB, frames - f0);
  float* ob = out + (int64_t)b * n_mels * frames + f0;
  for (int i = t; i < n_mels * FB; i += 256) {
    const int m = i / FB, fi = i % FB;
    if (fi < nf) ob[(int64_t)m * frames + fi] = tile[m][fi];
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
  float* blockmax = reinterpret_cast<float*>(workspace);
  double* partial = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + cdiv(B * nbm * 4, 16) * 16);
  MelTables tb{window, reinterpret_cast<const float2*>(tw512), reinterpret_cast<const float2*>(tw1024),
               band_start, band_len, band_off, band_w};
  hipStream_t s = as_stream(stream);
  fft_mel_db_kernel<<<dim3(nbm, (unsigned)B), 256, 0, s>>>(wav, ld_wav, (int)T, frames, cfg->n_mels, tb, out,
                                                         blockmax);
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
