/*
 * miaudio.h — C ABI of libmiaudio.so, the MI355X (gfx950) kernels behind the
 * youssefg7/dl-sound-classification training hot path:
 *   batched waveform -> STFT/log-mel -> EnvNet-v2 | AST fwd+bwd -> clip + Adam.
 *
 * The reference is pure Python and binds no native library; its "plugin API" is
 * Hydra `_target_` instantiation of nn.Modules (configs/model/<name>.yaml:10) driven by
 * LitClassifier (src/training/engine.py:67-310).  Each entry point below replaces a
 * third-party op the reference reaches through PyTorch on that path; the comment
 * on each names the reference call site (file:line, relative to the reference root).
 * The Python side binds these with ctypes.
 *
 * Conventions:
 *  - extern "C", plain pointers and sizes; no torch types.
 *  - Stream-ordered: every call enqueues on `stream` (a hipStream_t) and never syncs.
 *  - Caller owns ALL memory (inputs, outputs, workspaces); the library allocates nothing.
 *  - Return 0 on success, a negative code on error; mia_last_error_string() explains.
 *  - Reentrant and stateless (error string is thread-local).
 *  - Activations are channels-last (NHWC) unless stated; dtype codes MIA_F32/MIA_BF16.
 */
#ifndef MIAUDIO_H
#define MIAUDIO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mia_stream_t; /* hipStream_t */

enum { MIA_F32 = 0, MIA_BF16 = 1, MIA_U8 = 2 };
#define MIA_RM_DROP (-1) /* MiaEpilogue.rm_offset sentinel: drop-mode row map */
enum { MIA_OP_DENSE = 0, MIA_OP_CONV = 1, MIA_OP_CONVROW = 2 };
enum { MIA_LAYOUT_KC = 0, MIA_LAYOUT_RC = 1 };
enum { MIA_PRE_NONE = 0, MIA_PRE_AFFINE = 1, MIA_PRE_AFFINE_RELU = 2, MIA_PRE_GELU = 3 };
enum { MIA_ACT_NONE = 0, MIA_ACT_RELU = 1, MIA_ACT_GELU = 2, MIA_DACT_NZ = 3, MIA_DACT_GELU = 4,
       MIA_ACT_ADD_AUX = 5, MIA_ACT_GELU_SAVE = 6, MIA_ACT_GELU_SAVE_D = 7, MIA_DACT_MUL = 8 };

/* A GEMM operand = a logical 2-D source S[i][j] whose j axis is contiguous in memory.
 *  DENSE   : S[i][j] = ptr[i*ld + j], i < rows, j < cols (zero outside).
 *  CONV    : im2col of an NHWC tensor (n,h,w,c), c % 8 == 0:
 *            i = output pixel (b, y, x) over n*oh*ow, j = (ky, kx, ci) over kh*kw*c,
 *            S[i][j] = in[b][y*sh+ky-ph][x*sw+kx-pw][ci] (zero padding).
 *  CONVROW : same as CONV but for (kw*c) % 8 == 0 with pw == 0 (c may be 1 or 2):
 *            one chunk = 8 consecutive (kx, ci) of one kernel row.
 * layout KC: the operand's GEMM k axis is j (A: M x K stored [M][K]; B: stored [N][K]).
 * layout RC: the operand's GEMM k axis is i (A stored [K][M]; B stored [K][N]).
 * pre: optional per-channel transform applied while loading (BN affine [+ReLU]
 *      of the previous layer, or GELU), channel = j (DENSE) / ci (CONV). */
typedef struct MiaOperand {
  const void* ptr;
  int32_t kind, dtype, layout, pre;
  int64_t rows, cols, ld;
  int32_t n, h, w, c;
  int32_t oh, ow, kh, kw, sh, sw, ph, pw;
  const float* pre_scale;
  const float* pre_shift;
} MiaOperand;

/* Epilogue of C[m][n] = alpha * sum_k A[m][k] B[k][n]:
 *   v = alpha*acc (+ bias[n]); act; (v += old C if accumulate); store as dtype at
 *   ptr[prow(m)*ldc + n] with prow(m) = m if rm_inner == 0 else
 *   (m / rm_inner)*rm_outer + (m % rm_inner)*rm_istride + rm_offset.
 *   rm_offset == MIA_RM_DROP (drop mode; plain / bias / ReLU epilogues, rm_istride 1): prow(m) =
 *   (m / rm_inner)*rm_outer + m % rm_inner and rows with m % rm_inner >= rm_outer are not stored -- a (1, 2)
 *   conv computed over every input pixel (rm_inner = w) stores its w - 1 valid columns per row.
 *   DACT_NZ  : v *= (aux[m][n] != 0) * act_scale   (ReLU+dropout backward from saved output)
 *   DACT_GELU: v *= gelu'(aux[m][n])                (GELU backward from saved pre-activation)
 *   ADD_AUX  : v += aux[m][n]                       (residual connection into a new tensor)
 *   GELU_SAVE: aux[m][n] = v; v = gelu(v)          (MLP fc1: keeps the pre-activation for the backward)
 *   GELU_SAVE_D: aux[m][n] = gelu'(v); v = gelu(v) (MLP fc1: keeps the derivative the backward needs)
 *   DACT_MUL : v *= aux[m][n]                       (GELU backward from the saved derivative) */
typedef struct MiaEpilogue {
  void* ptr;
  int32_t dtype, act, accumulate, aux_dtype;
  int64_t ldc;
  int64_t rm_inner, rm_outer, rm_istride, rm_offset;  /* rm_offset MIA_RM_DROP: drop mode (above) */
  const float* bias;
  const void* aux;
  int64_t ldaux;
  float alpha, act_scale;
  /* Optional (NULL = off): per 128x128 output tile (bm, bn), slot bm * ceil(N/128) + bn receives the
   * sum of squares of the values the GEMM stored there (double), for a gradient-clip norm that does
   * not re-read the output.  Plain f32 output only (no act / bias / accumulate / row map, alpha 1). */
  double* sqsum;
  /* Optional (NULL = off): colsum[n] = sum over the M rows of the stored output column n (f32 result,
   * summed from the stored -- for bf16, rounded -- values): the bias gradient of the linear whose dy
   * this output is.  The 256x256 kernel (path 7) sums it in its dGELU epilogue (timm fc1 behind the
   * fc2 dgrad); any other path gets a column-sum pass over the output.  Row-major output, no
   * accumulate / row map / sqsum.  Needs the workspace of mia_gemm_workspace_bytes_ex. */
  float* colsum;
  /* Optional (NULL = off): an MX-fp8 copy of the stored bf16 output -- mx_q e4m3 [M][N] (row stride N
   * bytes), mx_scales [M][N / 32] E8M0 (mia_mx_quantize's format, of the rounded bf16 values) -- the next
   * MX GEMM's A operand, written in the same epilogue (fp8-mixed: fc1's gelu(u) for fc2).  256x256
   * kernels (path 7, mia_gemm_mxfp8) with a plain / GELU / GELU_SAVE bf16 output, ldc == N, N % 32 == 0. */
  void* mx_q;
  void* mx_scales;
  /* Optional (NULL = off): a_colsum[m] = sum over k of a k-by-m (MIA_LAYOUT_RC) dense A operand -- the bias
   * gradient of the linear whose weight gradient dW = dy^T x this GEMM is (A = dy), summed inside the
   * 256x256 kernel's main loop from the A fragments it already reads (split-K partials reduced in a fixed
   * order); any other path gets a column-sum pass over A.  Needs the workspace of mia_gemm_workspace_bytes_ex. */
  float* a_colsum;
} MiaEpilogue;

/* Implicit-GEMM on MFMA (bf16: v_mfma_f32_32x32x16_bf16 / 16x16x32; f32: v_mfma_f32_32x32x2_f32).
 * Replaces cuDNN conv2d fwd/dgrad/wgrad for every EnvNetV2 conv (envnet_v2.py:15,19,31,34),
 * the nn.Linear layers (envnet_v2.py:51,55,59; ast.py:40 and timm Block qkv/proj/fc1/fc2,
 * ast.py:38,60-61) and the AST patch-embed conv (ast.py:30,55).  Every path is a hand-written gfx950
 * kernel; the kernel choice is a fixed function of the shapes, layouts and epilogue (no run-time
 * timing), the library keeps no memory and never synchronises with the host.
 * Workspace: mia_gemm_workspace_bytes_ex(...) bytes for exactly this call (split-K slabs, column-sum
 * partials); mia_gemm_workspace_bytes(M, N, split_k) is the split-K part alone of paths 0-5. */
int64_t mia_gemm_workspace_bytes(int64_t M, int64_t N, int32_t split_k);
/* MX-fp8 (OCP e4m3fn elements, one E8M0 scale byte per 32 consecutive K-elements) for the AST block
 * linears' forward GEMMs under trainer.precision=fp8-mixed (north_star config 5; the reference has no fp8
 * path: it replaces the bf16 nn.Linear of timm's Block, ast.py:38,60-61, inside autocast).
 * mia_mx_quantize: x [rows][cols] (bf16 or f32, row stride ldx elements, cols % 32 == 0) -> q [rows][cols]
 * e4m3 bytes (row stride ldq bytes) and scales [rows][cols / 32] bytes.  OCP MX rule: e = floor(log2(amax
 * of the 32-block)) - 8, clamped to [-127, 127], scale byte e + 127; elements x * 2^-e saturated to +-448
 * and rounded to nearest even; an all-zero block gets scale byte 0.
 * mia_gemm_mxfp8: C[M][N] = epilogue(A[M][K] B[N][K]^T) with A, B e4m3 (row strides lda / ldb bytes,
 * multiples of 16, K % 128 == 0) and their scale arrays ([M][K/32], [N][K/32] bytes, 4-B aligned); the
 * epilogue is mia_gemm's dense one restricted to plain / bias / GELU / GELU_SAVE (bf16 out) and the f32
 * residual add (MIA_ACT_ADD_AUX); f32 accumulation; no workspace, no host sync. */
int mia_mx_quantize(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ldx, void* q, int64_t ldq,
                    void* scales, mia_stream_t stream);
int mia_gemm_mxfp8(const void* a, const void* a_scales, int64_t lda, const void* b, const void* b_scales, int64_t ldb,
                   const MiaEpilogue* E, int64_t M, int64_t N, int64_t K, mia_stream_t stream);
/* The fp8-mixed backward-data GEMMs (dX = dY W on MX operands; round 5):
 * mia_mx_quantize_t: the MX copy of a transpose, q [cols][rows] = x [rows][cols]^T with one scale per 32
 * consecutive rows (rows % 32 == 0; q row stride ldq bytes, scales [cols][rows / 32]) -- the B operand W^T
 * of a weight stored W[out][in], quantised from the f32 master each step like the forward's W.
 * mia_gemm_mxfp8_ex: mia_gemm_mxfp8 that also takes the fc2 backward-data epilogue (MIA_DACT_MUL: x the
 * saved gelu'(u), with the column sums of the stored values into E->colsum -- fc1's bias gradient), whose
 * partials need `workspace` of mia_gemm_mxfp8_workspace_bytes(M, N, colsum != 0) bytes (0 without). */
int mia_mx_quantize_t(const void* x, int32_t x_dtype, int64_t rows, int64_t cols, int64_t ldx, void* q, int64_t ldq,
                      void* scales, mia_stream_t stream);
int64_t mia_gemm_mxfp8_workspace_bytes(int64_t M, int64_t N, int32_t colsum);
int mia_gemm_mxfp8_ex(const void* a, const void* a_scales, int64_t lda, const void* b, const void* b_scales,
                      int64_t ldb, const MiaEpilogue* E, int64_t M, int64_t N, int64_t K, void* workspace,
                      mia_stream_t stream);
/* Quantise-on-store producers of the fp8-mixed AST forward (the MX GEMMs' A operands without a
 * separate pass; both also write their usual bf16 output, which the backward keeps using):
 * mia_layernorm_fwd_mx: mia_layernorm_fwd with a bf16 y plus q [rows][D] e4m3 and scales [rows][D/32]
 *   (D % 64 == 0, D <= 768) -- timm Block norm1 / norm2 feeding qkv / fc1;
 * mia_attn_fwd_mx: mia_attn_fwd (bf16) plus the output as q8 [B*N][H*64] e4m3 and s8 [B*N][H*2] --
 *   feeding proj.  Both quantise the rounded bf16 values exactly as mia_mx_quantize would. */
int mia_layernorm_fwd_mx(const void* x, int32_t xdtype, const float* gamma, const float* beta, void* y, void* q,
                         void* scales, float* mean, float* rstd, int64_t rows, int32_t D, float eps,
                         mia_stream_t stream);
int mia_attn_fwd_mx(const void* qkv, void* out, float* lse, void* q8, void* s8, int32_t B, int32_t N, int32_t H,
                    float scale, mia_stream_t stream);

int64_t mia_gemm_workspace_bytes_ex(const MiaOperand* A, const MiaOperand* B, const MiaEpilogue* E, int64_t M,
                                    int64_t N, int64_t K, int32_t compute_dtype, int32_t split_k);
/* number of MiaEpilogue.sqsum slots (doubles) of an M x N output */
int64_t mia_gemm_sqsum_slots(int64_t M, int64_t N);
/* Deferred weight gradient of a wide nn.Linear (EnvNet-v2 FC1, envnet_v2.py:51: dW = dY^T X, 4096 x 84480
 * f32 = 1.38 GB per step), so the gradient is never written: in the backward mia_gemm_sqsum_only leaves only
 * its per-tile sums of squares (mia_gemm_sqsum_slots(M, N) doubles, the clip norm's share), and after the
 * norm is known mia_gemm_adam recomputes the product (K = the batch: cheap) and applies torch's
 * single-tensor Adam to the parameter rows in the epilogue -- exactly mia_clip_adam's arithmetic, the
 * clip coefficient read from `coef` (mia_clip_adam's workspace + mia_adam_coef_offset(ntensors)), the
 * bias corrections as lr / bc1 and sqrt(bc2); p / m / v (and the optional bf16 shadow) rows of stride ld.
 * Full 128 x 128 tiles (M, N multiples of 128), bf16 dense operands, K a multiple of 64.  Replaces the
 * gradient write + re-read of the Linear backward + torch.optim.Adam (engine.py:299-310). */
int mia_gemm_sqsum_only(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K, double* sqsum,
                        mia_stream_t stream);
int mia_gemm_adam(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K, float* param,
                  float* exp_avg, float* exp_avg_sq, void* shadow_bf16, int64_t ld, const float* coef,
                  float lr_over_bc1, float bc2_sqrt, float beta1, float beta2, float eps, float weight_decay,
                  mia_stream_t stream);
int mia_gemm(const MiaOperand* A, const MiaOperand* B, const MiaEpilogue* E, int64_t M,
             int64_t N, int64_t K, int32_t compute_dtype, int32_t split_k, void* workspace,
             mia_stream_t stream);
/* Which kernel mia_gemm runs for these operands: 0 = implicit-GEMM tile kernel, 1 = row-window
 * direct conv (bf16 compute, stride (1,1|2), C in {32,64}, N in {32,64}: the EnvNet-v2 8x8 trunk
 * convs, the frontend conv2 and their dgrads), 2 = row-window weight gradient (A = dY as RC,
 * B = the conv input as RC, M = Cout in {32,64}, split_k >= 2 partial slabs: blocks = KH x split),
 * 3 = single-channel tap weight gradient (conv1 pair view / 1-channel 8x8 conv3, M = 32, N = 64,
 * split_k >= 2 blocks), 4 = single-channel tap conv forward (the same two convs, N = 32, K = 64),
 * 5 = dense bf16 GEMM with LDS-DMA staging, 128x128 tiles (bf16 DENSE operands, K % 64 == 0,
 * M, N >= 64: EnvNet FC layers, small token counts), 7 = dense bf16 GEMM, 256x256 tiles, 8 waves
 * (M >= 1024 rows, N >= 256: the AST block linears at training batch sizes; its own split-K for the
 * weight gradients, fused bias / GELU / GELU_SAVE / residual / dGELU + colsum epilogues).  Path 7
 * is taken only for an epilogue it implements; E may be NULL here (plain epilogue assumed). */
int mia_gemm_path(const MiaOperand* A, const MiaOperand* B, int64_t M, int64_t N, int64_t K,
                  int32_t compute_dtype, int32_t split_k);

/* Fused log-mel: frame gather + 1024-pt real FFT (LDS) + |X|^2 + htk mel (sparse bands)
 * + 10log10 + per-clip top_db clamp + per-clip mean/unbiased-std normalisation.
 * Replaces ASTPreprocessor.preprocess (src/datasets/preprocessing.py:1013-1039,
 * torchaudio MelSpectrogram/AmplitudeToDB at :988-998).
 * wav: (B, T) f32 rows of stride ld_wav; out: (B, n_mels, frames) f32, frames = 1 + T/hop.
 * Constant device tables built once by the caller: window[win_length] (periodic Hann),
 * tw512[512] / tw1024[513] complex twiddles exp(-2 pi i q/512), exp(-2 pi i k/1024) as float2,
 * mel bands: band_start/band_len/band_off[n_mels] into band_w[nnz] (htk filterbank, norm=None).
 * workspace: mia_logmel_workspace_bytes(B, frames) bytes.
 * err: NULL, or 8 caller-owned u32 words, zero before the first call and never cleared by the library.
 * Every frame's FFT is checked in the kernel (Parseval, and sum_k (-1)^k X_k = 1024 x_512 = 0) and
 * recomputed when a check fails: err[0] counts frames that still failed after 3 tries (their output is
 * invalid), err[1..3] = (clip + 1, frame, wave) of the first; err[4] counts frames that passed on a retry,
 * err[5..7] the first of those. */
typedef struct MiaMelCfg {
  int32_t sample_rate, n_fft, win_length, hop, n_mels, normalize;
  float top_db, target_mean, target_std;
} MiaMelCfg;
int64_t mia_logmel_workspace_bytes(int64_t B, int64_t frames);
int mia_logmel_fwd(const float* wav, int64_t B, int64_t T, int64_t ld_wav, const MiaMelCfg* cfg,
                   const float* window, const void* tw512, const void* tw1024,
                   const int32_t* band_start, const int32_t* band_len, const int32_t* band_off,
                   const float* band_w, float* out, void* workspace, uint32_t* err, mia_stream_t stream);

/* BatchNorm (train mode) — nn.BatchNorm2d after every conv (envnet_v2.py:16,20,32,35).
 * x: (P, C) channels-last.  stats out: mean[C], invstd[C]; running stats updated with
 * momentum and the unbiased variance; scale = gamma*invstd, shift = beta - mean*scale.
 * partial: workspace of mia_bn_partial_bytes(P, C) bytes. */
int64_t mia_bn_partial_bytes(int64_t P, int32_t C);
int mia_bn_fwd_stats(const void* x, int32_t dtype, int64_t P, int32_t C, const float* gamma,
                     const float* beta, float* running_mean, float* running_var, float momentum,
                     float eps, int32_t training, float* mean, float* invstd, float* scale,
                     float* shift, void* partial, mia_stream_t stream);
/* ReLU + BN backward reductions: dz = dact * (scale*x+shift > 0) (in place allowed; dz may be
 * NULL when mia_bn_relu_bwd_apply recomputes the mask), dgamma = sum dz*xhat, dbeta = sum dz
 * (written, not accumulated).  Replaces autograd of nn.ReLU + nn.BatchNorm2d (envnet_v2.py:16-17). */
int mia_bn_relu_bwd_reduce(const void* dact, void* dz, const void* x, int32_t dtype, int64_t P,
                           int32_t C, const float* scale, const float* shift, const float* mean,
                           const float* invstd, float* dgamma, float* dbeta, void* partial,
                           mia_stream_t stream);
/* dx = gamma*invstd*(dz - dbeta/P - xhat*dgamma/P); optional dbias[c] = sum_rows dx (the
 * gradient of the conv bias that precedes the BN, envnet_v2.py:15 bias=True). */
int mia_bn_bwd_apply(const void* dz, const void* x, void* dx, int32_t dtype, int64_t P, int32_t C,
                     const float* gamma, const float* mean, const float* invstd,
                     const float* dgamma, const float* dbeta, float* dbias, void* partial,
                     mia_stream_t stream);
/* mia_bn_bwd_apply with the ReLU mask recomputed from x: dz = dact * (scale*x+shift > 0) is never
 * materialised (dact = gradient of relu(bn(x))). */
int mia_bn_relu_bwd_apply(const void* dact, const void* x, void* dx, int32_t dtype, int64_t P, int32_t C,
                          const float* gamma, const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* dgamma, const float* dbeta, float* dbias,
                          void* partial, mia_stream_t stream);

/* Max-pool of relu(scale*x+shift) — nn.MaxPool2d (envnet_v2.py:23,37) fused with the
 * preceding BN+ReLU.  x: (n, h, w, c) NHWC; window (kh,kw) == stride, floor mode.
 * out layout: 0 = NHWC (n,oh,ow,c); 1 = "transposed frontend" (n, c, ow) for oh == 1
 * (envnet_v2.py:82 transpose(1,2)); 2 = NCHW flattened (n, c, oh, ow) (classifier Flatten).
 * argmax: (n, oh, ow, c) u8 window offset of the max. */
int mia_pool_fwd(const void* x, int32_t dtype, int32_t n, int32_t h, int32_t w, int32_t c,
                 int32_t kh, int32_t kw, const float* scale, const float* shift, void* out,
                 int32_t out_layout, uint8_t* argmax, void* win /* optional: raw winner x per cell, or NULL */,
                 mia_stream_t stream);
/* Forward of maxpool(relu(bn(x))) split around the BN statistics (training, bf16 x (n, h, w, c) NHWC):
 * mia_pool_raw_stats reads x once and writes each window's winner (raw bf16 value; raw max for gamma > 0,
 * raw min for gamma < 0, first position for gamma == 0; first occurrence on ties), its argmax (u8, as
 * mia_pool_fwd) and the BN shifted sums about kshift[c] of EVERY pixel (the w % kw right of the last window
 * included): partial[nblocks][c][2] for mia_bn_finalize_shifted (h % kh == 0).
 * mia_pool_apply then writes relu(scale*win + shift) in mia_pool_fwd's output layouts.  Replaces the
 * BatchNorm2d statistics pass + MaxPool2d of src/models/envnet_v2.py:20-24. */
int mia_pool_raw_stats(const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh, int32_t kw,
                       const float* gamma, const float* kshift, void* win, uint8_t* argmax, float* partial,
                       int32_t nblocks, mia_stream_t stream);
int mia_pool_apply(const void* win, int32_t n, int32_t oh, int32_t ow, int32_t c, const float* scale,
                   const float* shift, void* out, int32_t dtype, int32_t out_layout, mia_stream_t stream);
/* Backward of pool(relu(bn(x))) up to dz (the BN output grad) + BN reductions
 * (nn.MaxPool2d after BN+ReLU, envnet_v2.py:16-23,32-37). */
int mia_pool_bwd_bn_relu_reduce(const void* dout, int32_t out_layout, const uint8_t* argmax,
                                const void* x, int32_t dtype, int32_t n, int32_t h, int32_t w,
                                int32_t c, int32_t kh, int32_t kw, const float* scale,
                                const float* shift, const float* mean, const float* invstd,
                                void* dz, float* dgamma, float* dbeta, void* partial,
                                mia_stream_t stream);
/* Pooled backward, sparse half: at the argmax position of every pooled cell,
 * gm[cell][c] = dout[cell][c] * (scale*x+shift > 0) (f32, NHWC cells (n, h/kh, w/kw, c)), and the BN
 * reductions dgamma = sum gm*xhat, dbeta = sum gm (the other kh*kw-1 window pixels carry no
 * gradient and are never read).  Replaces autograd of nn.MaxPool2d + nn.ReLU (envnet_v2.py:16-23). */
int mia_pool_bwd_gather(const void* dout, int32_t out_layout, const uint8_t* argmax, const void* x,
                        const void* win /* optional raw winners (n, h/kh, w/kw, c), x's dtype, or NULL */,
                        int32_t dtype, int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh, int32_t kw,
                        const float* scale, const float* shift, const float* mean, const float* invstd,
                        float* gm, float* dgamma, float* dbeta, void* partial, mia_stream_t stream);
/* Pooled backward, dense half (one read of x, one write of dx): BN backward
 * dx = gamma*invstd*(g - dbeta/P - xhat*dgamma/P), g = gm[cell] at the argmax position, else 0;
 * optional dbias[c] = sum_rows dx (nn.BatchNorm2d backward, envnet_v2.py:16,33). */
int mia_pool_bn_relu_bwd_apply(const float* gm, const uint8_t* argmax, const void* x, int32_t dtype,
                               int32_t n, int32_t h, int32_t w, int32_t c, int32_t kh, int32_t kw,
                               const float* gamma, const float* mean, const float* invstd,
                               const float* dgamma, const float* dbeta, void* dx, float* dbias,
                               void* partial, mia_stream_t stream);

/* Column sums over rows of a (P, C) matrix: bias gradients. out f32[C] (overwritten).
 * partial: MIA_COLSUM_MAXBLK * C floats of workspace. */
#define MIA_COLSUM_MAXBLK 1024
int mia_colsum(const void* x, int32_t dtype, int64_t P, int32_t C, int64_t ld, float* out,
               void* partial, mia_stream_t stream);

/* out[b][ih][iw] = sum_{ky} p[b][ih-ky][iw][ky]   (dgrad of the 1-channel 8x8 trunk conv,
 * envnet_v2.py:41 first conv). p: (n, ph, w, kh) f32; out (n, ph+kh-1, w) dtype. */
int mia_col2im_rows(const float* p, int32_t n, int32_t ph, int32_t w, int32_t kh, void* out,
                    int32_t dtype, mia_stream_t stream);

/* Backward-data of the single-input-channel 8x8 conv, EnvNet-v2 trunk conv3
 * (reference src/models/envnet_v2.py:31 Conv2d(1, 32, (8, 8)); replaces cuDNN conv2d backward-data):
 *   dx[b][y][x] = sum_{ky,kx,co} dy[b][y-ky][x-kx][co] * w[co][0][ky][kx]
 * dy bf16 NHWC (n, oh, ow, 32), w f32 OIHW (32, 1, 8, 8), dx bf16 (n, oh+7, ow+7);
 * oh+7 <= 64, (ow+7) % 4 == 0, dy/dx 16-byte aligned.  Deterministic. */
int mia_conv1ch_dgrad(const void* dy, const float* w, void* dx, int32_t n, int32_t oh, int32_t ow,
                      mia_stream_t stream);

/* EnvNet-v2 frontend conv1 forward (reference src/models/envnet_v2.py:15 Conv2d(1, 32, (1, 64),
 * stride (1, 2)) on the raw waveform; replaces that cuDNN conv2d) with the BatchNorm1 batch
 * statistics (envnet_v2.py:16, training mode) accumulated from the stored bf16 values:
 *   y1[b][o][c] = bias[c] + sum_{k<64} w[c][k] * x[b][2o+k],  o < w1 = (t-64)/2+1
 * x f32 (n, t) (8-byte aligned), w bf16 (32, 64), bias f32 (32), y1 bf16 (n, w1, 32).
 * partial (or NULL): f32 [nwaves][32][2] sums of (y1 - bias[c]) and its square, for
 * mia_bn_finalize_shifted(kshift = bias).  nwaves: multiple of 4 (the launch is nwaves/4 x 256). */
int mia_fe_conv1_fwd(const float* x, const void* w, const float* bias, void* y1, float* partial, int32_t nwaves,
                     int32_t n, int32_t t, mia_stream_t stream);

/* EnvNet-v2 trunk conv3 forward (reference src/models/envnet_v2.py:31 Conv2d(1, 32, (8, 8)) on the
 * pooled frontend image; replaces that cuDNN conv2d) with the BatchNorm batch statistics of its
 * bf16 output accumulated in the epilogue (as mia_fe_conv1_fwd):
 *   y[b][oy][ox][c] = bias[c] + sum_{ky,kx<8} w[c][ky*8+kx] * x[b][oy+ky][ox+kx]
 * x bf16 (n, h, wd) (wd % 4 == 0, 8-byte aligned), w bf16 (32, 64), y bf16 (n, h-7, wd-7, 32);
 * partial (or NULL): f32 [nwaves][32][2] shifted sums about bias for mia_bn_finalize_shifted. */
int mia_fe_conv3_fwd(const void* x, const void* w, const float* bias, void* y, float* partial, int32_t nwaves,
                     int32_t n, int32_t h, int32_t wd, mia_stream_t stream);

/* EnvNet-v2 trunk conv4 (Conv2d(32, 32, (8, 8)), replaces the cuDNN conv of src/models/envnet_v2.py:34
 * and its backward-data): y[b][oy][ox][co] = bias[co] + sum a[b][oy+ky-ph][ox+kx-pw][ci] W[co][ky][kx][ci],
 * a = relu(x*pre_scale + pre_shift) when pre_scale is given (forward, BN+ReLU of the previous conv), else x
 * (backward-data: x = dY, ph = pw = 7, w = the flipped weights of mia_pack_weight layout 1).  x bf16
 * (n, h, wd, 32), w bf16 (32, 8, 8, 32) OHWI, y bf16 (n, h+2ph-7, wd+2pw-7, 32), all 16-byte aligned;
 * bias (or NULL) f32 (32); partial (or NULL, needs bias): f32 [4*nblocks][32][2] shifted sums about bias of
 * the stored outputs, for mia_bn_finalize_shifted.  Row-rolling MFMA kernel, one workgroup per CU. */
int mia_trunk_conv8(const void* x, const float* pre_scale, const float* pre_shift, const void* w, const float* bias,
                    void* y, float* partial, int32_t nblocks, int32_t n, int32_t h, int32_t wd, int32_t ph, int32_t pw,
                    mia_stream_t stream);

/* conv4 backward-data (mia_trunk_conv8 with x = dY (n, h, wd, 32), ph = pw = 7, w = layout-1 flipped weights ->
 * dx (n, h+7, wd+7, 32)) fused with the ReLU+BN backward reductions of mia_bn_relu_bwd_reduce (replaces the
 * BatchNorm2d + ReLU backward of src/models/envnet_v2.py:34-36 for conv3's BN): bx is that BN's input (the
 * conv3 output, dx's shape), scale / shift / mean / invstd its batch statistics; dgamma[c] = sum dx*m*xhat,
 * dbeta[c] = sum dx*m with m = [bx*scale + shift > 0], xhat = (bx - mean)*invstd, over the stored bf16 dx.
 * partial: f32 [4*nblocks][32][2] workspace. */
int mia_trunk_conv8_dgrad_bn(const void* dy, const void* w, void* dx, int32_t nblocks, int32_t n, int32_t h,
                             int32_t wd, const void* bx, const float* scale, const float* shift, const float* mean,
                             const float* invstd, float* dgamma, float* dbeta, float* partial, mia_stream_t stream);

/* Weight gradient of the EnvNet-v2 trunk conv3 (Conv2d(1, 32, (8, 8)), replaces the cuDNN backward-weight
 * of src/models/envnet_v2.py:31): dw[co][ky*8+kx] = sum dy[b][oy][ox][co] * x[b][oy+ky][ox+kx].  x bf16
 * (n, h, wd) (wd % 4 == 0, 8-byte aligned), dy bf16 (n, h-7, wd-7, 32) 16-byte aligned, dw f32 (32, 64);
 * part: f32 workspace of nwaves*2048 + 64*4096 floats, 8-byte aligned (one slab per wave, summed in fixed order). */
int mia_conv3_wgrad(const void* x, const void* dy, float* dw, float* part, int32_t nwaves, int32_t n, int32_t h,
                    int32_t wd, mia_stream_t stream);

/* mia_conv3_wgrad with the ReLU+BN backward of conv3's BN (BatchNorm2d + ReLU of src/models/envnet_v2.py:31-33;
 * mia_bn_relu_bwd_apply's arithmetic) formed while staging dY: dy = BN backward of da (the gradient of
 * relu(ya*scale + shift)), gamma, mean, invstd, dgamma, dbeta as mia_bn_relu_bwd_apply takes them, is written
 * to dy (n, h-7, wd-7, 32) bf16 (may alias da) and summed per channel into dbias f32 (32).  da, ya, dy 16-byte
 * aligned; part: f32 workspace of mia_conv3_wgrad_workspace_bytes(nwaves) bytes, 8-byte aligned. */
int64_t mia_conv3_wgrad_workspace_bytes(int32_t nwaves);
int mia_conv3_wgrad_bn(const void* x, const void* da, const void* ya, void* dy, float* dw, float* dbias, float* part,
                       int32_t nwaves, int32_t n, int32_t h, int32_t wd, const float* gamma, const float* scale,
                       const float* shift, const float* mean, const float* invstd, const float* dgamma,
                       const float* dbeta, mia_stream_t stream);

/* BatchNorm finalize from per-block shifted sums partial[nblk][C][2] about kshift[c]: writes mean,
 * invstd, the fused scale/shift (gamma*invstd, beta - mean*gamma*invstd) and updates the running
 * statistics (momentum, unbiased variance) exactly as mia_bn_fwd_stats.  Training mode only. */
int mia_bn_finalize_shifted(const float* partial, int32_t nblk, int64_t P, int32_t C, const float* kshift,
                            const float* gamma, const float* beta, float* running_mean, float* running_var,
                            float momentum, float eps, int32_t training, float* mean, float* invstd,
                            float* scale, float* shift, mia_stream_t stream);

/* EnvNet-v2 frontend conv2 forward (reference src/models/envnet_v2.py:19 Conv2d(32, 64, (1, 16),
 * stride (1, 2)) applied to relu(bn1(y1)), envnet_v2.py:20-21; replaces that cuDNN conv2d):
 *   y2[b][o][co] = bias[co] + sum_{kx,ci} w[co][kx][ci] * relu(y1[b][2o+kx][ci]*scale[ci] + shift[ci])
 * bf16 only.  y1 (n, w1, 32), w OHWI (64, 16, 32) (mia_pack_weight mode 0), bias f32 (64) or NULL,
 * y2 (n, w2, 64) with w2 = (w1-16)/2+1; scale/shift NULL = no BN/ReLU on the input.  Persistent,
 * weight-stationary (weights in registers), one workgroup per CU.  Deterministic. */
int mia_fe_conv2_fwd(const void* y1, const float* scale, const float* shift, const void* w,
                     const float* bias, void* y2, int32_t n, int32_t w1, int32_t w2, mia_stream_t stream);

/* Backward-data of the same conv (replaces cuDNN conv2d backward-data for envnet_v2.py:19):
 *   da1[b][p][ci] = sum_{o,kx: 2o+kx=p} w[co][kx][ci] * dy2[b][o][co]
 * dy2 (n, w2, 64) bf16, wpar = mia_pack_weight mode 2 of w (2, 32, 8, 64) bf16, da1 (n, w1, 32) bf16.
 * Both output parities come from one staged dY window.  Deterministic. */
int mia_fe_conv2_dgrad(const void* dy2, const void* wpar, void* da1, int32_t n, int32_t w1, int32_t w2,
                       mia_stream_t stream);

/* Weight gradient of the same conv (replaces cuDNN conv2d backward-weight for envnet_v2.py:19):
 *   dw[co][kx*32+ci] = sum_{b,o} dy2[b][o][co] * relu(y1[b][2o+kx][ci]*scale[ci] + shift[ci])
 * dy2 (n, w2, 64), y1 (n, w1, 32) bf16; dw f32 (64, 16*32) (OHWI); scale/shift NULL = no pre-op.
 * workspace: one 128 KB f32 slab per workgroup (<= #CU per 2 GB of y1).  Deterministic. */
int mia_fe_conv2_wgrad(const void* dy2, const void* y1, const float* scale, const float* shift, float* dw,
                       int32_t n, int32_t w1, int32_t w2, void* workspace, int64_t ws_bytes,
                       mia_stream_t stream);

/* EnvNet-v2 BatchNorm1+ReLU backward and conv1 weight + bias gradient in ONE pass over
 * (dact, y1, x) (reference src/models/envnet_v2.py:15-17 Conv2d(1, 32, (1, 64), stride (1, 2)) ->
 * BN -> ReLU; replaces the BN backward reductions, its elementwise pass and cuDNN conv2d
 * backward-weight).  With dz = mask * dact (mask = y1*scale + shift > 0), xhat = (y1-mean)*invstd:
 *   dbeta[c] = sum_p dz,  dgamma[c] = sum_p dz*xhat      (outputs)
 *   g = A dz + B + C y1,  A = gamma*invstd, B = -A dbeta/P + A invstd mean dgamma/P, C = -A invstd dgamma/P
 *   dw[c][k] = sum_p g[p][c] x[2p+k] = A G1 + B G2 + C G3,  dbias[c] = sum_p g[p][c]
 * where G1 = sum dz x, G3 = sum y1 x (bf16 MFMA, f32 accumulate), G2[k] = sum x[2p+k]; the
 * combination runs in double.  P = n*w1, w1 = (t-64)/2+1.  x f32 (n, t); dact, y1 bf16 (n, w1, 32);
 * dw f32 (32, 64); workspace >= (split*(2*2048+96) + 2*2048 + n*80 + 2*160 + 4) floats.  Deterministic. */
int mia_fe_conv1_wgrad_bn(const float* x, const void* dact, const void* y1, int32_t n, int32_t t,
                          const float* scale, const float* shift, const float* gamma, const float* mean,
                          const float* invstd, float* dgamma, float* dbeta, float* dw,
                          float* dbias, void* workspace, int32_t split, mia_stream_t stream);

/* EnvNet-v2 trunk (1, 2) conv weight gradient as one dense GEMM (reference
 * src/models/envnet_v2.py:38-49; replaces cuDNN conv2d backward-weight for those layers):
 *   dW[co][kx][ci] = sum_q Ashift[q][co*2+kx] * a[q][ci]  over the input pixels q,
 * Ashift from mia_shift_pad_w2, a = the conv input (after mia_bn_relu_apply when the layer's input
 * is relu(bn(.))); the GEMM itself is mia_gemm on two DENSE K-major (RC) bf16 operands. */
/* out = bf16(relu(x*scale + shift)), x/out bf16 (P, C), C % 8 == 0, 16-byte aligned. */
int mia_bn_relu_apply(const void* x, int64_t P, int32_t C, const float* scale, const float* shift, void* out,
                      mia_stream_t stream);
/* out[r][x][2c+kx] = dy[r][x-kx][c] (0 <= x-kx < w-1, else 0): dy bf16 (rows, w-1, c), out bf16
 * (rows, w, 2c), c % 8 == 0, 16-byte aligned. */
int mia_shift_pad_w2(const void* dy, int64_t rows, int32_t w, int32_t c, void* out, mia_stream_t stream);
/* The (1, 2)-conv backward's gradient on the input grid: dst (1 + rows*w pixels x c, bf16) = one zero pixel, then
 * dy (rows x (w-1) x c) re-laid with a zero at each row's last column; zero_pixel (zc bf16, may be null) is
 * zeroed too.  Both backward GEMMs then read dst through overlapping dense views (trunk_bwd_w2). */
int mia_pad_w2(const void* dy, int64_t rows, int32_t w, int32_t c, void* dst, void* zero_pixel, int32_t zc,
               mia_stream_t stream);
/* dst[r][x] = src[r][x] for x < w-1: src bf16 (rows, w, c) -> dst (rows, w-1, c); c % 8 == 0. */
int mia_drop_last_col(const void* src, int64_t rows, int32_t w, int32_t c, void* dst, mia_stream_t stream);

/* Weight repack: src f32 (cout, cin, kh, kw) (PyTorch OIHW) -> dst dtype.
 * mode 0: OHWI (cout, kh, kw, cin)            — forward operand
 * mode 1: flipped dgrad operand (cin, kh, kw, cout) with ky->kh-1-ky, kx->kw-1-kx
 * mode 2: parity dgrad operand for stride-2 1-D convs: (2, cin, kw/2, cout),
 *         [p][ci][j][co] = W[co][ci][0][2*(kw/2-1-j)+p]
 * mode 3: row-split dgrad for cin==1: (kh, kw, cout) with [ky][j][co] = W[co][0][ky][kw-1-j]
 * mode 4: inverse of mode 0 on f32 gradients: src (cout,kh,kw,cin) -> dst (cout,cin,kh,kw). */
int mia_pack_weight(const float* src, void* dst, int32_t dtype, int32_t cout, int32_t cin,
                    int32_t kh, int32_t kw, int32_t mode, mia_stream_t stream);
/* mia_pack_weight for up to MIA_PACK_BATCH weights in ONE launch (modes 0-3, bf16 or f32 outputs): the
 * per-step weight packs of a training step are launch-bound tiny kernels. */
#define MIA_PACK_BATCH 16
typedef struct MiaPackJob {
  const float* src;
  void* dst;
  int32_t dtype, cout, cin, kh, kw, mode;
} MiaPackJob;
int mia_pack_weights(const MiaPackJob* jobs, int32_t n, mia_stream_t stream);

/* out[m][n] = act(sum_s ws[s][m][n] * alpha + bias[n]) with MiaEpilogue semantics —
 * split-K combine; exposed for the FC layers. */
int mia_splitk_reduce(const float* ws, int32_t split_k, int64_t M, int64_t N,
                      const MiaEpilogue* E, mia_stream_t stream);

/* Inverted dropout on a (rows, cols) activation, in place, keep-mask = hash(seed, idx) >= p.
 * nn.Dropout (envnet_v2.py:53,57).  Output scaled by 1/(1-p). */
int mia_dropout(void* x, int32_t dtype, int64_t numel, float p, uint64_t seed,
                mia_stream_t stream);

/* Soft-label loss of LitClassifier._step (engine.py:175-176):
 *   loss = -mean_b sum_c y*log(softmax(z)+1e-8);  dz written (scaled by grad_scale).
 * If input_sigmoid, z = sigmoid(logits) first (ASTModel returns probabilities, ast.py:63)
 * and dlogits includes the sigmoid backward.  loss: f32[1]; correct: i32[1] argmax hits. */
int mia_soft_ce(const float* logits, const float* y, int32_t B, int32_t C, int32_t input_sigmoid,
                float* loss, float* dlogits, int32_t* correct, mia_stream_t stream);

/* Gradient clipping + Adam over a device-side table of tensors (Lightning
 * gradient_clip_val=1.0 + torch.optim.Adam(lr, weight_decay), base_training.yaml:51,56-59).
 * tables: f32* params[n], grads[n], m[n], v[n]; int64 sizes[n] (all device arrays).
 * shadow_bf16: optional table of bf16* (entries may be NULL): the bf16 GEMM-operand copy of each
 * updated parameter is written in the same pass (replaces a separate cast of the weights).
 * sqnorm_ws: f32 workspace of mia_adam_workspace_bytes(ntensors) bytes.
 * pre_sq / pre_n (optional device tables, may be NULL): for tensor i with pre_sq[i] != NULL the norm
 * pass reads pre_n[i] partial sums of squares (doubles, e.g. a GEMM's MiaEpilogue.sqsum slots of the
 * gradient it wrote) instead of re-reading grads[i]; the partials are added in a fixed order.
 * clip <= 0 disables clipping. step is 1-based; steps (optional device int32[n], may be NULL) gives
 * each tensor its own 1-based step for the bias corrections (torch.optim.Adam keeps a step count per
 * parameter; a parameter that had no gradient in some step is behind the others).
 * max_numel sizes the update grid (the largest tensor the update pass walks: NULL-gradient tensors
 * excluded), max_norm_numel the norm grid (the largest tensor whose gradient it reads: pre_sq tensors
 * excluded); the norm's summation order is a fixed function of max_norm_numel. */
int64_t mia_adam_workspace_bytes(int32_t ntensors);
/* byte offset of the device clip coefficient (f32) inside that workspace; a tensor whose grads[] entry is
 * NULL is counted in the norm through pre_sq only and not updated (its update is mia_gemm_adam's) */
int64_t mia_adam_coef_offset(int32_t ntensors);
int mia_clip_adam(void* const* params, void* const* grads, void* const* exp_avg,
                  void* const* exp_avg_sq, void* const* shadow_bf16, const int64_t* sizes, int32_t ntensors,
                  int64_t max_numel, int64_t max_norm_numel, float lr, float beta1, float beta2, float eps,
                  float weight_decay, int32_t step, float clip, float* total_norm_out,
                  void* sqnorm_ws, const void* const* pre_sq, const int64_t* pre_n, const int32_t* steps,
                  mia_stream_t stream);

/* LayerNorm over the last dim (timm Block norm1/norm2 and final norm, eps 1e-6).
 * x: (rows, D) -> y dtype; mean/rstd f32[rows] saved for backward. */
int mia_layernorm_fwd(const void* x, int32_t xdtype, const float* gamma, const float* beta,
                      void* y, int32_t ydtype, float* mean, float* rstd, int64_t rows,
                      int32_t D, float eps, mia_stream_t stream);
/* dx (+= if accumulate) and partial sums for dgamma/dbeta (f32 [nblk][2][D] in partial,
 * reduced into dgamma/dbeta). */
/* dx2 (optional, may be null): a second copy of the final dx in dx2dtype (the bf16 GEMM operand of
 * the next linear's backward, saving a separate cast pass). */
int mia_layernorm_bwd(const void* dy, int32_t dydtype, const void* x, int32_t xdtype,
                      const float* gamma, const float* mean, const float* rstd, void* dx,
                      int32_t dxdtype, int32_t accumulate, void* dx2, int32_t dx2dtype, float* dgamma,
                      float* dbeta, void* partial, int64_t rows, int32_t D, mia_stream_t stream);
/* As mia_layernorm_bwd, also writing dx2_colsum[D] = sum over rows of the stored dx2 values: the
 * bias gradient of the linear whose backward takes dx2 as its dy (timm Block proj / fc2 biases,
 * replacing a separate column-sum pass over the residual gradient).  D == 768, dx2 required. */
int mia_layernorm_bwd_colsum(const void* dy, int32_t dydtype, const void* x, int32_t xdtype,
                             const float* gamma, const float* mean, const float* rstd, void* dx,
                             int32_t dxdtype, int32_t accumulate, void* dx2, int32_t dx2dtype, float* dgamma,
                             float* dbeta, float* dx2_colsum, void* partial, int64_t rows, int32_t D,
                             mia_stream_t stream);
/* As mia_layernorm_bwd_colsum with a bf16 dx2, also writing the OCP MX-fp8 copy of the stored dx2 values
 * (q [rows][D] e4m3 bytes, 4-B aligned; scales [rows][D / 32], mia_mx_quantize's format): the A operand of
 * the fp8-mixed backward-data GEMMs of proj / fc2 (mia_gemm_mxfp8_ex) without a quantisation pass. */
int mia_layernorm_bwd_colsum_mx(const void* dy, int32_t dydtype, const void* x, int32_t xdtype,
                                const float* gamma, const float* mean, const float* rstd, void* dx,
                                int32_t dxdtype, int32_t accumulate, void* dx2, float* dgamma, float* dbeta,
                                float* dx2_colsum, void* q, void* scales, void* partial, int64_t rows, int32_t D,
                                mia_stream_t stream);
int64_t mia_layernorm_partial_bytes(int64_t rows, int32_t D);

/* Fused multi-head attention (timm Attention with F.scaled_dot_product_attention,
 * ast.py:60-61), head_dim 64.  dtype MIA_BF16: flash kernel on bf16 MFMA with online softmax;
 * dtype MIA_F32: exact-f32 reference-precision kernels (parity mode, N <= 3328).
 * qkv: (B, N, 3, H, 64) (the qkv Linear output as is); out: (B, N, H, 64);
 * lse: f32 (B, H, N) saved for backward. */
int mia_attn_fwd(const void* qkv, void* out, float* lse, int32_t dtype, int32_t B, int32_t N,
                 int32_t H, float scale, mia_stream_t stream);
/* Deterministic backward, no float atomics.  bf16: a key-parallel dK/dV kernel + a query-parallel dQ
 * kernel (each recomputes S and dP; mia_attn_bwd_fused below is the one-pass alternative).
 * f32: exact reference-precision kernels.
 * dout: (B, N, H, 64) bf16; dqkv: (B, N, 3, H, 64) bf16 (fully written);
 * work: 16-B aligned workspace of mia_attn_bwd_workspace_bytes() bytes (bf16: the scaled Q operand,
 * per-query row-constant fragments, hand-off flags and running sums; f32: rowsum(dO * O)). */
int64_t mia_attn_bwd_workspace_bytes(int32_t dtype, int32_t B, int32_t N, int32_t H);
int mia_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                 void* dqkv, void* work, int32_t dtype, int32_t B, int32_t N, int32_t H,
                 float scale, mia_stream_t stream);
/* Training form (bf16): mia_attn_fwd_save_q is mia_attn_fwd (q8 / s8 NULL) or mia_attn_fwd_mx (both
 * set) that also writes the backward's scaled query operand Q' into `work` (at least
 * mia_attn_saved_q_bytes: Q' + the row-constant fragments, kept from the forward to the backward; the
 * one-pass backward's flags and running sums are not part of it); mia_attn_bwd_saved_q is the two-kernel
 * mia_attn_bwd (bf16) on such a workspace: neither re-reads q nor rewrites Q'. */
int64_t mia_attn_saved_q_bytes(int32_t B, int32_t N, int32_t H);
int mia_attn_fwd_save_q(const void* qkv, void* out, float* lse, void* q8, void* s8, void* work, int32_t B,
                        int32_t N, int32_t H, float scale, mia_stream_t stream);
int mia_attn_bwd_saved_q(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                         void* work, int32_t B, int32_t N, int32_t H, float scale, mia_stream_t stream);
/* The bf16 backward in its two-kernel form (what mia_attn_bwd / mia_attn_bwd_saved_q run), and in a
 * fused one-pass form: per (b, h, 256-key block) S, dP, dS are computed once, dV / dK accumulate in
 * registers and dQ is summed over the key blocks by an ordered hand-off of running f32 sums in `work`
 * (fixed order: bit-reproducible).  q_ready: `work` already holds Q' (mia_attn_fwd_save_q).
 * mia_attn_bwd_fused returns 0 even when one of its bounded hand-off waits gave up: the caller MUST read the
 * u32 error word at byte offset mia_attn_bwd_error_offset(B, N, H) of `work` after the call (nonzero: that
 * call's dQ is invalid).  No model path calls it; mia_attn_bwd_onepass takes a caller-owned error word. */
int mia_attn_bwd_two_pass(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                          void* work, int32_t B, int32_t N, int32_t H, float scale, int32_t q_ready,
                          mia_stream_t stream);
int mia_attn_bwd_fused(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                       void* work, int32_t B, int32_t N, int32_t H, float scale, int32_t q_ready,
                       mia_stream_t stream);
/* The one-pass bf16 training backward: no recompute (S, dP, dS once per tile; dV, dK in registers;
 * dQ = dS K summed over the 256-key blocks of each (b, h) by an ordered hand-off of running f32 sums:
 * bit-reproducible).  Replaces F.scaled_dot_product_attention's backward inside timm's Attention
 * (reference src/models/ast.py:60-61); an alternative to mia_attn_bwd_saved_q, which is faster on MI355X
 * at the AST shape and is what the model calls.
 * saved: mia_attn_saved_q_bytes (Q' -- already there when q_ready, from mia_attn_fwd_save_q -- and the
 *   row-constant fragments, written here); chain: mia_attn_bwd_chain_bytes of scratch for this call only
 *   (hand-off flags + running sums; both 256-B aligned).
 * err: a caller-owned u32, zero before the first call and never cleared by the library: a bounded hand-off
 *   wait that gave up sets it to 1 (that call's dQ is invalid; every later call's waits give up at once).
 *   Check it at a convenient sync point; no wait ever hangs the GPU. */
int64_t mia_attn_bwd_chain_bytes(int32_t B, int32_t N, int32_t H);
int mia_attn_bwd_onepass(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                         void* saved, void* chain, uint32_t* err, int32_t B, int32_t N, int32_t H, float scale,
                         int32_t q_ready, mia_stream_t stream);
/* Byte offset in the bf16 workspace of a u32 error word: 0 after a fused backward = every dQ hand-off
 * matched; non-zero = a bounded wait gave up and that call's dQ is not valid. */
int64_t mia_attn_bwd_error_offset(int32_t B, int32_t N, int32_t H);

/* AST token assembly (ast.py:56-59): x[b][0] = cls + pos[0]; x[b][1+p] = patches[b][p] + pos[1+p].
 * patches: (B, Np, D) f32; out (B, Np+1, D) f32.  Backward: dpatch, dcls/dpos reductions. */
int mia_tokens_fwd(const float* patches, const float* cls, const float* pos, float* out,
                   int32_t B, int32_t Np, int32_t D, mia_stream_t stream);
int mia_tokens_bwd(const float* dout, float* dpatches, float* dcls, float* dpos, int32_t B,
                   int32_t Np, int32_t D, mia_stream_t stream);

/* bf16 patch embedding (ast.py:38 PatchEmbed = Conv2d(1, D, ps, stride st); replaces the implicit-GEMM
 * gather): mia_ast_patches writes the (B*N, ps*ps) bf16 patch matrix in TOKEN order (N = gh*gw + 1,
 * row b*N is a zero row in the cls slot), so one dense GEMM with the bias epilogue writes the token rows
 * of x directly and the weight gradient is one dense GEMM of the bf16 token gradient against it;
 * mia_tokens_fwd_inplace then sets x[b][0] = cls + pos[0] and adds pos[t] to every other row.
 * spec: (B, Fm, Tf) f32; out 16-B aligned; ps % 8 == 0; x, cls, pos 16-B aligned, D % 4 == 0. */
int mia_ast_patches(const float* spec, int32_t B, int32_t Fm, int32_t Tf, int32_t ps, int32_t st, void* out,
                    mia_stream_t stream);
int mia_tokens_fwd_inplace(float* x, const float* cls, const float* pos, int32_t B, int32_t N, int32_t D,
                           mia_stream_t stream);

/* Elementwise helpers. */
int mia_cast(const void* src, int32_t sdtype, void* dst, int32_t ddtype, int64_t numel,
             mia_stream_t stream);
/* x += y (f32) */
int mia_add_inplace(float* x, const void* y, int32_t ydtype, int64_t numel, mia_stream_t stream);

/* Between-class mixing on device (BCMixingDataset.apply_bc_mixing, preprocessing.py:564-609):
 * partner clips come from a resident pool (the preloaded training set, or the batch itself):
 * out[b] = (p*x[b] + (1-p)*pool[partner[b]]) / sqrt(p^2+(1-p)^2), p = r[b] adjusted by the
 * RMS-"SPL" rule (preprocessing.py:395-471); soft labels use r (not p) at labels[b] and
 * pool_labels[partner[b]]; partner < 0 keeps the clip (one-hot label).
 * workspace: 2*B floats. */
int mia_bc_mix(const float* x, const float* pool, int64_t T, int32_t B, const int32_t* partner,
               const float* r, const int64_t* labels, const int64_t* pool_labels,
               int32_t num_classes, float* out, float* yout, float* p_out, void* workspace,
               mia_stream_t stream);
/* BC-mixing partner draw (apply_bc_mixing's random.choice over different-class clips,
 * preprocessing.py:584-591): partner[b] = the k-th pool clip (pool order) whose label differs
 * from labels[b], k = min(floor(u[b] * n_diff), n_diff - 1); -1 when the pool has no other class
 * (the reference then returns the clip unmixed with a one-hot label, :585-588). */
int mia_bc_partner(const int64_t* labels, int32_t B, const int64_t* pool_labels, int32_t N,
                   const float* u, int32_t* partner, mia_stream_t stream);
/* Time stretch + gain (EnvNetPreprocessor.apply_augmentation, preprocessing.py:886-925) of a
 * (B, T) batch: clip b resampled to int(T / factor[b]) samples with F.interpolate's linear,
 * align_corners=False rule (factor <= 0: unchanged), times gain[b]; written into the T-sample
 * window (cropped past T, zero past the stretched length).  factor (f64) / gain (f32) may be NULL. */
int mia_stretch_gain(const float* x, int64_t T, int32_t B, const double* factor, const float* gain,
                     float* out, mia_stream_t stream);
/* SpecAugment zero masks then Mixup with an un-augmented partner from `pool`
 * (preprocessing.py:1075-1104, esc50.py:52-76) on (B, F, T) spectrograms; masks and partners
 * (partner < 0: no mixup) drawn by the caller. */
int mia_spec_augment_mixup(const float* spec, const float* pool, float* out, int32_t B, int32_t F,
                           int32_t T, const int32_t* t0, const int32_t* tlen, const int32_t* f0,
                           const int32_t* flen, const int32_t* partner, const float* lam,
                           mia_stream_t stream);

/* dst <- src (`bytes`, a multiple of 16, 16-B aligned): a plain streaming copy, non-temporal.  Not on the
 * training path: bench.py times it in the same process as the box's HBM calibration (read + write GB/s of
 * a 2 GB stream), so a kernel's achieved bandwidth can be read against both the 8 TB/s spec and the rate
 * this box's HBM actually streams at (`frac_vs_box`). */
int mia_stream_copy(const void* src, void* dst, int64_t bytes, mia_stream_t stream);

/* Back-to-back bf16 MFMAs on every SIMD (`waves_per_simd` 4-wave blocks per CU, each wave `iters` x 16
 * v_mfma_f32_16x16x32_bf16 on pseudo-random operands, 4 independent accumulators): bench.py's MFMA
 * calibration, the rate this box's matrix cores hold under load (FLOPs = cu_count * waves_per_simd * 4 *
 * iters * 16 * 16384).  `sink` (mia_mfma_rate_sink_floats floats) receives the accumulators.  Not on the
 * training path. */
int64_t mia_mfma_rate_sink_floats(int32_t waves_per_simd);
int mia_mfma_rate(float* sink, int32_t iters, int32_t waves_per_simd, mia_stream_t stream);

const char* mia_last_error_string(void);
int mia_device_arch(char* buf, int32_t len); /* gcnArchName of the current device */

#ifdef __cplusplus
}
#endif
#endif /* MIAUDIO_H */
