// Probe: hipBLASLt BGRADB epilogue on the AST weight-gradient shapes (issued like blaslt.hip):
// D'(Kf x Nf, col-major, f32) = X^T (Kf x M) . dY (M x Nf), bias grad[nf] = sum_m dY[m][nf] (f32).
// Compares time with / without the epilogue and checks the bias gradient against a column sum.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x) do { auto e = (x); if ((int)e) { printf("FAIL %s -> %d (line %d)\n", #x, (int)e, __LINE__); return 1; } } while (0)

__global__ void fill(__hip_bfloat16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = __float2bfloat16(((int)(h & 0xffff) - 32768) / 32768.f);
  }
}
__global__ void colsum(const __hip_bfloat16* y, long M, long N, double* out) {
  const long n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double s = 0;
  for (long m = 0; m < M; ++m) s += (double)__bfloat162float(y[m * N + n]);
  out[n] = s;
}

int run(hipblasLtHandle_t h, void* ws, long M, long Nf, long Kf, bool bgrad) {
  __hip_bfloat16 *X, *Y; float *D, *bg; double* ref;
  CK(hipMalloc(&X, M * Kf * 2)); CK(hipMalloc(&Y, M * Nf * 2)); CK(hipMalloc(&D, Kf * Nf * 4));
  CK(hipMalloc(&bg, Nf * 4)); CK(hipMalloc(&ref, Nf * 8));
  fill<<<4096, 256>>>(X, M * Kf, 1); fill<<<4096, 256>>>(Y, M * Nf, 2);
  hipblasLtMatmulDesc_t desc; CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = HIPBLAS_OP_N, tb = HIPBLAS_OP_T;  // A' = X^T: col-major Kf x M (ld Kf); B' = dY: col-major Nf x M, op T
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (bgrad) {
    hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BGRADB;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    hipDataType bt = HIP_R_32F;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bg, sizeof(bg)));
  }
  hipblasLtMatrixLayout_t la, lb, ld;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, Kf, M, Kf));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, Nf, M, Nf));
  CK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_32F, Kf, Nf, Kf));
  hipblasLtMatmulPreference_t pref; CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = 64 << 20;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[8]; int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 8, res, &got);
  if (st || !got) { printf("M=%ld Nf=%ld Kf=%ld bgrad=%d: no algorithm (status %d)\n", M, Nf, Kf, bgrad, (int)st); return 0; }
  float alpha = 1.f, beta = 0.f;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  double best = 1e30; int bi = -1;
  for (int a = 0; a < got; ++a) {
    if (res[a].workspaceSize > wsb) continue;
    if (hipblasLtMatmul(h, desc, &alpha, X, la, Y, lb, &beta, D, ld, D, ld, &res[a].algo, ws, res[a].workspaceSize, 0)) continue;
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r)
      hipblasLtMatmul(h, desc, &alpha, X, la, Y, lb, &beta, D, ld, D, ld, &res[a].algo, ws, res[a].workspaceSize, 0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms / 5 < best) { best = ms / 5; bi = a; }
  }
  double err = 0;
  if (bgrad && bi >= 0) {
    hipblasLtMatmul(h, desc, &alpha, X, la, Y, lb, &beta, D, ld, D, ld, &res[bi].algo, ws, res[bi].workspaceSize, 0);
    colsum<<<(Nf + 255) / 256, 256>>>(Y, M, Nf, ref);
    CK(hipDeviceSynchronize());
    std::vector<float> b(Nf); std::vector<double> r(Nf);
    CK(hipMemcpy(b.data(), bg, Nf * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(r.data(), ref, Nf * 8, hipMemcpyDeviceToHost));
    double mx = 0;
    for (long n = 0; n < Nf; ++n) { err = std::fmax(err, std::fabs(b[n] - r[n])); mx = std::fmax(mx, std::fabs(r[n])); }
    err /= mx;
  }
  printf("M=%ld Nf=%ld Kf=%ld bgrad=%d: %d algos, best %.3f ms (algo %d)%s%.2e\n", M, Nf, Kf, bgrad, got, best, bi,
         bgrad ? " bias-grad max rel err " : "", err);
  (void)hipFree(X); (void)hipFree(Y); (void)hipFree(D); (void)hipFree(bg); (void)hipFree(ref);
  return 0;
}

int main() {
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  void* ws; CK(hipMalloc(&ws, 64 << 20));
  const long T = 256L * 1645;
  const long shapes[4][2] = {{2304, 768}, {768, 768}, {3072, 768}, {768, 3072}};  // (Nf, Kf)
  for (auto& s : shapes) { run(h, ws, T, s[0], s[1], false); run(h, ws, T, s[0], s[1], true); }
  return 0;
}
