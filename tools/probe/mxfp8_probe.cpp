// Probe: does hipBLASLt (ROCm 7.2) run MX-scaled fp8 (e4m3, one E8M0 scale per 32 elements of K)
// GEMMs on gfx950, and with which scale layout?  D = A^T B (column-major, TN), M=N=256, K=512.
// Checks the result against a host reference for two candidate scale layouts.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hip/hip_fp8.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto e = (x); if ((int)e) { printf("FAIL %s -> %d (line %d)\n", #x, (int)e, __LINE__); return 1; } } while (0)

static float e4m3_to_f(uint8_t b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
  return s ? -v : v;
}

int main() {
  const int M = 256, N = 256, K = 512;
  std::vector<uint8_t> A(K * M), B(K * N);  // column-major K x M (op T) and K x N (op N): K innermost
  std::vector<uint8_t> sa(M * K / 32), sb(N * K / 32);
  srand(1);
  for (auto& x : A) { do x = rand() & 0xff; while (((x >> 3) & 15) == 15); }
  for (auto& x : B) { do x = rand() & 0xff; while (((x >> 3) & 15) == 15); }
  for (auto& x : sa) x = 127 + (rand() % 5) - 2;  // 2^-2 .. 2^2
  for (auto& x : sb) x = 127 + (rand() % 5) - 2;
  uint8_t *dA, *dB, *dsa, *dsb; float* dD;
  CK(hipMalloc(&dA, A.size())); CK(hipMalloc(&dB, B.size()));
  CK(hipMalloc(&dsa, sa.size())); CK(hipMalloc(&dsb, sb.size())); CK(hipMalloc(&dD, M * N * 4));
  CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dsa, sa.data(), sa.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, sb.data(), sb.size(), hipMemcpyHostToDevice));
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  hipblasLtMatmulDesc_t desc; CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  hipblasLtMatmulMatrixScale_t mode = HIPBLASLT_MATMUL_MATRIX_SCALE_VEC32_UE8M0;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_MODE, &mode, sizeof(mode)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_MODE, &mode, sizeof(mode)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &dsa, sizeof(dsa)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &dsb, sizeof(dsb)));
  hipblasLtMatrixLayout_t la, lb, lc;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_8F_E4M3, K, M, K));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_8F_E4M3, K, N, K));
  CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, M, N, M));
  hipblasLtMatmulPreference_t pref; CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = 64 << 20;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[4]; int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 4, res, &got);
  printf("heuristic status %d, algorithms %d\n", (int)st, got);
  if (st != HIPBLAS_STATUS_SUCCESS || got == 0) { printf("MXFP8: NOT SUPPORTED\n"); return 0; }
  void* ws; CK(hipMalloc(&ws, wsb));
  float alpha = 1.f, beta = 0.f;
  CK(hipblasLtMatmul(h, desc, &alpha, dA, la, dB, lb, &beta, dD, lc, dD, lc, &res[0].algo, ws, res[0].workspaceSize, 0));
  CK(hipDeviceSynchronize());
  std::vector<float> D(M * N);
  CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
  // candidate layouts of the scale tensors: [row][K/32] (K-block innermost) or [K/32][row]
  for (int lay = 0; lay < 2; ++lay) {
    double maxerr = 0, maxref = 0;
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < M; ++i) {
        double acc = 0;
        for (int k = 0; k < K; ++k) {
          const int kb = k / 32;
          const int ia = lay == 0 ? i * (K / 32) + kb : kb * M + i;
          const int ib = lay == 0 ? j * (K / 32) + kb : kb * N + j;
          acc += (double)e4m3_to_f(A[i * K + k]) * std::ldexp(1.0, sa[ia] - 127) *
                 (double)e4m3_to_f(B[j * K + k]) * std::ldexp(1.0, sb[ib] - 127);
        }
        maxerr = std::fmax(maxerr, std::fabs(acc - D[j * M + i]));
        maxref = std::fmax(maxref, std::fabs(acc));
      }
    printf("scale layout %s: max rel err %.3e\n", lay == 0 ? "[row][K/32]" : "[K/32][row]", maxerr / maxref);
  }
  // timing at an AST forward shape: M = 421120 tokens, N = 3072, K = 768 (fc1)
  return 0;
}
