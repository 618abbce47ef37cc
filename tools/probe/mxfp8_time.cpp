// Time hipBLASLt MX-fp8 (e4m3 + E8M0 per 32 of K) vs bf16 at the AST forward linear shapes,
// issued like blaslt.hip: D'(N x M, col-major) = op_T(W: K x N) * op_N(X: K x M), bf16 output.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <vector>

#define CK(x) do { auto e = (x); if ((int)e) { printf("FAIL %s -> %d (line %d)\n", #x, (int)e, __LINE__); return 1; } } while (0)

__global__ void fill(uint8_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    uint8_t b = h & 0xff;
    if (((b >> 3) & 15) == 15) b &= 0xF7;  // no NaN / large exponents
    p[i] = b;
  }
}

int run(hipblasLtHandle_t h, void* ws, bool mx, long M, long N, long K) {
  const hipDataType it = mx ? HIP_R_8F_E4M3 : HIP_R_16BF;
  const size_t es = mx ? 1 : 2;
  uint8_t *W, *X, *sw = nullptr, *sx = nullptr; void* D;
  CK(hipMalloc(&W, N * K * es)); CK(hipMalloc(&X, M * K * es)); CK(hipMalloc(&D, M * N * 2));
  fill<<<4096, 256>>>(W, N * K * es, 1); fill<<<4096, 256>>>(X, M * K * es, 2);
  hipblasLtMatmulDesc_t desc; CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  if (mx) {
    CK(hipMalloc(&sw, N * K / 32)); CK(hipMalloc(&sx, M * K / 32));
    CK(hipMemset(sw, 127, N * K / 32)); CK(hipMemset(sx, 127, M * K / 32));
    hipblasLtMatmulMatrixScale_t mode = HIPBLASLT_MATMUL_MATRIX_SCALE_VEC32_UE8M0;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_MODE, &mode, sizeof(mode)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_MODE, &mode, sizeof(mode)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &sw, sizeof(sw)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_B_SCALE_POINTER, &sx, sizeof(sx)));
  }
  hipblasLtMatrixLayout_t la, lb, ld;
  CK(hipblasLtMatrixLayoutCreate(&la, it, K, N, K));
  CK(hipblasLtMatrixLayoutCreate(&lb, it, K, M, K));
  CK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_16BF, N, M, N));
  hipblasLtMatmulPreference_t pref; CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = 64 << 20;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  hipblasLtMatmulHeuristicResult_t res[8]; int got = 0;
  CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 8, res, &got));
  float alpha = 1.f, beta = 0.f;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  double best = 1e30; int bi = -1;
  for (int a = 0; a < got; ++a) {
    if (res[a].workspaceSize > wsb) continue;
    bool ok = true;
    for (int w = 0; w < 2 && ok; ++w)
      ok = hipblasLtMatmul(h, desc, &alpha, W, la, X, lb, &beta, D, ld, D, ld, &res[a].algo, ws, res[a].workspaceSize, 0) == 0;
    if (!ok) continue;
    CK(hipEventRecord(e0));
    for (int r = 0; r < 10; ++r)
      hipblasLtMatmul(h, desc, &alpha, W, la, X, lb, &beta, D, ld, D, ld, &res[a].algo, ws, res[a].workspaceSize, 0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms / 10 < best) { best = ms / 10; bi = a; }
  }
  printf("%s M=%ld N=%ld K=%ld: %d algos, best %.3f ms = %.0f TFLOP/s (algo %d)\n", mx ? "mxfp8" : "bf16 ", M, N, K,
         got, best, 2.0 * M * N * K / best / 1e9, bi);
  hipFree(W); hipFree(X); hipFree(D); if (sw) { hipFree(sw); hipFree(sx); }
  return 0;
}

int main() {
  hipblasLtHandle_t h; CK(hipblasLtCreate(&h));
  void* ws; CK(hipMalloc(&ws, 64 << 20));
  const long T = 256L * 1645;
  const long shapes[4][2] = {{2304, 768}, {768, 768}, {3072, 768}, {768, 3072}};
  for (auto& s : shapes) { run(h, ws, false, T, s[0], s[1]); run(h, ws, true, T, s[0], s[1]); }
  return 0;
}
