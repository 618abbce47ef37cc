// Library path of mia_gemm: plain dense bf16 GEMMs (no fused pre-op, epilogue = bias / ReLU /
// residual add / f32 output) may run on hipBLASLt instead of the hand-written tile kernels.  The
// fused GEMMs (GELU_SAVE, dGELU, ReLU-mask backward, row maps, implicit convolutions) never do.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/miaudio.h"
#include "common.h"

namespace mblas {

// operands/epilogue expressible as one hipBLASLt matmul with identical semantics
bool eligible(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
              int compute);
// run it (plan + heuristic algorithm cached per shape/layout/epilogue key and device)
int run(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
        hipStream_t s);
// MIA_GEMM_POLICY_* (mia_gemm_set_policy)
int policy();
// auto policy: the measured winner for this key on this device, -1 = not measured yet, 0 = tile
// kernel, 1 = library
int choice(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K);
void set_choice(const MiaOperand& A, const MiaOperand& B, const MiaEpilogue& E, int64_t M, int64_t N, int64_t K,
                int v);
// whether run() delivers E.colsum itself (the dGELU pass sums its output's columns, GELU_CS_BLOCKS
// row walkers with one f32 partial row each in the 64 MB library workspace, then the slice sums of
// colsum_pass1 behind them)
constexpr int GELU_CS_BLOCKS = 4096;
inline int64_t gelu_cs_rows_bytes(int64_t N) { return ((int64_t)GELU_CS_BLOCKS * N * 4 + 255) / 256 * 256; }
inline bool fuses_colsum(const MiaEpilogue& E, int64_t N) {
  return E.colsum && E.act == MIA_DACT_GELU && N < (1 << 30) &&
         gelu_cs_rows_bytes(N) + (int64_t)COLSUM_SLICES * N * 8 <= (int64_t)(64ull << 20);
}
// the device's library workspace (stream-ordered scratch) if `bytes` fit, else null
void* scratch(size_t bytes);

}  // namespace mblas
