// Lane layout of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4x1): which lane's A and which lane's B
// feed accumulator r of lane l.  Prints "lane r : A-lane B-lane".
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out) {
  const int l = threadIdx.x;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  const f32x4 da = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.f, z, 0, 0, 0);
  const f32x4 db = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, (float)(l + 1), z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) { out[(l * 4 + r) * 2] = da[r]; out[(l * 4 + r) * 2 + 1] = db[r]; }
}
int main() {
  float* d; hipMalloc(&d, 64 * 4 * 2 * 4);
  probe<<<1, 64>>>(d);
  float h[512]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) printf("%d %d : %g %g\n", l, r, h[(l * 4 + r) * 2] - 1, h[(l * 4 + r) * 2 + 1] - 1);
  return 0;
}
