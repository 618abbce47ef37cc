// Probe: operand / scale lane maps of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3) on gfx950.
// Each lane passes 32 fp8 bytes of A and of B and one E8M0 scale byte each; the host tests
// candidate maps (lane, byte) -> k and reports the max error of each against a host reference.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void mx_kernel(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = a[l * 8 + i]; B[i] = b[l * 8 + i]; }
  v16f c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 16; ++r) d[l * 16 + r] = c[r];
}

static uint8_t enc(int v) {  // small integers exactly in e4m3fn
  static const uint8_t pos[4] = {0x00, 0x38, 0x40, 0x44};
  return v < 0 ? (uint8_t)(0x80 | pos[-v]) : pos[v];
}

int main() {
  srand(7);
  float Am[32][64], Bm[64][32];
  for (auto& r : Am) for (auto& x : r) x = (float)(rand() % 7 - 3);
  for (auto& r : Bm) for (auto& x : r) x = (float)(rand() % 7 - 3);
  using Map = std::function<int(int, int)>;  // (lane, byte) -> k
  std::vector<std::pair<const char*, Map>> maps = {
      {"k = 32*(l>>5) + j", [](int l, int j) { return 32 * (l >> 5) + j; }},
      {"k = 8*(l>>5) + (j&7) + 16*(j>>3)", [](int l, int j) { return 8 * (l >> 5) + (j & 7) + 16 * (j >> 3); }},
      {"k = 16*(l>>5) + (j&15) + 32*(j>>4)", [](int l, int j) { return 16 * (l >> 5) + (j & 15) + 32 * (j >> 4); }},
      {"k = 4*(l>>5) + (j&3) + 8*(j>>2)", [](int l, int j) { return 4 * (l >> 5) + (j & 3) + 8 * (j >> 2); }},
  };
  int *da, *db, *dsa, *dsb; float* dd;
  hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
  hipMalloc(&dd, 64 * 16 * 4);
  for (int scaled = 0; scaled < 2; ++scaled) {
    std::vector<int> sa(64), sb(64);
    for (int l = 0; l < 64; ++l) {
      sa[l] = scaled ? 127 + rand() % 5 - 2 : 127;
      sb[l] = scaled ? 127 + rand() % 5 - 2 : 127;
    }
    for (auto& [name, km] : maps) {
      std::vector<uint8_t> a(64 * 32), b(64 * 32);
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
          a[l * 32 + j] = enc((int)Am[l & 31][km(l, j)]);
          b[l * 32 + j] = enc((int)Bm[km(l, j)][l & 31]);
        }
      hipMemcpy(da, a.data(), a.size(), hipMemcpyHostToDevice);
      hipMemcpy(db, b.data(), b.size(), hipMemcpyHostToDevice);
      hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
      mx_kernel<<<1, 64>>>(da, db, dsa, dsb, dd);
      std::vector<float> d(64 * 16);
      hipMemcpy(d.data(), dd, d.size() * 4, hipMemcpyDeviceToHost);
      // reference: scale of A row i, k-block kb = the scale byte of the lane holding (i, k) under the
      // same map (one lane per (row, 32-k block) if the map keeps blocks within a lane half)
      double err = 0, mag = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
          const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
          double ref = 0;
          for (int lk = 0; lk < 64; ++lk) {  // lane halves: lanes with (lk & 31) == row hold A's row
            if ((lk & 31) != row) continue;
            for (int j = 0; j < 32; ++j) {
              const int k = km(lk, j);
              // candidate: the scale of (row, k-block kb = k / 32) comes from lane row + 32 * kb
              const int kb = k / 32;
              ref += (double)Am[row][k] * std::ldexp(1.0, sa[row + 32 * kb] - 127) * Bm[k][col] *
                     std::ldexp(1.0, sb[col + 32 * kb] - 127);
            }
          }
          err = std::fmax(err, std::fabs(ref - d[l * 16 + r]));
          mag = std::fmax(mag, std::fabs(ref));
        }
      printf("scaled=%d  %-40s max err %g (max |ref| %g)\n", scaled, name, err, mag);
    }
  }
  return 0;
}
