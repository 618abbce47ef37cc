// Probe: operand / scale lane maps of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) on gfx950.
// Each lane passes 32 fp8 bytes of each operand and one E8M0 scale byte each.  The host tests
// candidate maps (lane, byte) -> k and candidate scale owners (row, k-block) -> lane, and prints the
// max error of each against a double reference.  Also checks the output map of the f32x4
// accumulator (lane & 15 = column of src1 ... as for the bf16 16x16x32 form).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void mx_kernel(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  v8i A, B;
  for (int i = 0; i < 8; ++i) { A[i] = a[l * 8 + i]; B[i] = b[l * 8 + i]; }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

static uint8_t enc(int v) {  // small integers exactly in e4m3fn
  static const uint8_t pos[4] = {0x00, 0x38, 0x40, 0x44};
  return v < 0 ? (uint8_t)(0x80 | pos[-v]) : pos[v];
}

int main() {
  srand(11);
  static float Am[16][128], Bm[128][16];
  for (auto& r : Am) for (auto& x : r) x = (float)(rand() % 7 - 3);
  for (auto& r : Bm) for (auto& x : r) x = (float)(rand() % 7 - 3);
  using Map = std::function<int(int, int)>;  // (lane, byte) -> k
  std::vector<std::pair<const char*, Map>> maps = {
      {"k = 32*(l>>4) + j", [](int l, int j) { return 32 * (l >> 4) + j; }},
      {"k = 16*(l>>4) + (j&15) + 64*(j>>4)", [](int l, int j) { return 16 * (l >> 4) + (j & 15) + 64 * (j >> 4); }},
      {"k = 8*(l>>4) + (j&7) + 32*(j>>3)", [](int l, int j) { return 8 * (l >> 4) + (j & 7) + 32 * (j >> 3); }},
      {"k = 4*(l>>4) + (j&3) + 16*(j>>2)", [](int l, int j) { return 4 * (l >> 4) + (j & 3) + 16 * (j >> 2); }},
  };
  // candidate output maps: (lane, r) -> (row of src0 matrix "A", column of src1 matrix "B")
  using OMap = std::function<void(int, int, int&, int&)>;
  std::vector<std::pair<const char*, OMap>> omaps = {
      {"row = 4*(l>>4)+r, col = l&15", [](int l, int r, int& i, int& n) { i = 4 * (l >> 4) + r; n = l & 15; }},
      {"row = l&15, col = 4*(l>>4)+r", [](int l, int r, int& i, int& n) { i = l & 15; n = 4 * (l >> 4) + r; }},
  };
  using SMap = std::function<int(int, int)>;  // (row, k-block) -> lane holding its scale
  std::vector<std::pair<const char*, SMap>> smaps = {
      {"scale lane = row + 16*kb", [](int i, int kb) { return i + 16 * kb; }},
      {"scale lane = row + 32*(kb&1) + 16*(kb>>1)", [](int i, int kb) { return i + 32 * (kb & 1) + 16 * (kb >> 1); }},
      {"scale lane = row (one per row)", [](int i, int kb) { return i; }},
  };
  int *da, *db, *dsa, *dsb; float* dd;
  hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
  hipMalloc(&dd, 64 * 4 * 4);
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
          a[l * 32 + j] = enc((int)Am[l & 15][km(l, j)]);
          b[l * 32 + j] = enc((int)Bm[km(l, j)][l & 15]);
        }
      hipMemcpy(da, a.data(), a.size(), hipMemcpyHostToDevice);
      hipMemcpy(db, b.data(), b.size(), hipMemcpyHostToDevice);
      hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
      hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
      mx_kernel<<<1, 64>>>(da, db, dsa, dsb, dd);
      std::vector<float> d(64 * 4);
      hipMemcpy(d.data(), dd, d.size() * 4, hipMemcpyDeviceToHost);
      for (auto& [oname, om] : omaps)
        for (auto& [sname, sm] : smaps) {
          if (!scaled && sm(0, 1) != 16) continue;  // unit scales: one scale map suffices
          double err = 0, mag = 0;
          for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) {
              int i, n;
              om(l, r, i, n);
              double ref = 0;
              for (int k = 0; k < 128; ++k)
                ref += (double)Am[i][k] * std::ldexp(1.0, sa[sm(i, k / 32)] - 127) * Bm[k][n] *
                       std::ldexp(1.0, sb[sm(n, k / 32)] - 127);
              err = std::fmax(err, std::fabs(ref - d[l * 4 + r]));
              mag = std::fmax(mag, std::fabs(ref));
            }
          printf("scaled=%d  %-38s %-32s %-44s max err %g (max |ref| %g)\n", scaled, name, oname, sname, err, mag);
        }
    }
  }
  return 0;
}
