// Probe: lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) and of v_cvt_pk_fp8_f32 on gfx950.
// Exact small-integer data; prints the max error of each layout hypothesis against a CPU product.
//   hipcc --offload-arch=gfx950 -O2 tools/fp8_probe.hip -o build/fp8_probe && ./build/fp8_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// a/b: [64 lanes][32 bytes] register images; sa/sb: [64] scale bytes; d: [64][4]
__global__ void k_mfma(const uint8_t* a, const uint8_t* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  i32x8_t av, bv;
  for (int r = 0; r < 8; ++r) {
    av[r] = *reinterpret_cast<const int*>(a + l * 32 + 4 * r);
    bv[r] = *reinterpret_cast<const int*>(b + l * 32 + 4 * r);
  }
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

__global__ void k_cvt(const float* x, int* out, int n) {
  int i = threadIdx.x;
  if (2 * i + 1 < n) out[i] = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}

static float e4m3_to_f(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r = e == 0 ? ldexpf((float)m, -9) : ldexpf(1.f + m / 8.f, e - 7);
  if (e == 15 && m == 7) r = NAN;
  return s ? -r : r;
}

int main() {
  // e4m3 codes of small integers -4..4 (0 -> 0x00)
  const uint8_t codes[9] = {0xC8, 0xC4, 0xC0, 0xB8, 0x00, 0x38, 0x40, 0x44, 0x48};
  for (int i = 0; i < 9; ++i) printf("%g ", e4m3_to_f(codes[i]));
  printf("<- e4m3 decode check\n");
  uint8_t ha[64 * 32], hb[64 * 32];
  int hsa[64], hsb[64];
  srand(1);
  for (int i = 0; i < 64 * 32; ++i) { ha[i] = codes[rand() % 9]; hb[i] = codes[rand() % 9]; }
  for (int pass = 0; pass < 2; ++pass) {
    for (int l = 0; l < 64; ++l) {
      hsa[l] = pass ? 127 + (rand() % 5) - 2 : 127;
      hsb[l] = pass ? 127 + (rand() % 5) - 2 : 127;
    }
    uint8_t *da, *db; int *dsa, *dsb; float* dd;
    hipMalloc(&da, 2048); hipMalloc(&db, 2048); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dd, 1024);
    hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice); hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
    k_mfma<<<1, 64>>>(da, db, dsa, dsb, dd);
    float hd[256];
    hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost);
    // hypotheses for (lane, byte) -> k ; rows / cols = lane & 15
    for (int h = 0; h < 3; ++h) {
      float A[16][128], Bm[128][16];
      float As[16][4], Bs[16][4];  // block scale per row / col per 32-k block
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 32; ++j) {
          int k;
          if (h == 0) k = 32 * (l >> 4) + j;
          else if (h == 1) k = j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16);
          else k = 8 * (l >> 4) + (j & 7) + 32 * (j >> 3);
          A[l & 15][k] = e4m3_to_f(ha[l * 32 + j]);
          Bm[k][l & 15] = e4m3_to_f(hb[l * 32 + j]);
        }
      for (int l = 0; l < 64; ++l) { As[l & 15][l >> 4] = ldexpf(1.f, hsa[l] - 127); Bs[l & 15][l >> 4] = ldexpf(1.f, hsb[l] - 127); }
      double maxerr = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
          int row = (l >> 4) * 4 + r, col = l & 15;
          double s = 0;
          for (int k = 0; k < 128; ++k) s += (double)A[row][k] * As[row][k / 32] * Bm[k][col] * Bs[col][k / 32];
          maxerr = fmax(maxerr, fabs(s - hd[l * 4 + r]));
        }
      printf("pass %d (scales %s) hypothesis %d: max err %g\n", pass, pass ? "random" : "unit", h, maxerr);
    }
  }
  // conversion check
  float hx[8] = {1.f, -1.f, 0.5f, 448.f, 3.3f, 0.0078125f, 464.f, 1e-3f};
  float* dx; int* dout; int hout[4];
  hipMalloc(&dx, 32); hipMalloc(&dout, 16);
  hipMemcpy(dx, hx, 32, hipMemcpyHostToDevice);
  k_cvt<<<1, 4>>>(dx, dout, 8);
  hipMemcpy(hout, dout, 16, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i)
    printf("cvt %g %g -> %02x %02x (%g %g)\n", hx[2 * i], hx[2 * i + 1], hout[i] & 255, (hout[i] >> 8) & 255,
           e4m3_to_f(hout[i] & 255), e4m3_to_f((hout[i] >> 8) & 255));
  return 0;
}
