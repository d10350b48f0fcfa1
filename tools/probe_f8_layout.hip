// Diagnostic: operand lane map of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3, unit scales) and
// v_mfma_scale_f32_16x16x128_f8f6f4, tested with small exact integers against candidate maps.
#include <hip/hip_runtime.h>
#include <hip/hip_fp8.h>
#include <stdio.h>
#include <math.h>
typedef __attribute__((ext_vector_type(8))) int v8i;
typedef __attribute__((ext_vector_type(16))) float v16f;
typedef __attribute__((ext_vector_type(4))) float v4f;

__global__ void k32(const v8i* a, const v8i* b, v16f* d) {
  v16f c = {};
  d[threadIdx.x] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[threadIdx.x], b[threadIdx.x], c, 0, 0, 0, 127, 0, 127);
}
__global__ void k16(const v8i* a, const v8i* b, v4f* d) {
  v4f c = {};
  d[threadIdx.x] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[threadIdx.x], b[threadIdx.x], c, 0, 0, 0, 127, 0, 127);
}
static unsigned char f8(float v) { __hip_fp8_e4m3 x(v); return *(unsigned char*)&x; }

// candidate maps: lane l, byte t (0..31) -> (row-or-col index, k)
// map 0: k = KH*(l/LN) + t (contiguous per lane half)
// map 1: k = 16*(t/16)*HALVES + 16*(l/LN) + t%16 (16-byte groups interleaved over halves)
static void kidx(int map, int l, int t, int LN, int KW, int& idx, int& k) {
  const int nh = 64 / LN;  // lane groups
  idx = l % LN;
  const int g = l / LN;
  if (map == 0) k = (KW / nh) * g + t;
  else k = 16 * nh * (t / 16) + 16 * g + t % 16;
}
int main() {
  const int LN[2] = {32, 16}, KW[2] = {64, 128}, MN[2] = {32, 16};
  for (int shape = 0; shape < 2; ++shape) {
    const int ln = LN[shape], kw = KW[shape], mn = MN[shape];
    static float A[32][128], B[128][32];
    for (int i = 0; i < mn; ++i)
      for (int k = 0; k < kw; ++k) A[i][k] = (float)((i * 7 + k * 3) % 5) - 2.0f, B[k][i] = (float)((i * 5 + k * 11) % 7) - 3.0f;
    for (int map = 0; map < 2; ++map) {
      unsigned char ha[64][32], hb[64][32];
      for (int l = 0; l < 64; ++l)
        for (int t = 0; t < 32; ++t) {
          int idx, k;
          kidx(map, l, t, ln, kw, idx, k);
          ha[l][t] = f8(A[idx][k]);
          hb[l][t] = f8(B[k][idx]);
        }
      void *da, *db, *dd;
      hipMalloc(&da, 2048), hipMalloc(&db, 2048), hipMalloc(&dd, 64 * 16 * 4);
      hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice), hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
      if (shape == 0) k32<<<1, 64>>>((v8i*)da, (v8i*)db, (v16f*)dd);
      else k16<<<1, 64>>>((v8i*)da, (v8i*)db, (v4f*)dd);
      float hd[64][16];
      hipMemcpy(hd, dd, 64 * 16 * 4, hipMemcpyDeviceToHost);
      int bad = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < (shape == 0 ? 16 : 4); ++r) {
          const int col = l % mn;
          const int row = shape == 0 ? (r & 3) + 8 * (r >> 2) + 4 * (l >> 5) : 4 * (l >> 4) + r;
          float ref = 0;
          for (int k = 0; k < kw; ++k) ref += A[row][k] * B[k][col];
          if (fabsf(ref - hd[l][r]) > 1e-3f) ++bad;
        }
      printf("shape %s map %d: %d mismatches\n", shape == 0 ? "32x32x64" : "16x16x128", map, bad);
      hipFree(da), hipFree(db), hipFree(dd);
    }
  }
  return 0;
}
