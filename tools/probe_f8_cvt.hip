// Diagnostic: semantics of the gfx950 scaled fp8 conversions used by the fp8 P.V attention
// (attention_pipe.hip, F8 variants): direction of the scale operand, overflow / underflow results,
// and the byte order of the packed words; read back through the unscaled fp8 -> f32 conversions.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(2))) short s16x2;

__global__ void cvt_kernel(const float* in, const float* scale, int n, unsigned* out8, unsigned* outb8,
                           float* back8, float* backb8, unsigned* sat8) {
  const int i = threadIdx.x;
  if (i >= n) return;
  s16x2 z = {0, 0};
  s16x2 a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, in[i], -in[i], scale[i], false);
  a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(a, 2.0f * in[i], 0.5f, scale[i], true);
  s16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(z, in[i], -in[i], scale[i], false);
  const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
  out8[i] = ua;
  outb8[i] = ub;
  back8[i] = __builtin_amdgcn_cvt_f32_fp8((int)ua, 0);
  backb8[i] = __builtin_amdgcn_cvt_f32_bf8((int)ub, 0);
  sat8[i] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(in[i], 1.0f, 0, false);  // unscaled: saturation?
}

int main() {
  const float vin[] = {1.0f, 8.0f, 8.0f, 8.0f, 300.0f, 1000.0f, 1000.0f, 1e-3f, 3.0f, 0.0f, 100000.0f, 1.0f};
  const float vsc[] = {1.0f, 4.0f, 0.25f, 2.0f, 1.0f, 1.0f, 4.0f, 1.0f, 1.5f, 1.0f, 1.0f, 0x1p-20f};
  const int n = sizeof(vin) / sizeof(float);
  float *din, *dsc, *db8, *dbb8;
  unsigned *d8, *db, *dsat;
  hipMalloc(&din, 64 * 4), hipMalloc(&dsc, 64 * 4), hipMalloc(&d8, 64 * 4), hipMalloc(&db, 64 * 4);
  hipMalloc(&db8, 64 * 4), hipMalloc(&dbb8, 64 * 4), hipMalloc(&dsat, 64 * 4);
  hipMemcpy(din, vin, n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dsc, vsc, n * 4, hipMemcpyHostToDevice);
  cvt_kernel<<<1, 64>>>(din, dsc, n, d8, db, db8, dbb8, dsat);
  unsigned h8[64], hb[64], hs[64];
  float hb8[64], hbb8[64];
  hipMemcpy(h8, d8, n * 4, hipMemcpyDeviceToHost), hipMemcpy(hb, db, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hb8, db8, n * 4, hipMemcpyDeviceToHost), hipMemcpy(hbb8, dbb8, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hs, dsat, n * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i)
    printf("in %-10g scale %-10g  e4m3 word %08x -> %-12g  e5m2 word %08x -> %-12g  unscaled e4m3 %08x\n", vin[i],
           vsc[i], h8[i], hb8[i], hb[i], hbb8[i], hs[i]);
  return 0;
}
