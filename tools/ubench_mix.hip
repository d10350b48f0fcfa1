// Microbenchmark (diagnostic tool): does v_exp_f32 / v_cvt_pk_bf16_f32 issue overlap
// v_mfma_f32_32x32x16_bf16 on one gfx950 SIMD?  Loop body = NM independent-chain MFMAs +
// NE exps (+ NC cvt_pk), cycles per body per SIMD at 1/2/4 waves per SIMD (2.0 GHz basis).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;

#define E16 asm volatile("v_exp_f32 %0, %0\nv_exp_f32 %1, %1\nv_exp_f32 %2, %2\nv_exp_f32 %3, %3\nv_exp_f32 %4, %4\nv_exp_f32 %5, %5\nv_exp_f32 %6, %6\nv_exp_f32 %7, %7\nv_exp_f32 %8, %8\nv_exp_f32 %9, %9\nv_exp_f32 %10, %10\nv_exp_f32 %11, %11\nv_exp_f32 %12, %12\nv_exp_f32 %13, %13\nv_exp_f32 %14, %14\nv_exp_f32 %15, %15\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define E4(q) asm volatile("v_exp_f32 %0, %0\nv_exp_f32 %1, %1\nv_exp_f32 %2, %2\nv_exp_f32 %3, %3\n" : "+v"(r[4*(q)]), "+v"(r[4*(q)+1]), "+v"(r[4*(q)+2]), "+v"(r[4*(q)+3]))
#define H16 asm volatile("v_exp_f16 %0, %0\nv_exp_f16 %1, %1\nv_exp_f16 %2, %2\nv_exp_f16 %3, %3\nv_exp_f16 %4, %4\nv_exp_f16 %5, %5\nv_exp_f16 %6, %6\nv_exp_f16 %7, %7\nv_exp_f16 %8, %8\nv_exp_f16 %9, %9\nv_exp_f16 %10, %10\nv_exp_f16 %11, %11\nv_exp_f16 %12, %12\nv_exp_f16 %13, %13\nv_exp_f16 %14, %14\nv_exp_f16 %15, %15\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define W16 asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %1, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %2, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %4, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %5, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %6, %6 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %7, %7 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %8, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %9, %9 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %10, %10 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %11, %11 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %12, %12 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %13, %13 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %14, %14 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\nv_exp_f16_sdwa %15, %15 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define C8 asm volatile("v_cvt_pk_bf16_f32 %0, %0, %1\nv_cvt_pk_bf16_f32 %1, %1, %2\nv_cvt_pk_bf16_f32 %2, %2, %3\nv_cvt_pk_bf16_f32 %3, %3, %4\nv_cvt_pk_bf16_f32 %4, %4, %5\nv_cvt_pk_bf16_f32 %5, %5, %6\nv_cvt_pk_bf16_f32 %6, %6, %7\nv_cvt_pk_bf16_f32 %7, %7, %0\n" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]))

#define F16 asm volatile("v_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\nv_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8\n" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]) : "v"(k))
#define P16 asm volatile("v_pk_fma_f32 %0, %0, %8, %8\nv_pk_fma_f32 %1, %1, %8, %8\nv_pk_fma_f32 %2, %2, %8, %8\nv_pk_fma_f32 %3, %3, %8, %8\nv_pk_fma_f32 %4, %4, %8, %8\nv_pk_fma_f32 %5, %5, %8, %8\nv_pk_fma_f32 %6, %6, %8, %8\nv_pk_fma_f32 %7, %7, %8, %8\n" : "+v"(pf[0]), "+v"(pf[1]), "+v"(pf[2]), "+v"(pf[3]), "+v"(pf[4]), "+v"(pf[5]), "+v"(pf[6]), "+v"(pf[7]) : "v"(pk))
typedef __attribute__((__vector_size__(2 * sizeof(float)))) float f32x2;

template <int NM, int NE, int NC, int NA = 4, bool AG = false, int NF = 0, int NP = 0, int XV = 0>
__global__ void kern(float* out, int iters) {
  float r[16], c[8], f[8];
  f32x2 pf[8];
  const float k = 0.999f;
  f32x2 pk = {0.999f, 0.5f};
  for (int i = 0; i < 8; ++i) f[i] = 0.1f * i, pf[i] = f32x2{0.2f * i, 0.3f};
  for (int i = 0; i < 16; ++i) r[i] = -1.0f / (threadIdx.x + i + 1);
  for (int i = 0; i < 8; ++i) c[i] = 0.5f / (threadIdx.x + i + 1);
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)(threadIdx.x * 0.001f), b[i] = (__bf16)(i * 0.01f);
  for (int it = 0; it < iters; ++it) {
    if constexpr (XV == 3) {  // interleaved in program order: MFMA, 4 exps, MFMA, 4 exps ...
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
        E4(j);
      }
      continue;
    }
    if constexpr (XV == 4) {  // same, with the 4-exp groups behind s_setprio 0 / MFMA at prio 1
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __builtin_amdgcn_s_setprio(1);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        E4(j);
      }
      continue;
    }
    if constexpr (XV == 6) {  // 8 x 16x16x32 (same flops as 4 x 32x32x16) + the exps
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f32x4 t = {acc[j & 3][4 * (j >> 2)], acc[j & 3][4 * (j >> 2) + 1], acc[j & 3][4 * (j >> 2) + 2], acc[j & 3][4 * (j >> 2) + 3]};
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, t, 0, 0, 0);
        acc[j & 3][4 * (j >> 2)] = t[0], acc[j & 3][4 * (j >> 2) + 1] = t[1], acc[j & 3][4 * (j >> 2) + 2] = t[2], acc[j & 3][4 * (j >> 2) + 3] = t[3];
      }
#pragma unroll
      for (int j = 0; j < NE / 16; ++j) E16;
      continue;
    }
    if constexpr (XV == 5) {  // 16x16x32 MFMAs (4 per 32x32x16 equivalent) interleaved with exps
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        f32x4 t = {acc[j & 3][0], acc[j & 3][1], acc[j & 3][2], acc[j & 3][3]};
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, t, 0, 0, 0);
        acc[j & 3][0] = t[0], acc[j & 3][1] = t[1], acc[j & 3][2] = t[2], acc[j & 3][3] = t[3];
        if ((j & 3) == 3) E4(j >> 2);
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < NM; ++j) {
      if constexpr (AG)  // accumulator in AGPRs (separate from the VALU's VGPR operands)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j % NA]) : "v"(a), "v"(b));
      else
        acc[j % NA] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j % NA], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NE / 16; ++j) {
      if constexpr (XV == 1) H16; else if constexpr (XV == 2) W16; else E16;
    }
#pragma unroll
    for (int j = 0; j < NC / 8; ++j) C8;
#pragma unroll
    for (int j = 0; j < NF / 16; ++j) F16;
#pragma unroll
    for (int j = 0; j < NP / 8; ++j) P16;
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += r[i] + acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
  for (int i = 0; i < 8; ++i) s += c[i] + f[i] + pf[i][0] + pf[i][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NM, int NE, int NC, int NA = 4, bool AG = false, int NF = 0, int NP = 0, int XV = 0>
void run() {
  const int shapes[][2] = {{512, 256}, {512, 512}};
  for (auto& sh : shapes) {
    const int blocks = sh[0], threads = sh[1], iters = 4000;
    float* out;
    (void)hipMalloc(&out, blocks * threads * 4);
    kern<NM, NE, NC, NA, AG, NF, NP, XV><<<blocks, threads>>>(out, iters);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<NM, NE, NC, NA, AG, NF, NP, XV><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wps = (double)blocks * threads / 64 / 1024;
    const double per = ms * 1e-3 / (iters * wps) * 2.0e9;
    printf("exp%s %s chains %d mfma32 x%d + exp x%2d + cvt x%2d + fma x%2d + pkfma x%2d grid %4dx%3d waves/SIMD %.0f: %6.1f cyc/body/SIMD\n", XV == 0 ? "f32" : XV == 1 ? "f16" : XV == 2 ? "f16sdwa" : XV == 3 ? "f32-il" : XV == 4 ? "f32-il-prio" : XV == 5 ? "f32-il-16x16" : "8x16x16x32", AG ? "agpr" : "vgpr", NA, NM, NE, NC, NF, NP, blocks,
           threads, wps, per);
    (void)hipFree(out);
  }
}

int main() {
  run<4, 0, 0, 4, false, 0, 0, 0>();
  run<4, 0, 0, 4, false, 0, 0, 6>();
  run<4, 16, 0, 4, false, 0, 0, 0>();
  run<4, 16, 0, 4, false, 0, 0, 6>();
  run<4, 32, 0, 4, false, 0, 0, 0>();
  run<4, 32, 0, 4, false, 0, 0, 6>();
  return 0;
}
