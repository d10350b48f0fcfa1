// Shared device helpers for the MMPFN gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; all MFMA fragment maps are the gfx950 ones
//    (cdna_hip_programming.md section 3):
//      16x16x32 bf16 : lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j=0..7
//      16x16x4  f32  : lane l holds A[l&15][l>>4],      B[l>>4][l&15]
//      32x32x16 bf16 : lane l holds A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31]
//      32x32x2  f32  : lane l holds A[l&31][l>>5],      B[l>>5][l&31]
//      C/D 16x16     : col = l&15, row = 4(l>>4)+r            (r = 0..3)
//      C/D 32x32     : col = l&31, row = (r&3)+8(r>>2)+4(l>>5) (r = 0..15)
//  * "bf16" storage is the clang __bf16 type (RNE conversion, NaN preserving).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace mmpfn {

// Opt-in of a kernel to more than 64 KiB of dynamic LDS.  HIP keeps the attribute per device, so it
// is set once per device that launches the kernel (`opted`: one bit per device, owned by the call
// site) and a failure is returned, never remembered.
inline hipError_t lds_optin(std::atomic<uint64_t>& opted, const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? (uint64_t)1 << dev : 0;
  if (bit && (opted.load(std::memory_order_relaxed) & bit)) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) opted.fetch_or(bit, std::memory_order_relaxed);
  return e;
}

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

// 16-bit MFMA operand types of the performance modes: bf16 (PREC_BF16: fp32 state) or fp16 (PREC_F16:
// fp16 state, the reference's autocast dtype); gfx950 runs both forms at one rate
template <bool F16> struct Op16;
template <> struct Op16<false> {
  typedef __bf16 t;
  typedef bf16x8 x8;
  typedef bf16x4 x4;
};
template <> struct Op16<true> {
  typedef _Float16 t;
  typedef f16x8 x8;
  typedef f16x4 x4;
};
__device__ __forceinline__ f32x4 mfma16x(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ _Float16 from_f32<_Float16>(float x) { return (_Float16)x; }

// erf, branch-free (Abramowitz & Stegun 7.1.26, |abs err| <= 1.5e-7): the libm
// erff is a multi-branch routine that dominated the MLP epilogue.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.0f), x);
}

// GELU with the exact-erf formulation (torch default, approximate='none')
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}

// tanh-form GELU, x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)): |err| <= 3e-4, below the
// bf16 resolution of the activations it feeds; 7 VALU ops (2 transcendental).  Used
// only on the bf16 performance path; the fp32 parity path keeps gelu_erf.
__device__ __forceinline__ float gelu_tanh_fast(float x) {
  const float k = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2 sqrt(2/pi) log2(e)
  const float x2 = x * x;
  const float u = x * fmaf(k * 0.044715f, x2, k);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
}

// the same tanh form on a pair of fp16 values in packed 16-bit arithmetic (fp16 mode, whose hidden
// activations are fp16 MFMA operands anyway): v_pk_mul / v_pk_fma / v_pk_add_f16 take one issue slot per
// pair where the fp32 form takes one per element; v_exp_f16 / v_rcp_f16 per element.  2^u overflowing fp16
// (x < -5.6) gives rcp(inf) = 0, x * 0 = 0, and underflow gives x: GELU's own limits.
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
__device__ __forceinline__ f16x2_t gelu_tanh_h2(f16x2_t x) {
  constexpr float k = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const f16x2_t kk = {(_Float16)k, (_Float16)k}, kc = {(_Float16)(k * 0.044715f), (_Float16)(k * 0.044715f)};
  const f16x2_t one = {(_Float16)1.0f, (_Float16)1.0f};
  const f16x2_t u = x * __builtin_elementwise_fma(kc, x * x, kk);
  const f16x2_t d = f16x2_t{(_Float16)__builtin_exp2f16(u[0]), (_Float16)__builtin_exp2f16(u[1])} + one;
  return x * f16x2_t{(_Float16)__builtin_amdgcn_rcph(d[0]), (_Float16)__builtin_amdgcn_rcph(d[1])};
}

// gelu_tanh_h2 on two pairs at once, bitwise the same values.  The compiler builds each pair's exp / rcp from
// one v_exp_f16 / v_rcp_f16 on the low half, one SDWA form reading the high half, and a v_pack_b32_f16 (2 of
// the pair's 12 issue slots); here the SDWA form writes the high half in place (dst_sel WORD_1, preserve).
// The two pairs alternate so that every read of a transcendental's result comes one instruction after it
// (gfx950's one-wait-state trans-use rule, which the compiler keeps with s_nop outside asm), and the block
// ends with non-transcendental instructions.
__device__ __forceinline__ void gelu_tanh_h2x2(f16x2_t& a, f16x2_t& b) {
  constexpr float k = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const f16x2_t kk = {(_Float16)k, (_Float16)k}, kc = {(_Float16)(k * 0.044715f), (_Float16)(k * 0.044715f)};
  const f16x2_t ua = a * __builtin_elementwise_fma(kc, a * a, kk), ub = b * __builtin_elementwise_fma(kc, b * b, kk);
  f16x2_t ea, eb, ra, rb;
  asm("v_exp_f16_e32 %0, %4\n\t"
      "v_exp_f16_e32 %1, %5\n\t"
      "v_exp_f16_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_exp_f16_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_pk_add_f16 %0, %0, 1.0 op_sel_hi:[1,0]\n\t"
      "v_pk_add_f16 %1, %1, 1.0 op_sel_hi:[1,0]\n\t"
      "v_rcp_f16_e32 %2, %0\n\t"
      "v_rcp_f16_e32 %3, %1\n\t"
      "v_rcp_f16_sdwa %2, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_rcp_f16_sdwa %3, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_pk_mul_f16 %2, %6, %2\n\t"
      "v_pk_mul_f16 %3, %7, %3"
      : "=&v"(ea), "=&v"(eb), "=&v"(ra), "=&v"(rb)
      : "v"(ua), "v"(ub), "v"(a), "v"(b));
  a = ra, b = rb;
}

// gelu_tanh_h2x2 from the four fp32 values (h0, h1) (h2, h3) themselves, conversion and the cubic included: the
// whole two-pair chain in one block, every dependent instruction one slot behind its producer (the wait state
// the compiler keeps after v_pk_fma_f16 and after a transcendental), so that no s_nop is needed inside and the
// block's inputs are old accumulators (no conservative s_nop in front of it either)
__device__ __forceinline__ void gelu_tanh_h2x2_f32(float h0, float h1, float h2, float h3, f16x2_t& a, f16x2_t& b) {
  constexpr float k = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const f16x2_t kk = {(_Float16)k, (_Float16)k}, kc = {(_Float16)(k * 0.044715f), (_Float16)(k * 0.044715f)};
  f16x2_t xa, xb, ua, ub, ra, rb;
  asm("v_cvt_pk_f16_f32 %2, %8, %9\n\t"
      "v_cvt_pk_f16_f32 %3, %10, %11\n\t"
      "v_pk_mul_f16 %4, %2, %2\n\t"
      "v_pk_mul_f16 %5, %3, %3\n\t"
      "v_pk_fma_f16 %4, %4, %6, %7\n\t"
      "v_pk_fma_f16 %5, %5, %6, %7\n\t"
      "v_pk_mul_f16 %4, %2, %4\n\t"
      "v_pk_mul_f16 %5, %3, %5\n\t"
      "v_exp_f16_e32 %0, %4\n\t"
      "v_exp_f16_e32 %1, %5\n\t"
      "v_exp_f16_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_exp_f16_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_pk_add_f16 %4, %0, 1.0 op_sel_hi:[1,0]\n\t"
      "v_pk_add_f16 %5, %1, 1.0 op_sel_hi:[1,0]\n\t"
      "v_rcp_f16_e32 %0, %4\n\t"
      "v_rcp_f16_e32 %1, %5\n\t"
      "v_rcp_f16_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_rcp_f16_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
      "v_pk_mul_f16 %0, %2, %0\n\t"
      "v_pk_mul_f16 %1, %3, %1"
      : "=&v"(ra), "=&v"(rb), "=&v"(xa), "=&v"(xb), "=&v"(ua), "=&v"(ub)
      : "v"(kc), "v"(kk), "v"(h0), "v"(h1), "v"(h2), "v"(h3));
  a = ra, b = rb;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Reductions over the four 16-lane rows of an MFMA C fragment (lanes l, l^16, l^32, l^48):
// v_permlane16/32_swap exchange halves in registers (no LDS round trip like ds_bpermute);
// the swap returns {own, partner} in some order, so combining both words is order-free.
__device__ __forceinline__ float sum_rows4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float max_rows4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// wave sum on DPP row operations + permlane swaps (no LDS round trip, unlike __shfl_xor's ds_bpermute);
// every lane ends with the same value
__device__ __forceinline__ float wave_sum_dpp_f(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));   // quad [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));   // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false));  // row_mirror
  return sum_rows4(v);
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum for 256-thread blocks (4 waves); `red` needs 4 slots
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double r = 0.0;
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 0; i < nw; ++i) r += red[i];
  return r;
}

}  // namespace mmpfn
