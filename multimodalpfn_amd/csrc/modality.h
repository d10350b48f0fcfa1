// Internal launch interface of the modality-encoder kernels (modality.hip; not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace mmpfn {

enum GtEpi : int {
  GT_BF16 = 0,   // C bf16 [M][ldc] = act(acc + bias)
  GT_RESID = 1,  // C fp32 [M][ldc] += gamma (.) (acc + bias)   (gamma null: 1)
  GT_F32 = 2,    // C fp32 [M][ldc] = acc + bias
};

// bf16 C = A[M][K] . W[N][K]^T on 256 x 256 tiles; N % 256 == 0, K % 32 == 0, A rows K apart;
// act (GT_BF16 only): 0 none, 1 GELU (erf)
hipError_t launch_gemm_tile(const void* A, const void* W, const float* bias, const float* gamma, void* C,
                            int64_t ldc, int M, int N, int K, int epi, int act, hipStream_t st);

// softmax attention, head_dim 64, over B sequences of L tokens; qkv rows (b * L + t) = [q | k | v]
// (each H x 64, element type of prec); queries [q0, q0 + nq) of every head; output row
// b * o_bstride + (q - q0), column h * 64 + d; kbias [B][L] additive key bias (0 / -inf) or null
hipError_t launch_attn64(const void* qkv, const float* kbias, void* out, int B, int L, int H, int q0, int nq,
                         int64_t o_bstride, int prec, hipStream_t st);

// LayerNorm over rows (affine when gamma / beta given): fp32 out (may alias in) and / or bf16 out;
// row strides in elements (<= 0: dim)
hipError_t launch_ln_dual(const float* in, int64_t rows, int dim, float eps, float* out32, void* out16,
                          const float* gamma, const float* beta, hipStream_t st, int64_t in_rstride = 0,
                          int64_t out_rstride = 0);

hipError_t launch_im2col(const float* img, int B, int C, int H, int W, int P, int Kpad, void* out, bool out_f32,
                         hipStream_t st);
// bicubic resampling of a [1 + M*M][D] positional table to [1 + oh*ow][D]; sh / sw = source pixels
// per output pixel (torch upsample_bicubic2d with the given scale factors)
hipError_t launch_pos_interp(const float* pos, int M, int D, int oh, int ow, float sh, float sw, float* out,
                             hipStream_t st);
hipError_t launch_vit_assemble(const float* patches, const float* cls, const float* pe, int B, int np, int D,
                               float* X, hipStream_t st);
// flag |= 1 when an id / type is out of range (clamped)
hipError_t launch_text_embed(const int* ids, const int* types, int64_t ntok, int L, int E, const float* wemb,
                             const float* pemb, const float* temb, const float* g, const float* b, float eps,
                             float* out32, void* out16, int vocab, int ntypes, int* flag, hipStream_t st);
hipError_t launch_resid(float* X, const float* Y, const float* gamma, int64_t rows, int dim, hipStream_t st);
hipError_t launch_gather_rows(const void* in, int64_t in_rstride, int rows, int dim, void* out, int elem_bytes,
                              hipStream_t st);
hipError_t launch_mask_bias(const int* mask, float* out, int64_t n, hipStream_t st);
hipError_t launch_cast_bf16(const float* in, void* out, int64_t n, hipStream_t st);

}  // namespace mmpfn
