// Fused MLP sublayer of the PerFeatureEncoderLayer for gfx950:
//   X <- LayerNorm(X + GELU(X W1^T) W2^T)          (mlp.py:93-104, layer.py:437-455)
//
// One 256-thread block owns 64 rows.  The row tile of X is converted once into LDS;
// the 768-wide hidden layer is produced in four 192-column chunks, each GELU'd into
// an LDS tile and immediately contracted with the matching 192-column slice of W2,
// so the [rows, 768] hidden activations never touch HBM (the unfused pair moved
// 2 x 127 MB per layer at the PAD-UFES shape).  Weights stream from L2 in 128-byte
// K slices (64 bf16 / 32 f32) with the next slice's loads in flight during the
// current slice's MFMAs.  bf16: v_mfma_f32_16x16x32_bf16; f32 (parity):
// v_mfma_f32_16x16x4_f32.  Residual + LayerNorm(no affine) in the epilogue.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int MBM = 64;   // rows per block
constexpr int ME = 192;   // model width
constexpr int MWROW = 144;  // LDS bytes per staged W row (128 + 16 pad)
constexpr int MLN_STRIDE = 196;

// MODE 0: fp32-input MFMA (PREC_F32_MFMA), 1: bf16, 2: parity mode (PREC_F32): X and the GELU'd hidden
// chunk split into bf16 hi / lo planes in LDS, W1 / W2 given as hi | lo planes (capi.cpp upsplit), three
// bf16 products per contraction; 157 KB of LDS, one block per CU
template <int MODE>
struct MlpLds {
  static constexpr int NP = MODE == 2 ? 2 : 1;  // operand planes
  static constexpr int EB = MODE == 0 ? 4 : 2;
  // x3: unpadded 384-B A / H rows with 16-B units XOR-swizzled by (row >> 1) & 7 and 160-B W rows -- both
  // conflict-free for the 16x16x32 fragment reads, and the five images fit 160 KB (2-way conflicts with
  // the padded 400 / 144-B rows of the other modes)
  static constexpr int AROW = MODE == 2 ? ME * EB : ME * EB + 16;  // bytes per A / H row
  static constexpr int WROW = MODE == 2 ? 160 : MWROW;             // bytes per staged W row
  static constexpr int A_BYTES = MBM * AROW;
  static constexpr int W_BYTES = ME * WROW;
  static constexpr int TOTAL = NP * (2 * A_BYTES + W_BYTES);
  static constexpr int LN_BYTES = MBM * MLN_STRIDE * 4;
  static constexpr int BYTES = TOTAL > LN_BYTES ? TOTAL : LN_BYTES;
};

// byte offset of byte b of row r in an x3 A / H image
__device__ __forceinline__ int x3_aoff(int r, int b) { return r * (ME * 2) + ((((b >> 4) ^ ((r >> 1) & 7))) << 4) + (b & 15); }

template <int MODE>
__global__ __launch_bounds__(256, MODE == 2 ? 1 : 2) void mlp_fused_kernel(float* __restrict__ X,
                                                                           const void* __restrict__ W1p,
                                                                           const void* __restrict__ W2p, int M, int Fh,
                                                                           float eps) {
  constexpr bool BF16 = MODE != 0, X3 = MODE == 2;
  using L = MlpLds<MODE>;
  constexpr int EB = L::EB;
  constexpr int BK = 128 / EB;          // K per W slice
  constexpr int SPC = ME / BK;          // slices per 192-wide contraction (3 bf16 / 6 f32)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* As = smem;
  unsigned char* Hs = smem + L::A_BYTES;
  unsigned char* Ws = smem + 2 * L::A_BYTES;
  unsigned char* Asl = smem + 2 * L::A_BYTES + L::W_BYTES;  // x3 lo planes
  unsigned char* Hsl = Asl + L::A_BYTES;
  unsigned char* Wsl = Hsl + L::A_BYTES;
  const unsigned char* W1 = (const unsigned char*)W1p;
  const unsigned char* W2 = (const unsigned char*)W2p;
  const int64_t lo1 = X3 ? (int64_t)Fh * ME * 2 : 0, lo2 = lo1;  // bytes from a hi plane to its lo plane

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int m0 = blockIdx.x * MBM;
  const int nchunks = Fh / ME;

  // ---- X tile -> LDS (compute dtype); rows beyond M are zero
  for (int i = tid; i < MBM * ME / 4; i += 256) {
    const int row = i / (ME / 4), c4 = i % (ME / 4);
    const int64_t m = m0 + row;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (m < M) v = *(const f32x4*)(X + m * ME + c4 * 4);
    if constexpr (X3) {
      bf16x4 b, l;
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = (bf16)v[i], l[i] = (bf16)(v[i] - (float)b[i]);
      *(bf16x4*)(As + x3_aoff(row, c4 * 8)) = b;
      *(bf16x4*)(Asl + x3_aoff(row, c4 * 8)) = l;
    } else if constexpr (BF16) {
      bf16x4 b;
      b[0] = (bf16)v[0]; b[1] = (bf16)v[1]; b[2] = (bf16)v[2]; b[3] = (bf16)v[3];
      *(bf16x4*)(As + row * L::AROW + c4 * 8) = b;
    } else {
      *(f32x4*)(As + row * L::AROW + c4 * 16) = v;
    }
  }

  // ---- W slice staging (16-byte chunks, 6 per thread); a slice is 192 rows x 128 B
  constexpr int WCH = ME * 8 / 256;
  u32x4 rw[WCH], rwl[X3 ? WCH : 1];
  auto wload = [&](const unsigned char* base, int64_t ld_bytes) {
#pragma unroll
    for (int j = 0; j < WCH; ++j) {
      const int cidx = tid + 256 * j;
      rw[j] = *(const u32x4*)(base + (cidx >> 3) * ld_bytes + (cidx & 7) * 16);
      if constexpr (X3) rwl[j] = *(const u32x4*)(base + lo1 + (cidx >> 3) * ld_bytes + (cidx & 7) * 16);
    }
  };
  // W1 [Fh][E]: slice (c, ks) = rows c*192.., cols ks*BK..;  W2 [E][Fh]: rows 0..191, cols c*192 + ks*BK..
  auto w1slice = [&](int c, int ks) { wload(W1 + ((int64_t)c * ME * ME + ks * BK) * EB, (int64_t)ME * EB); };
  auto w2slice = [&](int c, int ks) { wload(W2 + ((int64_t)c * ME + ks * BK) * EB, (int64_t)Fh * EB); };
  auto wstore = [&]() {
#pragma unroll
    for (int j = 0; j < WCH; ++j) {
      const int cidx = tid + 256 * j;
      *(u32x4*)(Ws + (cidx >> 3) * L::WROW + (cidx & 7) * 16) = rw[j];
      if constexpr (X3) *(u32x4*)(Wsl + (cidx >> 3) * L::WROW + (cidx & 7) * 16) = rwl[j];
    }
  };
  (void)lo2;

  f32x4 accy[2][6], acch[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) accy[a][b] = acch[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma_slice = [&](const unsigned char* Asrc, int ks, f32x4 (&acc)[2][6]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kb = ks * 128 + kk * 64 + fg * 16;  // byte offset inside the A/H row
      if constexpr (X3) {
        const unsigned char* Asl_ = Asrc == As ? Asl : Hsl;
        bf16x8 af[2], afl[2], bw[6], bwl[6];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          af[mt] = *(const bf16x8*)(Asrc + x3_aoff(wm * 32 + mt * 16 + fr, kb));
          afl[mt] = *(const bf16x8*)(Asl_ + x3_aoff(wm * 32 + mt * 16 + fr, kb));
        }
#pragma unroll
        for (int nt = 0; nt < 6; ++nt) {
          bw[nt] = *(const bf16x8*)(Ws + (wn * 96 + nt * 16 + fr) * L::WROW + kk * 64 + fg * 16);
          bwl[nt] = *(const bf16x8*)(Wsl + (wn * 96 + nt * 16 + fr) * L::WROW + kk * 64 + fg * 16);
        }
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 6; ++nt) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[mt], bw[nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bwl[nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[nt], acc[mt][nt], 0, 0, 0);
          }
      } else if constexpr (BF16) {
        bf16x8 af[2], bw[6];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) af[mt] = *(const bf16x8*)(Asrc + (wm * 32 + mt * 16 + fr) * L::AROW + kb);
#pragma unroll
        for (int nt = 0; nt < 6; ++nt)
          bw[nt] = *(const bf16x8*)(Ws + (wn * 96 + nt * 16 + fr) * MWROW + kk * 64 + fg * 16);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 6; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[nt], acc[mt][nt], 0, 0, 0);
      } else {
        f32x4 af[2], bw[6];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) af[mt] = *(const f32x4*)(Asrc + (wm * 32 + mt * 16 + fr) * L::AROW + kb);
#pragma unroll
        for (int nt = 0; nt < 6; ++nt)
          bw[nt] = *(const f32x4*)(Ws + (wn * 96 + nt * 16 + fr) * MWROW + kk * 64 + fg * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < 6; ++nt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt][e], bw[nt][e], acc[mt][nt], 0, 0, 0);
      }
    }
  };

  w1slice(0, 0);
  for (int c = 0; c < nchunks; ++c) {
    // hidden chunk c = GELU(A . W1[c*192 : c*192+192]^T)
#pragma unroll
    for (int ks = 0; ks < SPC; ++ks) {
      __syncthreads();
      wstore();
      __syncthreads();
      if (ks + 1 < SPC) w1slice(c, ks + 1);
      else w2slice(c, 0);
      mma_slice(As, ks, acch);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 6; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = wm * 32 + mt * 16 + fg * 4 + r;
          const int cl = wn * 96 + nt * 16 + fr;
          if constexpr (X3) {
            const float g = gelu_erf(acch[mt][nt][r]);
            const bf16 gh = (bf16)g;
            *(bf16*)(Hs + x3_aoff(rl, cl * 2)) = gh;
            *(bf16*)(Hsl + x3_aoff(rl, cl * 2)) = (bf16)(g - (float)gh);
          } else if constexpr (BF16)
            *(bf16*)(Hs + rl * L::AROW + cl * 2) = (bf16)gelu_tanh_fast(acch[mt][nt][r]);
          else
            *(float*)(Hs + rl * L::AROW + cl * 4) = gelu_erf(acch[mt][nt][r]);
          acch[mt][nt][r] = 0.f;
        }
    // Y += H_c . W2[:, c*192 : c*192+192]^T  (the first slice's barrier publishes H_c)
#pragma unroll
    for (int ks = 0; ks < SPC; ++ks) {
      __syncthreads();
      wstore();
      __syncthreads();
      if (ks + 1 < SPC) w2slice(c, ks + 1);
      else if (c + 1 < nchunks) w1slice(c + 1, 0);
      mma_slice(Hs, ks, accy);
    }
  }

  // ---- residual + LayerNorm epilogue (rows owned by this block only)
  float* Es = (float*)smem;
  __syncthreads();
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 6; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 32 + mt * 16 + fg * 4 + r;
        const int cl = wn * 96 + nt * 16 + fr;
        const int64_t m = m0 + rl;
        float v = accy[mt][nt][r];
        const float xr = X[min(m, (int64_t)M - 1) * ME + cl];
        v += (m < M) ? xr : 0.f;
        Es[rl * MLN_STRIDE + cl] = v;
      }
  __syncthreads();
  const int row = tid >> 2, part = tid & 3;
  const int64_t m = m0 + row;
  const float* er = Es + row * MLN_STRIDE + part * 48;
  float s = 0.f;
#pragma unroll 8
  for (int i = 0; i < 48; ++i) s += er[i];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  const float mean = s * (1.0f / ME);
  float q = 0.f;
#pragma unroll 8
  for (int i = 0; i < 48; ++i) {
    const float dl = er[i] - mean;
    q += dl * dl;
  }
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  const float inv = 1.0f / sqrtf(q * (1.0f / ME) + eps);
  if (m < M) {
    float* xo = X + m * ME + part * 48;
#pragma unroll
    for (int i = 0; i < 48; i += 4) {
      f32x4 o;
      o[0] = (er[i] - mean) * inv;
      o[1] = (er[i + 1] - mean) * inv;
      o[2] = (er[i + 2] - mean) * inv;
      o[3] = (er[i + 3] - mean) * inv;
      *(f32x4*)(xo + i) = o;
    }
  }
}

}  // namespace

hipError_t launch_mlp_fused(float* X, const void* W1, const void* W2, int64_t M, int E, int Fh, float eps, int prec,
                            hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (E != ME || Fh % ME != 0) return hipErrorInvalidValue;
  dim3 grid((M + MBM - 1) / MBM);
  static bool attr_set = false;  // > 64 KiB dynamic LDS needs an explicit opt-in
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)mlp_fused_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       MlpLds<1>::BYTES);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)mlp_fused_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            MlpLds<0>::BYTES);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)mlp_fused_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            MlpLds<2>::BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (prec == PREC_BF16)
    hipLaunchKernelGGL(mlp_fused_kernel<1>, grid, dim3(256), MlpLds<1>::BYTES, st, X, W1, W2, (int)M, Fh, eps);
  else if (prec == PREC_F32)  // W1 / W2: hi | lo planes
    hipLaunchKernelGGL(mlp_fused_kernel<2>, grid, dim3(256), MlpLds<2>::BYTES, st, X, W1, W2, (int)M, Fh, eps);
  else
    hipLaunchKernelGGL(mlp_fused_kernel<0>, grid, dim3(256), MlpLds<0>::BYTES, st, X, W1, W2, (int)M, Fh, eps);
  return hipGetLastError();
}

}  // namespace mmpfn
