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

// MODE 0: fp32-input MFMA (PREC_F32_MFMA), 1: bf16 (the parity mode runs mlp_x3_kernel below)
template <int MODE>
struct MlpLds {
  static constexpr int EB = MODE == 0 ? 4 : 2;
  static constexpr int AROW = ME * EB + 16;  // bytes per A / H row
  static constexpr int WROW = MWROW;         // bytes per staged W row
  static constexpr int A_BYTES = MBM * AROW;
  static constexpr int W_BYTES = ME * WROW;
  static constexpr int TOTAL = 2 * A_BYTES + W_BYTES;
  static constexpr int LN_BYTES = MBM * MLN_STRIDE * 4;
  static constexpr int BYTES = TOTAL > LN_BYTES ? TOTAL : LN_BYTES;
};

template <int MODE>
__global__ __launch_bounds__(256, 2) void mlp_fused_kernel(float* __restrict__ X,
                                                                           const void* __restrict__ W1p,
                                                                           const void* __restrict__ W2p, int M, int Fh,
                                                                           float eps) {
  constexpr bool BF16 = MODE != 0;
  using L = MlpLds<MODE>;
  constexpr int EB = L::EB;
  constexpr int BK = 128 / EB;          // K per W slice
  constexpr int SPC = ME / BK;          // slices per 192-wide contraction (3 bf16 / 6 f32)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* As = smem;
  unsigned char* Hs = smem + L::A_BYTES;
  unsigned char* Ws = smem + 2 * L::A_BYTES;
  const unsigned char* W1 = (const unsigned char*)W1p;
  const unsigned char* W2 = (const unsigned char*)W2p;

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
    if constexpr (BF16) {
      bf16x4 b;
      b[0] = (bf16)v[0]; b[1] = (bf16)v[1]; b[2] = (bf16)v[2]; b[3] = (bf16)v[3];
      *(bf16x4*)(As + row * L::AROW + c4 * 8) = b;
    } else {
      *(f32x4*)(As + row * L::AROW + c4 * 16) = v;
    }
  }

  // ---- W slice staging (16-byte chunks, 6 per thread); a slice is 192 rows x 128 B
  constexpr int WCH = ME * 8 / 256;
  u32x4 rw[WCH];
  auto wload = [&](const unsigned char* base, int64_t ld_bytes) {
#pragma unroll
    for (int j = 0; j < WCH; ++j) {
      const int cidx = tid + 256 * j;
      rw[j] = *(const u32x4*)(base + (cidx >> 3) * ld_bytes + (cidx & 7) * 16);
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
    }
  };


  f32x4 accy[2][6], acch[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) accy[a][b] = acch[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma_slice = [&](const unsigned char* Asrc, int ks, f32x4 (&acc)[2][6]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kb = ks * 128 + kk * 64 + fg * 16;  // byte offset inside the A/H row
      if constexpr (BF16) {
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
          if constexpr (BF16)
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

// ---------------------------------------------------------------- parity mode, row-resident
// PREC_F32 MLP sublayer with the layout of mlp_rows.hip (each wave keeps its 16 tokens in registers:
// X^T as B fragments, the 192 x 16 Y^T accumulators initialised with the fp32 residual; H^T = W1c . X^T
// per 32-hidden chunk, its GELU(erf) the B fragment of Y^T += W2c . H^T) on split-bf16 operands: X^T, H^T
// and the weights as bf16 hi + lo, three products per contraction.  Only the weights go through LDS: a
// chunk's W1 rows and W2 columns (hi and lo planes, 48 KB, XOR-swizzled for conflict-free ds_read_b128)
// staged by registers once per 64-token block, so no activation moves through LDS and two waves share a
// SIMD (the LDS-staged GEMM form of mlp_fused_kernel<2> ran one).
constexpr int X3_HC = 32;                        // hidden chunk
constexpr int X3_W1P = X3_HC * ME * 2;           // W1 chunk plane: 32 rows x 384 B
constexpr int X3_W2P = ME * X3_HC * 2;           // W2 chunk plane: 192 rows x 64 B
constexpr int X3_LDS = 2 * X3_W1P + 2 * X3_W2P;  // 48 KB

__device__ __forceinline__ bf16x8 x3_hi(const f32x4& a, const f32x4& b, bf16x8& lo) {
  bf16x8 hi;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    hi[i] = (bf16)a[i], hi[4 + i] = (bf16)b[i];
    lo[i] = (bf16)(a[i] - (float)hi[i]), lo[4 + i] = (bf16)(b[i] - (float)hi[4 + i]);
  }
  return hi;
}

__global__ __launch_bounds__(256, 2) void mlp_x3_kernel(float* __restrict__ X, const bf16* __restrict__ W1,
                                                        const bf16* __restrict__ W2p, int M, int Fh, float eps) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[X3_LDS];
  unsigned char* W1h = lds;
  unsigned char* W1l = lds + X3_W1P;
  unsigned char* W2h = lds + 2 * X3_W1P;
  unsigned char* W2l = W2h + X3_W2P;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * 64 + wave * 16;
  const int64_t mrow = min(m0 + fr, (int64_t)M - 1);
  const int nchunks = Fh / X3_HC;
  const int64_t n1 = (int64_t)Fh * ME, n2 = n1;  // elements of one plane (W1 / W2)

  // ---- staging: 3 units per thread and plane for W1 (rows c*32.., 24 units each) and W2 (192 rows x 4 units)
  u32x4 s1h[3], s1l[3], s2h[3], s2l[3];
  auto gload = [&](int c) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int q = tid + 256 * j;
      const int r1 = q / 24, u1 = q % 24;
      const bf16* a = W1 + ((int64_t)(c * X3_HC + r1) * ME + u1 * 8);
      s1h[j] = *(const u32x4*)a, s1l[j] = *(const u32x4*)(a + n1);
      const int r2 = q >> 2, u2 = q & 3;
      const bf16* b = W2p + ((int64_t)r2 * Fh + c * X3_HC + u2 * 8);
      s2h[j] = *(const u32x4*)b, s2l[j] = *(const u32x4*)(b + n2);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int q = tid + 256 * j;
      const int r1 = q / 24, u1 = q % 24;
      const int o1 = r1 * 384 + ((u1 ^ ((r1 >> 1) & 7)) << 4);
      *(u32x4*)(W1h + o1) = s1h[j], *(u32x4*)(W1l + o1) = s1l[j];
      const int r2 = q >> 2, u2 = q & 3;
      const int o2 = r2 * 64 + ((u2 ^ ((r2 >> 1) & 3)) << 4);
      *(u32x4*)(W2h + o2) = s2h[j], *(u32x4*)(W2l + o2) = s2l[j];
    }
  };
  gload(0);

  // ---- the wave's 16 tokens: Y^T accumulators (residual) and X^T fragments (hi / lo)
  f32x4 y[ME / 16];
  bf16x8 xh[ME / 32], xl[ME / 32];
  {
    const float* xr = X + mrow * ME;
#pragma unroll
    for (int o = 0; o < ME / 16; ++o) y[o] = *(const f32x4*)(xr + 16 * o + 4 * fg);
#pragma unroll
    for (int ks = 0; ks < ME / 32; ++ks)
      xh[ks] = x3_hi(*(const f32x4*)(xr + 32 * ks + 8 * fg), *(const f32x4*)(xr + 32 * ks + 8 * fg + 4), xl[ks]);
  }
  const int w1o = fr * 384, w1s = (fr >> 1) & 7;  // W1 fragment row 16 ht + fr (the swizzle ignores ht)
  const int w2o = fr * 64 + ((fg ^ ((fr >> 1) & 3)) << 4);

  for (int c = 0; c < nchunks; ++c) {
    __syncthreads();  // every wave is done with chunk c-1's images
    lstore();
    __syncthreads();
    if (c + 1 < nchunks) gload(c + 1);
    // H^T [32 hidden][16 tokens] = W1c . X^T
    f32x4 h[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < ME / 32; ++ks)
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) {
        const int off = ht * 16 * 384 + w1o + (((4 * ks + fg) ^ w1s) << 4);
        const bf16x8 wh = *(const bf16x8*)(W1h + off), wl = *(const bf16x8*)(W1l + off);
        h[ht] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh[ks], h[ht], 0, 0, 0);
        h[ht] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl[ks], h[ht], 0, 0, 0);
        h[ht] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh[ks], h[ht], 0, 0, 0);
      }
    // GELU(erf) -> B fragment of the down-projection: position 8fg + j <-> hidden (j < 4 ? 4fg + j : 16 + 4fg + j-4)
    bf16x8 gh, gl;
    {
      f32x4 g0, g1;
#pragma unroll
      for (int i = 0; i < 4; ++i) g0[i] = gelu_erf(h[0][i]), g1[i] = gelu_erf(h[1][i]);
      gh = x3_hi(g0, g1, gl);
    }
    // Y^T [192][16 tokens] += W2c(perm) . GELU(H^T)
#pragma unroll
    for (int o = 0; o < ME / 16; ++o) {
      const int off = o * 16 * 64 + w2o;
      const bf16x8 wh = *(const bf16x8*)(W2h + off), wl = *(const bf16x8*)(W2l + off);
      y[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, gh, y[o], 0, 0, 0);
      y[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, gl, y[o], 0, 0, 0);
      y[o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, gh, y[o], 0, 0, 0);
    }
  }

  // ---- residual (in y) + LayerNorm: lane = token fr, features 16o + 4fg + i
  float sm = 0.f;
#pragma unroll
  for (int o = 0; o < ME / 16; ++o)
#pragma unroll
    for (int i = 0; i < 4; ++i) sm += y[o][i];
  const float mean = sum_rows4(sm) * (1.0f / ME);
  float q = 0.f;
#pragma unroll
  for (int o = 0; o < ME / 16; ++o)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dl = y[o][i] - mean;
      q += dl * dl;
    }
  const float inv = 1.0f / sqrtf(sum_rows4(q) * (1.0f / ME) + eps);
  if (m0 + fr < M) {
    float* xo = X + (m0 + fr) * ME + 4 * fg;
#pragma unroll
    for (int o = 0; o < ME / 16; ++o)
      *(f32x4*)(xo + 16 * o) =
          f32x4{(y[o][0] - mean) * inv, (y[o][1] - mean) * inv, (y[o][2] - mean) * inv, (y[o][3] - mean) * inv};
  }
}

}  // namespace

hipError_t launch_mlp_fused(float* X, const void* W1, const void* W2, int64_t M, int E, int Fh, float eps, int prec,
                            hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (E != ME || Fh % ME != 0) return hipErrorInvalidValue;
  dim3 grid((M + MBM - 1) / MBM);
  static std::atomic<uint64_t> opted1{0}, opted0{0};  // > 64 KiB dynamic LDS needs an explicit opt-in
  hipError_t e = lds_optin(opted1, (const void*)mlp_fused_kernel<1>, MlpLds<1>::BYTES);
  if (e != hipSuccess) return e;
  e = lds_optin(opted0, (const void*)mlp_fused_kernel<0>, MlpLds<0>::BYTES);
  if (e != hipSuccess) return e;
  if (prec == PREC_BF16)
    hipLaunchKernelGGL(mlp_fused_kernel<1>, grid, dim3(256), MlpLds<1>::BYTES, st, X, W1, W2, (int)M, Fh, eps);
  else if (prec == PREC_F32)  // W1 natural, W2 in the pack_mlp2_perm order, each as hi | lo planes
    hipLaunchKernelGGL(mlp_x3_kernel, dim3((unsigned)((M + 63) / 64)), dim3(256), 0, st, X, (const bf16*)W1,
                       (const bf16*)W2, (int)M, Fh, eps);
  else
    hipLaunchKernelGGL(mlp_fused_kernel<0>, grid, dim3(256), MlpLds<0>::BYTES, st, X, W1, W2, (int)M, Fh, eps);
  return hipGetLastError();
}

}  // namespace mmpfn
