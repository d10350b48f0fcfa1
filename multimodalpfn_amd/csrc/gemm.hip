// MFMA GEMM  C[M,N] = A[M,K] . W[N,K]^T  with fused epilogues, for gfx950.
//
// Used for every dense contraction of the PerFeatureTransformer forward:
//   QKV projections (transformer.py / multi_head_attention.py:423-445),
//   attention output projection + residual + LayerNorm (layer.py:437-455),
//   MLP up (+GELU) and down (+residual+LN) (mlp.py:93-104),
//   MGM / CAP / MoE projection heads (transformer.py:33-128).
//
// Tile: 64 (M) x 192 (N) per 256-thread block, 4 waves as 2 (M) x 2 (N), each wave
// 32 x 96 = 2 x 6 MFMA tiles of 16 x 16.  K is staged through LDS in 128-byte row
// slices (64 bf16 or 32 f32), with the next slice's global loads in flight while
// the current one is consumed (register staging, issue-early / write-late).
//   bf16 path : v_mfma_f32_16x16x32_bf16, fp32 accumulate
//   x3   path : parity mode (PREC_F32): A (fp32) split into bf16 hi + lo planes as it is staged,
//               W pre-split on the host; acc += Ah.Wh + Ah.Wl + Al.Wh on v_mfma_f32_16x16x32_bf16
//   f32  path : v_mfma_f32_16x16x4_f32 (exact fp32 fma chain; PREC_F32_MFMA)
// A may be stored fp32 while the bf16 path computes: it is converted when written
// to LDS, so the fp32 residual stream is never materialised in bf16 in HBM.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int BM = 64;
constexpr int BN = 192;
constexpr int ROWB = 160;  // LDS bytes per staged row: 128 data + 32 pad (32 mod 64: conflict-free ds_read_b128)
constexpr int LDS_STAGE = (BM + BN) * ROWB;
constexpr int LDS_STAGE_X3 = 2 * (BM + BN) * ROWB;  // hi and lo planes of A and W
constexpr int LN_STRIDE = 196;  // floats per row of the LayerNorm epilogue buffer
constexpr int LDS_LN = BM * LN_STRIDE * 4;
constexpr int A_CHUNKS = BM * 8 / 256;  // 16-byte LDS chunks per thread
constexpr int W_CHUNKS = BN * 8 / 256;

template <bool BF16, bool AF32>
struct Stage {
  // raw staged A data per chunk: f32 source feeding bf16 compute needs 32 bytes
  static constexpr int AWORDS = (BF16 && AF32) ? 2 : 1;
};

// hi = bf16(x), lo = bf16(x - hi): x = hi + lo to 2^-17 relative (parity mode)
__device__ __forceinline__ void split8(const f32x4& f0, const f32x4& f1, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    hi[i] = (bf16)f0[i], hi[4 + i] = (bf16)f1[i];
    lo[i] = (bf16)(f0[i] - (float)hi[i]), lo[4 + i] = (bf16)(f1[i] - (float)hi[4 + i]);
  }
}

// MODE 0: fp32-input MFMA, 1: bf16, 2: x3 (split bf16, A fp32)
template <int MODE, bool AF32, bool OF32, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs p) {
  constexpr bool BF16 = MODE != 0;
  constexpr bool X3 = MODE == 2;
  static_assert(!X3 || AF32, "x3 splits an fp32 A");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* As = smem;
  unsigned char* Ws = smem + (X3 ? 2 : 1) * BM * ROWB;
  unsigned char* Asl = smem + BM * ROWB;          // x3: A lo plane
  unsigned char* Wsl = Ws + BN * ROWB;            // x3: W lo plane
  typedef typename std::conditional<OF32, float, bf16>::type TO;
  constexpr int EB = BF16 ? 2 : 4;       // compute element bytes
  constexpr int BK = 128 / EB;           // K per staged slice
  constexpr int AW = Stage<BF16, AF32>::AWORDS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int z = blockIdx.z;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int M = p.M, K = p.K;

  const unsigned char* Abase = (const unsigned char*)p.A + (int64_t)z * p.a_zstride * (AF32 ? 4 : 2);
  const unsigned char* Wbase = (const unsigned char*)p.W + (int64_t)z * p.w_zstride * EB;

  // per-thread A row pointers (row -> memory row remap), computed once
  const unsigned char* arow[A_CHUNKS];
  int ach[A_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    const int c = tid + 256 * i;
    const int r = c >> 3;
    ach[i] = c & 7;
    const int64_t m = m0 + r;
    if (m < M) {
      const int64_t mr = (m / p.a_rdiv) * p.a_rmul + (m % p.a_rdiv) * p.a_rmul2 + p.a_roff;
      arow[i] = Abase + mr * p.lda * (AF32 ? 4 : 2);
    } else {
      arow[i] = nullptr;
    }
  }

  u32x4 ra[A_CHUNKS][AW];
  u32x4 rw[W_CHUNKS];
  u32x4 rwl[X3 ? W_CHUNKS : 1];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      if (arow[i]) {
        if (BF16 && AF32) {
          const float* src = (const float*)arow[i] + k0 + ach[i] * 8;
          ra[i][0] = *(const u32x4*)src;
          ra[i][AW - 1] = *(const u32x4*)(src + 4);
        } else {
          ra[i][0] = *(const u32x4*)(arow[i] + ((int64_t)k0 + ach[i] * (16 / EB)) * EB);
        }
      } else {
#pragma unroll
        for (int w = 0; w < AW; ++w) ra[i][w] = u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < W_CHUNKS; ++i) {
      const int c = tid + 256 * i;
      const int r = c >> 3, ch = c & 7;
      rw[i] = *(const u32x4*)(Wbase + ((int64_t)(n0 + r) * K + k0 + ch * (16 / EB)) * EB);
      if constexpr (X3) rwl[i] = *(const u32x4*)(Wbase + (p.w_lo_off + (int64_t)(n0 + r) * K + k0 + ch * 8) * 2);
    }
  };

  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int c = tid + 256 * i;
      const int r = c >> 3;
      u32x4 v;
      if constexpr (X3) {
        bf16x8 hi, lo;
        split8(__builtin_bit_cast(f32x4, ra[i][0]), __builtin_bit_cast(f32x4, ra[i][AW - 1]), hi, lo);
        v = __builtin_bit_cast(u32x4, hi);
        *(u32x4*)(Asl + r * ROWB + ach[i] * 16) = __builtin_bit_cast(u32x4, lo);
      } else if (BF16 && AF32) {
        const f32x4 f0 = __builtin_bit_cast(f32x4, ra[i][0]);
        const f32x4 f1 = __builtin_bit_cast(f32x4, ra[i][AW - 1]);
        bf16x8 b;
        b[0] = (bf16)f0[0]; b[1] = (bf16)f0[1]; b[2] = (bf16)f0[2]; b[3] = (bf16)f0[3];
        b[4] = (bf16)f1[0]; b[5] = (bf16)f1[1]; b[6] = (bf16)f1[2]; b[7] = (bf16)f1[3];
        v = __builtin_bit_cast(u32x4, b);
      } else {
        v = ra[i][0];
      }
      *(u32x4*)(As + r * ROWB + ach[i] * 16) = v;
    }
#pragma unroll
    for (int i = 0; i < W_CHUNKS; ++i) {
      const int c = tid + 256 * i;
      *(u32x4*)(Ws + (c >> 3) * ROWB + (c & 7) * 16) = rw[i];
      if constexpr (X3) *(u32x4*)(Wsl + (c >> 3) * ROWB + (c & 7) * 16) = rwl[i];
    }
  };

  f32x4 acc[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  load_tile(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
    const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if constexpr (X3) {
        bf16x8 af[2], afl[2], bw[6], bwl[6];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          af[mt] = *(const bf16x8*)(As + (wm * 32 + mt * 16 + fr) * ROWB + ks * 64 + fg * 16);
          afl[mt] = *(const bf16x8*)(Asl + (wm * 32 + mt * 16 + fr) * ROWB + ks * 64 + fg * 16);
        }
#pragma unroll
        for (int nt = 0; nt < 6; ++nt) {
          bw[nt] = *(const bf16x8*)(Ws + (wn * 96 + nt * 16 + fr) * ROWB + ks * 64 + fg * 16);
          bwl[nt] = *(const bf16x8*)(Wsl + (wn * 96 + nt * 16 + fr) * ROWB + ks * 64 + fg * 16);
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
        for (int mt = 0; mt < 2; ++mt)
          af[mt] = *(const bf16x8*)(As + (wm * 32 + mt * 16 + fr) * ROWB + ks * 64 + fg * 16);
#pragma unroll
        for (int nt = 0; nt < 6; ++nt)
          bw[nt] = *(const bf16x8*)(Ws + (wn * 96 + nt * 16 + fr) * ROWB + ks * 64 + fg * 16);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 6; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[nt], acc[mt][nt], 0, 0, 0);
      } else {
        f32x4 af[2], bw[6];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          af[mt] = *(const f32x4*)(As + (wm * 32 + mt * 16 + fr) * ROWB + ks * 64 + fg * 16);
#pragma unroll
        for (int nt = 0; nt < 6; ++nt)
          bw[nt] = *(const f32x4*)(Ws + (wn * 96 + nt * 16 + fr) * ROWB + ks * 64 + fg * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < 6; ++nt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt][e], bw[nt][e], acc[mt][nt], 0, 0, 0);
      }
    }
  }

  // ---------------------------------------------------------------- epilogues
  const int fr = lane & 15, fg = lane >> 4;
  const float* bias = p.bias ? p.bias + (int64_t)z * p.b_zstride : nullptr;

  if constexpr (EPI == EPI_RES_LN) {
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
          float v = acc[mt][nt][r] + (bias ? bias[cl] : 0.f);
          const float xr = p.X[min(m, (int64_t)M - 1) * 192 + cl];
          v += (m < M) ? xr : 0.f;
          Es[rl * LN_STRIDE + cl] = v;
        }
    __syncthreads();
    const int row = tid >> 2, part = tid & 3;
    const int64_t m = m0 + row;
    const float* er = Es + row * LN_STRIDE + part * 48;
    float s = 0.f;
#pragma unroll 8
    for (int i = 0; i < 48; ++i) s += er[i];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    const float mean = s * (1.0f / 192.0f);
    float q = 0.f;
#pragma unroll 8
    for (int i = 0; i < 48; ++i) {
      const float dlt = er[i] - mean;
      q += dlt * dlt;
    }
    q += __shfl_xor(q, 1, 64);
    q += __shfl_xor(q, 2, 64);
    const float inv = 1.0f / sqrtf(q * (1.0f / 192.0f) + p.ln_eps);
    if (m < M) {
      float* xo = p.X + m * 192 + part * 48;
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
    return;
  } else {
    // Stage the finished tile (bias + activation / GLU applied) in LDS in the output
    // dtype, then write 16-byte units ordered so that consecutive lanes hit
    // consecutive addresses of the destination layout (4 KB runs per head for the
    // attention scatter layouts instead of 2-byte / 32-byte fragments).
    constexpr int OB = sizeof(TO);
    constexpr int UE = 16 / OB;                  // elements per 16-byte unit
    constexpr bool GLU = EPI == EPI_GLU;
    constexpr int TCOLS = GLU ? BN / 2 : BN;     // staged columns
    constexpr int LDC = TCOLS + UE;              // padded LDS row (elements)
    TO* Ct = (TO*)smem;
    __syncthreads();
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 32 + mt * 16 + fg * 4 + r;
        if constexpr (GLU) {
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const int na = n0 + wn * 96 + q * 32 + fr;
            const float a = acc[mt][2 * q][r] + (bias ? bias[na] : 0.f);
            const float b = acc[mt][2 * q + 1][r] + (bias ? bias[na + 16] : 0.f);
            Ct[rl * LDC + wn * 48 + q * 16 + fr] = from_f32<TO>(a * sigmoidf_(b));
          }
        } else {
#pragma unroll
          for (int nt = 0; nt < 6; ++nt) {
            const int cl = wn * 96 + nt * 16 + fr;
            float v = acc[mt][nt][r] + (bias ? bias[n0 + cl] : 0.f);
            if (p.act == ACT_GELU) v = gelu_erf(v);
            Ct[rl * LDC + cl] = from_f32<TO>(v);
          }
        }
      }
    __syncthreads();
    const int E = p.H * 32;
    const bool vt_block = (EPI == EPI_ITEM_QKV) && (n0 / 192 == 2);
    if (!vt_block) {
      constexpr int CPB = 32 / UE;  // units per 32-column block per row
      constexpr int UNITS = BM * TCOLS / UE;
      for (int u = tid; u < UNITS; u += 256) {
        const int cb = u / (BM * CPB), rem = u % (BM * CPB);
        const int rl = rem / CPB, cl = cb * 32 + (rem % CPB) * UE;
        const int64_t m = m0 + rl;
        if (m >= M) continue;
        const u32x4 val = *(const u32x4*)(Ct + rl * LDC + cl);
        TO* dst;
        if constexpr (EPI == EPI_STORE) {
          dst = (TO*)p.C + (int64_t)z * p.c_zstride + m * p.ldc + n0 + cl;
        } else if constexpr (EPI == EPI_GLU) {
          dst = (TO*)p.C + (int64_t)z * p.c_zstride + m * p.ldc + n0 / 2 + cl;
        } else if constexpr (EPI == EPI_REMAP) {
          const int64_t dr = (m / p.rdiv2) * p.rmul2 + (int64_t)z * p.zmul + (m % p.rdiv2);
          dst = (TO*)p.C + dr * p.ldc + n0 + cl;
        } else {  // EPI_ITEM_QKV, Q or K block
          const int n = n0 + cl;
          const int j = n / E, h = (n % E) >> 5, d = n & 31;
          const int64_t t = m / p.a_rdiv, s = p.a_roff + m % p.a_rdiv;
          const int64_t th = t * p.H + h;
          dst = j == 0 ? (TO*)p.q + (th * p.S + s) * 32 + d : (TO*)p.k + (th * p.Npad + s) * 32 + d;
        }
        *(u32x4*)dst = val;
      }
    } else {
      // V^T [T][H][32][Npad]: units of UE consecutive rows s of one (h, d) column
      constexpr int RPC = BM / UE;  // units per column
      for (int u = tid; u < BN * RPC; u += 256) {
        const int cl = u / RPC, rc = u % RPC;
        const int n = n0 + cl;
        const int h = (n % E) >> 5, d = n & 31;
        const int64_t ma = m0 + rc * UE;
        if (ma >= M) continue;
        const int64_t mb = ma + UE - 1;
        const int64_t ta = ma / p.a_rdiv, sa = p.a_roff + ma % p.a_rdiv;
        if (mb < M && mb / p.a_rdiv == ta && (sa % UE) == 0) {
          TO* dst = (TO*)p.v + ((ta * p.H + h) * 32 + d) * p.Npad + sa;
          if constexpr (OB == 2) {
            bf16x8 w;
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = Ct[(rc * UE + i) * LDC + cl];
            *(bf16x8*)dst = w;
          } else {
            f32x4 w;
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] = Ct[(rc * UE + i) * LDC + cl];
            *(f32x4*)dst = w;
          }
        } else {
          for (int i = 0; i < UE; ++i) {
            const int64_t m = ma + i;
            if (m >= M) break;
            const int64_t t = m / p.a_rdiv, s = p.a_roff + m % p.a_rdiv;
            ((TO*)p.v)[((t * p.H + h) * 32 + d) * p.Npad + s] = Ct[(rc * UE + i) * LDC + cl];
          }
        }
      }
    }
  }
}

template <int MODE, bool AF32, bool OF32, int EPI>
hipError_t launch_t(const GemmArgs& a, int groups, hipStream_t st) {
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, groups);
  constexpr int OUTB = (EPI == EPI_RES_LN || OF32) ? 4 : 2;
  constexpr int STAGED = EPI == EPI_RES_LN ? LDS_LN : BM * (BN + 16 / OUTB) * OUTB;
  constexpr int STAGE = MODE == 2 ? LDS_STAGE_X3 : LDS_STAGE;
  const int lds = STAGED > STAGE ? STAGED : STAGE;
  if (lds > 65536) {  // x3: 80 KB of hi / lo planes
    static std::atomic<uint64_t> opted{0};
    const hipError_t e = lds_optin(opted, (const void*)gemm_kernel<MODE, AF32, OF32, EPI>, lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((gemm_kernel<MODE, AF32, OF32, EPI>), grid, dim3(256), lds, st, a);
  return hipGetLastError();
}

template <int MODE, bool AF32, bool OF32>
hipError_t launch_e(const GemmArgs& a, int epi, int groups, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_t<MODE, AF32, OF32, EPI_STORE>(a, groups, st);
    case EPI_ITEM_QKV: return launch_t<MODE, AF32, OF32, EPI_ITEM_QKV>(a, groups, st);
    case EPI_RES_LN: return launch_t<MODE, AF32, true, EPI_RES_LN>(a, groups, st);
    case EPI_GLU: return launch_t<MODE, AF32, OF32, EPI_GLU>(a, groups, st);
    case EPI_REMAP: return launch_t<MODE, AF32, OF32, EPI_REMAP>(a, groups, st);
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------- large-tile GLU GEMM (bf16)
// The MGM head bank (transformer.py:33-60): C[M][N/2] = GLU(A[M][K] . W[N][K]^T + bias), N = heads x
// 768 (~49 k), K = 768, M = rows: one 174-GFLOP GEMM per predict.  The 64 x 192 tile above
// re-reads W once per 64 rows (2.7 GB of L2 traffic at PAD-UFES size); this tile is 256 rows x
// 256 W rows per 512-thread block (8 waves as 2 x 4, each 128 x 64 = 8 x 4 MFMA-16 tiles), and
// blocks that share a W tile are scheduled on one XCD back to back so the tile is fetched from
// HBM about once.  K moves in 32-wide slices through a 4-stage LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4: no staging registers, no LDS write pass after the MFMAs): slice
// kt+1..kt+3 are in flight while slice kt computes; one barrier per slice.  LDS images are unpadded
// 64-B rows with 16-B chunk c of row r at slot c ^ ((r >> 1) & 3) (conflict-free ds_read_b128 for
// the 16x16x32 operands); the DMA writes lane-linear, so each lane fetches the chunk that belongs
// at its slot.  The DMA is inline asm so the compiler adds no vmcnt(0) before the LDS reads of
// the other stages; the kernel waits for its own slices explicitly.
// GLU pairs: W rows interleaved in 16-row blocks [a | b] (capi.cpp), so tiles 2q / 2q+1 of a
// wave are the a / b halves of the same 16 output columns.
constexpr int GB_M = 256, GB_N = 256, GB_K = 32;
constexpr int GB_ROW = GB_K * 2;                    // 64-B LDS rows
constexpr int GB_STAGE = (GB_M + GB_N) * GB_ROW;    // 32 KB
#ifndef GB_STAGES
#define GB_STAGES 4
#endif
constexpr int GB_NST = GB_STAGES;                   // ring stages (128 KB)
constexpr int GB_OST = GB_N / 2 + 8;                // output staging row stride (bf16)
constexpr int GB_DMA = (GB_M + GB_N) * (GB_ROW / 16) / 512;  // 16-B DMA pieces per thread and slice (4)
constexpr int GB_MT = GB_M / 32;                    // 16-row MFMA tiles per wave (8)

__device__ __forceinline__ int gb_slot(int r, int c) { return c ^ ((r >> 1) & 3); }

// "m0" in the clobber list: clang keeps m0 reserved and ignores the entry (-Winline-asm; the ISA is identical with
// and without it), and every m0 use the compiler emits itself is preceded by its own write -- test_codegen checks
// that no m0 read other than these DMA issues exists in the kernels
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void gb_dma16(const void* src, unsigned lds_base) {
  // m0 = the wave's LDS destination; lane i's 16 B land at m0 + 16 i
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_base) : "memory", "m0");
}
#pragma clang diagnostic pop

// F16: the same kernel on fp16 operands (the fp16 mode's mixer: the reference's autocast runs these Linears in fp16)
template <bool F16>
__global__ __launch_bounds__(512, 1) void gemm_glu_big_kernel(const typename Op16<F16>::t* __restrict__ A,
                                                              const typename Op16<F16>::t* __restrict__ W,
                                                              const float* __restrict__ bias,
                                                              typename Op16<F16>::t* __restrict__ C, int M, int N, int K,
                                                              int mtiles) {
  typedef typename Op16<F16>::t T;
  typedef typename Op16<F16>::x8 X8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  // XCD-aware tile order: XCD x (= block % 8) runs a contiguous range of (W tile, M tile) tasks,
  // W-tile-major, so the M tiles of one W tile run back to back on one L2
  int mt, nt;
  {
    const int nb = gridDim.x;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int per = nb >> 3, extra = nb & 7;
    const int t = xcd * per + min(xcd, extra) + slot;
    nt = t / mtiles, mt = t - nt * mtiles;
  }
  const int m0 = mt * GB_M, n0 = nt * GB_N;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)smem;

  // DMA piece j of this wave: LDS chunk q = (wave * GB_DMA + j) * 64 + lane of the stage image
  // (rows 0-255 = A, 256-511 = W); row r = q / 4 holds global chunk c with gb_slot(r, c) = q % 4
  const T* src[GB_DMA];
#pragma unroll
  for (int j = 0; j < GB_DMA; ++j) {
    const int q = (wave * GB_DMA + j) * 64 + lane, r = q >> 2, c = gb_slot(r, q & 3);
    src[j] = r < GB_M ? A + (int64_t)min(m0 + r, M - 1) * K + c * 8 : W + (int64_t)(n0 + r - GB_M) * K + c * 8;
  }
  auto dma = [&](int kt) {
    const unsigned base = lds0 + (kt % GB_NST) * GB_STAGE + wave * GB_DMA * 1024;
#pragma unroll
    for (int j = 0; j < GB_DMA; ++j)
      gb_dma16(src[j] + kt * GB_K, __builtin_amdgcn_readfirstlane(base + j * 1024));
  };
  f32x4 acc[GB_MT][4];
#pragma unroll
  for (int a = 0; a < GB_MT; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GB_K;
#pragma unroll
  for (int i = 0; i < GB_NST - 1; ++i)
    if (i < nk) dma(i);
  for (int kt = 0; kt < nk; ++kt) {
    // this thread's pieces of slice kt have landed (up to two later slices may still fly)
    const int ahead = min(nk - 1 - kt, GB_NST - 2);
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GB_DMA) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GB_DMA) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GB_DMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // stage (kt+3) % 4 was last read in slice kt-1, before the barrier above
    if (kt + GB_NST - 1 < nk) dma(kt + GB_NST - 1);
    const unsigned char* As = smem + (kt % GB_NST) * GB_STAGE;
    const unsigned char* Ws = As + GB_M * GB_ROW;
    X8 af[GB_MT], bw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rb = wn * 64 + i * 16 + fr;
      bw[i] = *(const X8*)(Ws + rb * GB_ROW + 16 * gb_slot(rb, fg));
    }
#pragma unroll
    for (int i = 0; i < GB_MT; ++i) {
      const int ra = wm * (GB_M / 2) + i * 16 + fr;
      af[i] = *(const X8*)(As + ra * GB_ROW + 16 * gb_slot(ra, fg));
    }
#pragma unroll
    for (int a = 0; a < GB_MT; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = mfma16x(af[a], bw[b], acc[a][b]);
  }
  __syncthreads();  // every wave is done with the ring before it is reused for the output tile
  // GLU epilogue: C tile lane layout (row 16a + 4fg + r, column fr of tile b); a = tile 2q, b = 2q+1
  T* Ct = (T*)smem;  // [GB_M][GB_OST]
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int na = n0 + wn * 64 + q * 32 + fr;
    const float ba = bias[na], bb = bias[na + 16];
#pragma unroll
    for (int a = 0; a < GB_MT; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float va = acc[a][2 * q][r] + ba, vb = acc[a][2 * q + 1][r] + bb;
        Ct[(wm * (GB_M / 2) + a * 16 + fg * 4 + r) * GB_OST + wn * 32 + q * 16 + fr] = (T)(va * sigmoidf_(vb));
      }
  }
  __syncthreads();
  const int ldc = N / 2, c0 = n0 / 2;
#pragma unroll
  for (int i = 0; i < GB_M * 16 / 512; ++i) {  // GB_M rows x 16 chunks of 16 B
    const int u = tid + 512 * i, r = u >> 4, ch = u & 15;
    if (m0 + r < M) *(u32x4*)(C + (int64_t)(m0 + r) * ldc + c0 + ch * 8) = *(const u32x4*)(Ct + r * GB_OST + ch * 8);
  }
}


// ---------------------------------------------------------------- large-tile MGM down-projection (bf16)
// Per head z (transformer.py:52-55: Linear(D/2 -> E) after the GLU): C[(s, z, mod)][E] = A[r][z D/2 + k] .
// W2[z][E][k]^T + b2[z], the rows remapped head-major into the [S][mgm n_mod][E] token tensor.  The 64 x 192
// tile of gemm_kernel re-reads its W (one head's 192 x 384) per 64 rows and runs at the L2 -> LDS fill
// rate (75 us at PAD-UFES size); here 320 rows x the head's 192 outputs per 512-thread block (8 waves as
// 2 x 4, each 160 x 48 = 10 x 3 MFMA-16 tiles), the same four-stage LDS-DMA ring and swizzled 64-B rows
// as the GLU kernel (320 + 192 = 512 rows: four 16-B pieces per thread and slice), the M tiles of one
// head back to back on one XCD.
constexpr int GR_M = 320, GR_N = 192;
static_assert(GR_M + GR_N == GB_M + GB_N, "four DMA pieces per thread and K slice, as the GLU kernel");
constexpr int GR_MT = GR_M / 32;  // 16-row tiles per wave (10)
constexpr int GR_NT = GR_N / 64;  // 16-column tiles per wave (3)

// TO: fp32 tokens, or 16-bit (the MGM+CAP chain's intermediate, read by the CAP K|V projection); F16: fp16 operands
template <typename TO, bool F16>
__global__ __launch_bounds__(512, 1) void gemm_remap_big_kernel(const typename Op16<F16>::t* __restrict__ A, int64_t lda,
                                                                const typename Op16<F16>::t* __restrict__ W,
                                                                const float* __restrict__ bias, TO* __restrict__ C,
                                                                int M, int K, int mtiles, int n_mod, int Mtok) {
  typedef typename Op16<F16>::t T;
  typedef typename Op16<F16>::x8 X8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  int mt, z;
  {
    const int nb = gridDim.x;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int per = nb >> 3, extra = nb & 7;
    const int t = xcd * per + min(xcd, extra) + slot;
    z = t / mtiles, mt = t - z * mtiles;
  }
  const int m0 = mt * GR_M;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
  const T* src[GB_DMA];
#pragma unroll
  for (int j = 0; j < GB_DMA; ++j) {
    const int q = (wave * GB_DMA + j) * 64 + lane, r = q >> 2, c = gb_slot(r, q & 3);
    src[j] = r < GR_M ? A + (int64_t)min(m0 + r, M - 1) * lda + (int64_t)z * K + c * 8
                      : W + ((int64_t)z * GR_N + (r - GR_M)) * K + c * 8;
  }
  auto dma = [&](int kt) {
    const unsigned base = lds0 + (kt % GB_NST) * GB_STAGE + wave * GB_DMA * 1024;
#pragma unroll
    for (int j = 0; j < GB_DMA; ++j)
      gb_dma16(src[j] + kt * GB_K, __builtin_amdgcn_readfirstlane(base + j * 1024));
  };
  f32x4 acc[GR_MT][GR_NT];
#pragma unroll
  for (int a = 0; a < GR_MT; ++a)
#pragma unroll
    for (int b = 0; b < GR_NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / GB_K;
#pragma unroll
  for (int i = 0; i < GB_NST - 1; ++i)
    if (i < nk) dma(i);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, GB_NST - 2);
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GB_DMA) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GB_DMA) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GB_DMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + GB_NST - 1 < nk) dma(kt + GB_NST - 1);
    const unsigned char* As = smem + (kt % GB_NST) * GB_STAGE;
    const unsigned char* Ws = As + GR_M * GB_ROW;
    X8 af[GR_MT], bw[GR_NT];
#pragma unroll
    for (int i = 0; i < GR_NT; ++i) {
      const int rb = wn * (GR_N / 4) + i * 16 + fr;
      bw[i] = *(const X8*)(Ws + rb * GB_ROW + 16 * gb_slot(rb, fg));
    }
#pragma unroll
    for (int i = 0; i < GR_MT; ++i) {
      const int ra = wm * (GR_M / 2) + i * 16 + fr;
      af[i] = *(const X8*)(As + ra * GB_ROW + 16 * gb_slot(ra, fg));
    }
#pragma unroll
    for (int a = 0; a < GR_MT; ++a)
#pragma unroll
      for (int b = 0; b < GR_NT; ++b) acc[a][b] = mfma16x(af[a], bw[b], acc[a][b]);
  }
  // C tile lane layout: row 16a + 4fg + r, column 16b + fr of the wave's 160 x 48 block; + b2[z], row remap
#pragma unroll
  for (int b = 0; b < GR_NT; ++b) {
    const int n = wn * (GR_N / 4) + b * 16 + fr;
    const float bv = bias[z * GR_N + n];
#pragma unroll
    for (int a = 0; a < GR_MT; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (GR_M / 2) + a * 16 + fg * 4 + r;
        if (m < M) {
          const int64_t dr = (int64_t)(m / n_mod) * Mtok + (int64_t)z * n_mod + m % n_mod;
          C[dr * GR_N + n] = (TO)(acc[a][b][r] + bv);
        }
      }
  }
}

}  // namespace

hipError_t launch_gemm(const GemmArgs& a, int prec, int epi, bool a_f32, bool out_f32, int groups,
                       hipStream_t st) {
  if (a.M <= 0) return hipSuccess;
  if (a.N % BN != 0) return hipErrorInvalidValue;
  if (prec == PREC_F32_MFMA) {
    if (!a_f32 || !out_f32) return hipErrorInvalidValue;
    if (a.K % 32 != 0) return hipErrorInvalidValue;
    return launch_e<0, true, true>(a, epi, groups, st);
  }
  if (a.K % 64 != 0) return hipErrorInvalidValue;
  if (prec == PREC_F32) {  // x3: fp32 A split while staged, W given as hi | lo planes (w_lo_off)
    if (!a_f32 || !out_f32 || a.w_lo_off <= 0) return hipErrorInvalidValue;
    return launch_e<2, true, true>(a, epi, groups, st);
  }
  if (a_f32) {
    return out_f32 ? launch_e<1, true, true>(a, epi, groups, st) : launch_e<1, true, false>(a, epi, groups, st);
  }
  return out_f32 ? launch_e<1, false, true>(a, epi, groups, st) : launch_e<1, false, false>(a, epi, groups, st);
}

hipError_t launch_gemm_remap_big(const void* A, int64_t lda, const void* W, const float* bias, void* C, bool c_bf16,
                                 int M, int K, int nheads, int n_mod, int E, hipStream_t st, bool f16) {
  if (M <= 0) return hipSuccess;
  if (E != GR_N || K % GB_K != 0 || K <= 0 || nheads <= 0 || n_mod <= 0) return hipErrorInvalidValue;
  const int mtiles = (M + GR_M - 1) / GR_M;
  const int64_t nb = (int64_t)mtiles * nheads;
  const int lds = GB_NST * GB_STAGE;
  if (f16) {  // fp16 operands; a 16-bit token output is fp16 too
    if (c_bf16)
      hipLaunchKernelGGL((gemm_remap_big_kernel<_Float16, true>), dim3((unsigned)nb), dim3(512), lds, st,
                         (const _Float16*)A, lda, (const _Float16*)W, bias, (_Float16*)C, M, K, mtiles, n_mod, nheads * n_mod);
    else
      hipLaunchKernelGGL((gemm_remap_big_kernel<float, true>), dim3((unsigned)nb), dim3(512), lds, st,
                         (const _Float16*)A, lda, (const _Float16*)W, bias, (float*)C, M, K, mtiles, n_mod, nheads * n_mod);
  } else if (c_bf16) {
    hipLaunchKernelGGL((gemm_remap_big_kernel<bf16, false>), dim3((unsigned)nb), dim3(512), lds, st, (const bf16*)A, lda,
                       (const bf16*)W, bias, (bf16*)C, M, K, mtiles, n_mod, nheads * n_mod);
  } else {
    hipLaunchKernelGGL((gemm_remap_big_kernel<float, false>), dim3((unsigned)nb), dim3(512), lds, st, (const bf16*)A,
                       lda, (const bf16*)W, bias, (float*)C, M, K, mtiles, n_mod, nheads * n_mod);
  }
  return hipGetLastError();
}

hipError_t launch_gemm_glu_big(const void* A, const void* W, const float* bias, void* C, int M, int N, int K,
                               hipStream_t st, bool f16) {
  if (M <= 0) return hipSuccess;
  if (N % GB_N != 0 || K % GB_K != 0 || K <= 0) return hipErrorInvalidValue;
  const int mtiles = (M + GB_M - 1) / GB_M;
  const int64_t nb = (int64_t)mtiles * (N / GB_N);
  const int lds = GB_NST * GB_STAGE;  // 144 KB
  static_assert(GB_M * GB_OST * 2 <= GB_NST * GB_STAGE, "output staging fits the ring");
  if (f16)
    hipLaunchKernelGGL((gemm_glu_big_kernel<true>), dim3((unsigned)nb), dim3(512), lds, st, (const _Float16*)A,
                       (const _Float16*)W, bias, (_Float16*)C, M, N, K, mtiles);
  else
    hipLaunchKernelGGL((gemm_glu_big_kernel<false>), dim3((unsigned)nb), dim3(512), lds, st, (const bf16*)A,
                       (const bf16*)W, bias, (bf16*)C, M, N, K, mtiles);
  return hipGetLastError();
}

}  // namespace mmpfn
