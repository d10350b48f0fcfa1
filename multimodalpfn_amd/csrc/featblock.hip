// Fused attention-between-features sublayer for gfx950 (bf16 performance mode):
//   X <- LayerNorm(X + MHA_features(X))        (layer.py:332-339,437-455; multi_head_attention.py:547-736)
//
// Attention between features is independent per table row: a row's T tokens attend
// to each other.  One 256-thread block owns R consecutive rows (R*T <= 112 tokens),
// so the whole sublayer runs out of LDS:
//   phase 0  the R*T token rows of X (fp32, [T][S][E]) -> bf16 A tile in LDS
//   per head h (6):
//     QKV_h^T = W_h . A^T          96 x R*T, v_mfma_f32_16x16x32_bf16; W_h staged once
//                                  per block in LDS (the next head's slice is fetched
//                                  into registers while this head's attention runs)
//     per row (one wave): S^T = K Q^T (keys x queries), softmax over keys in
//                         registers, O^T = V^T P^T with P^T taken straight from the
//                         S^T accumulators (key order permuted identically in V^T)
//     O_h -> LDS O tile (bf16)
//   out-projection Y^T = Wout . O^T (all heads; Wout staged over the dead tiles),
//   residual + LayerNorm per token in registers, X written back in place (a block
//   touches only its own rows).
// HBM traffic: X read + X written once (2 x 63.5 MB at the PAD-UFES shape) instead of
// the QKV / O round trips of the unfused three-kernel form.  LDS row strides are
// 32 mod 64 bytes so the 16-lane groups of ds_read_b128 hit 16 distinct 4-bank
// sets (MI355X_MICROARCH.md, LDS table).
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace mmpfn {

namespace {

constexpr int FE = 192;           // model width
constexpr int FH = 6;             // heads
constexpr int FD = 32;            // head dim
constexpr int AST = FE + 16;      // A / O / W LDS row stride (bf16): 416 B
constexpr int QST = 3 * FD + 16;  // per-head QKV LDS row stride: 224 B
constexpr int QTAIL = 16;         // zero rows after the QKV tile (key tiles past the last row)
constexpr int MAXTOK = 112;       // tokens per block (7 tiles of 16)
constexpr int WROWS = 3 * FD;     // rows of one head's QKV weight slice
constexpr int WPIECES = WROWS * (FE / 8) / 256;  // 16-B pieces per thread (9)
constexpr int OPIECES = FE * (FE / 8) / 256;     // Wout pieces per thread (18)

struct FbArgs {
  float* X;
  const bf16* wqkv;  // [3*H*D][E]   rows (j*H + h)*D + d, j = q/k/v
  const bf16* wout;  // [E][H*D]     (out feature, h*D + d)
  int S, T, R, Mp;
  float eps, qscale;
};

#ifdef MMPFN_STAMPS  // phase timestamps of one block (diagnostics build only: make dbg)
__device__ unsigned long long g_fb_stamps[32];
#define FB_STAMP(k) \
  if (blockIdx.x == gridDim.x / 2 && threadIdx.x == 0) g_fb_stamps[(k)] = __builtin_amdgcn_s_memtime()
#else
#define FB_STAMP(k) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// piece i of head h's weight slice: LDS row r = i / 24 (q 0-31, k 32-63, v 64-95), 16-B column i % 24
__device__ __forceinline__ const bf16* wslice_src(const bf16* w, int h, int i) {
  const int r = i / (FE / 8);
  return w + (int64_t)((r >> 5) * (FH * FD) + h * FD + (r & 31)) * FE + (i % (FE / 8)) * 8;
}

__global__ __launch_bounds__(256, 1) void feat_block_kernel(const FbArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Mp = p.Mp, T = p.T;
  bf16* Os = (bf16*)smem;            // [Mp][AST]
  bf16* As = Os + Mp * AST;          // [Mp][AST]
  bf16* Qs = As + Mp * AST;          // [Mp + QTAIL][QST]
  bf16* Wh = Qs + (Mp + QTAIL) * QST;  // [96][AST]
  bf16* Wo = As;                     // after the heads: Wout [E][AST] over A / QKV / W_h
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int s0 = blockIdx.x * p.R;
  const int R = min(p.R, p.S - s0);
  const int RT = R * T;
  const int ntt = Mp >> 4;  // token tiles (<= 7)
  const int qrows = Mp + QTAIL;
  const int64_t SE = (int64_t)p.S * FE;

  u32x4 wpf[WPIECES];
  auto wfetch = [&](int h) {
#pragma unroll
    for (int j = 0; j < WPIECES; ++j) wpf[j] = *(const u32x4*)wslice_src(p.wqkv, h, tid + 256 * j);
  };
  auto wstash = [&]() {
#pragma unroll
    for (int j = 0; j < WPIECES; ++j) {
      const int i = tid + 256 * j;
      *(u32x4*)(Wh + (i / (FE / 8)) * AST + (i % (FE / 8)) * 8) = wpf[j];
    }
  };

  FB_STAMP(0);
  // ---- phase 0: token rows -> bf16 A (pad rows zero), head-0 weights, zero the QKV tail.
  // All of a thread's loads are issued before the first use.
  wfetch(0);
  constexpr int P0 = MAXTOK * (FE / 4) / 256;  // 21 16-B pieces per thread at most
  {
    f32x4 v[P0];
#pragma unroll
    for (int j = 0; j < P0; ++j) {
      const int i = tid + 256 * j;
      const int m = i / (FE / 4), c4 = i - m * (FE / 4);
      v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < RT) {
        const int r = m / T, t = m - r * T;
        v[j] = *(const f32x4*)(p.X + t * SE + (int64_t)(s0 + r) * FE + c4 * 4);
      }
    }
#pragma unroll
    for (int j = 0; j < P0; ++j) {
      const int i = tid + 256 * j;
      const int m = i / (FE / 4), c4 = i - m * (FE / 4);
      if (m < Mp) {
        bf16x4 b;
        b[0] = (bf16)v[j][0], b[1] = (bf16)v[j][1], b[2] = (bf16)v[j][2], b[3] = (bf16)v[j][3];
        *(bf16x4*)(As + m * AST + c4 * 4) = b;
      }
    }
  }
  for (int i = tid; i < QTAIL * QST / 8; i += 256) *(u32x4*)(Qs + Mp * QST + i * 8) = u32x4{0u, 0u, 0u, 0u};
  wstash();
  __syncthreads();
  FB_STAMP(1);

  const int nt = (T + 15) >> 4;  // 16-token tiles per row (<= 4)
  for (int h = 0; h < FH; ++h) {
    // ---- QKV_h^T [96 features][tokens]: wave owns token tiles wave, wave + 4
    f32x4 acc[2][6];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int f = 0; f < 6; ++f) acc[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};
    // operands of k-step ks+1 read while k-step ks multiplies (sched barriers keep them early)
    bf16x8 bq[2][2], wq[2][6];
    auto qkv_frags = [&](int ks, int buf) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (wave + 4 * j < ntt)
          bq[buf][j] = *(const bf16x8*)(As + ((wave + 4 * j) * 16 + fr) * AST + ks * 32 + fg * 8);
#pragma unroll
      for (int f = 0; f < 6; ++f) wq[buf][f] = *(const bf16x8*)(Wh + (f * 16 + fr) * AST + ks * 32 + fg * 8);
    };
    qkv_frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < FE / 32; ++ks) {
      if (ks + 1 < FE / 32) qkv_frags(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < 6; ++f)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (wave + 4 * j < ntt) acc[j][f] = mfma16(wq[ks & 1][f], bq[ks & 1][j], acc[j][f]);
    }
    // C^T layout: lane = token (tile col fr), rows = 4 consecutive features -> one 8-B store
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tt = wave + 4 * j;
      if (tt < ntt) {
#pragma unroll
        for (int f = 0; f < 6; ++f) {
          const float sc = f < 2 ? p.qscale : 1.0f;  // Q pre-scaled by log2(e)/sqrt(D)
          bf16x4 o;
          o[0] = (bf16)(acc[j][f][0] * sc), o[1] = (bf16)(acc[j][f][1] * sc);
          o[2] = (bf16)(acc[j][f][2] * sc), o[3] = (bf16)(acc[j][f][3] * sc);
          *(bf16x4*)(Qs + (tt * 16 + fr) * QST + f * 16 + fg * 4) = o;
        }
      }
    }
    __syncthreads();
    FB_STAMP(2 + 3 * h);
    if (h + 1 < FH) wfetch(h + 1);  // lands while this head's attention runs

    // ---- attention of each row (one wave per row)
    for (int r = wave; r < R; r += 4) {
      const int rb = r * T;
      const bf16* rq = Qs + rb * QST;
      f32x4 sc[4][4];
      bf16x8 qf[4];
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
        if (qt < nt) qf[qt] = *(const bf16x8*)(rq + (qt * 16 + fr) * QST + fg * 8);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        if (kt < nt) {
          const bf16x8 kf = *(const bf16x8*)(rq + (kt * 16 + fr) * QST + FD + fg * 8);
#pragma unroll
          for (int qt = 0; qt < 4; ++qt)
            if (qt < nt) sc[kt][qt] = mfma16(kf, qf[qt], f32x4{0.f, 0.f, 0.f, 0.f});
        }
      }
      // softmax over keys (rows of S^T); lane holds keys kt*16 + 4*fg + i for query qt*16 + fr
      float inv_l[4];
      bf16x8 pb[2][4];
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        if (qt >= nt) continue;
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (kt >= nt) continue;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (kt * 16 + fg * 4 + i >= T) sc[kt][qt][i] = -INFINITY;
            mx = fmaxf(mx, sc[kt][qt][i]);
          }
        }
        mx = max_rows4(mx);
        float sum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          if (kt >= nt) continue;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float e = __builtin_amdgcn_exp2f(sc[kt][qt][i] - mx);
            sc[kt][qt][i] = e;
            sum += e;
          }
        }
        sum = sum_rows4(sum);
        inv_l[qt] = __builtin_amdgcn_rcpf(sum);
        // P^T as the B operand: K positions 8*fg + j <-> keys 32*ks + 4*fg + j (j < 4),
        // 32*ks + 16 + 4*fg + (j - 4) (j >= 4): exactly this lane's accumulator rows
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8 b;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            b[j] = (2 * ks < nt) ? (bf16)sc[2 * ks][qt][j] : (bf16)0.f;
            b[4 + j] = (2 * ks + 1 < nt) ? (bf16)sc[2 * ks + 1][qt][j] : (bf16)0.f;
          }
          pb[ks][qt] = b;
        }
      }
      // O^T [D][queries] = V^T P^T with V^T gathered in the same permuted key order
      // (key rows past the buffer are clamped: their P is 0 and the clamped rows are finite)
      f32x4 o[2][4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) o[mt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int nks = (nt + 1) >> 1;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks >= nks) continue;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const bf16* vcol = Qs + 2 * FD + mt * 16 + fr;
          bf16x8 va;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            va[j] = vcol[min(rb + ks * 32 + fg * 4 + j, qrows - 1) * QST];
            va[4 + j] = vcol[min(rb + ks * 32 + 16 + fg * 4 + j, qrows - 1) * QST];
          }
#pragma unroll
          for (int qt = 0; qt < 4; ++qt)
            if (qt < nt) o[mt][qt] = mfma16(va, pb[ks][qt], o[mt][qt]);
        }
      }
      // O^T layout: lane = query, rows = 4 consecutive head dims -> 8-B store into O[token][h*D + d]
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        if (qt >= nt) continue;
        const int q = qt * 16 + fr;
        if (q < T) {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            bf16x4 b;
            b[0] = (bf16)(o[mt][qt][0] * inv_l[qt]), b[1] = (bf16)(o[mt][qt][1] * inv_l[qt]);
            b[2] = (bf16)(o[mt][qt][2] * inv_l[qt]), b[3] = (bf16)(o[mt][qt][3] * inv_l[qt]);
            *(bf16x4*)(Os + (rb + q) * AST + h * FD + mt * 16 + fg * 4) = b;
          }
        }
      }
    }
    __syncthreads();
    FB_STAMP(3 + 3 * h);
    if (h + 1 < FH) {
      wstash();  // W_h's readers (the QKV phase) finished before the barrier above
      __syncthreads();
      FB_STAMP(4 + 3 * h);
    }
  }

  // ---- Wout -> LDS over the dead A / QKV / W_h tiles
  {
    u32x4 w[OPIECES];
#pragma unroll
    for (int j = 0; j < OPIECES; ++j) {
      const int i = tid + 256 * j;
      w[j] = *(const u32x4*)(p.wout + (i / (FE / 8)) * FE + (i % (FE / 8)) * 8);
    }
#pragma unroll
    for (int j = 0; j < OPIECES; ++j) {
      const int i = tid + 256 * j;
      *(u32x4*)(Wo + (i / (FE / 8)) * AST + (i % (FE / 8)) * 8) = w[j];
    }
  }
  __syncthreads();
  FB_STAMP(20);

  // ---- out-projection Y^T [E][tokens] = Wout . O^T, wave owns token tiles wave, wave + 4
  f32x4 y[2][12];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int f = 0; f < 12; ++f) y[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    bf16x8 ob[2][2], ow[2][12];
    auto out_frags = [&](int ks, int buf) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (wave + 4 * j < ntt)
          ob[buf][j] = *(const bf16x8*)(Os + ((wave + 4 * j) * 16 + fr) * AST + ks * 32 + fg * 8);
#pragma unroll
      for (int f = 0; f < 12; ++f) ow[buf][f] = *(const bf16x8*)(Wo + (f * 16 + fr) * AST + ks * 32 + fg * 8);
    };
    out_frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < FE / 32; ++ks) {
      if (ks + 1 < FE / 32) out_frags(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < 12; ++f)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (wave + 4 * j < ntt) y[j][f] = mfma16(ow[ks & 1][f], ob[ks & 1][j], y[j][f]);
    }
  }

  FB_STAMP(21);
  // ---- residual + LayerNorm per token (lane = token, 48 of its 192 features in registers)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tt = wave + 4 * j;
    if (tt >= ntt) continue;  // wave-uniform
    const int m = tt * 16 + fr;
    const bool valid = m < RT;
    const int mr = valid ? m : 0;
    const int r = mr / T, t = mr - r * T;
    float* xr = p.X + t * SE + (int64_t)(s0 + r) * FE + fg * 4;
    float s = 0.f;
#pragma unroll
    for (int f = 0; f < 12; ++f) {
      const f32x4 xv = *(const f32x4*)(xr + f * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[j][f][i] += xv[i];
        s += y[j][f][i];
      }
    }
    s = sum_rows4(s);
    const float mean = s * (1.0f / FE);
    float q = 0.f;
#pragma unroll
    for (int f = 0; f < 12; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dl = y[j][f][i] - mean;
        q += dl * dl;
      }
    q = sum_rows4(q);
    const float inv = 1.0f / sqrtf(q * (1.0f / FE) + p.eps);
    if (valid) {
#pragma unroll
      for (int f = 0; f < 12; ++f) {
        f32x4 ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) ov[i] = (y[j][f][i] - mean) * inv;
        *(f32x4*)(xr + f * 16) = ov;
      }
    }
  }
}

size_t feat_block_lds(int mp) {
  const size_t heads = (size_t)mp * AST + (size_t)(mp + QTAIL) * QST + (size_t)WROWS * AST;
  return ((size_t)mp * AST + std::max(heads, (size_t)FE * AST)) * sizeof(bf16);
}

}  // namespace

#ifdef MMPFN_STAMPS
extern "C" int mmpfn_dbg_featblock_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fb_stamps), sizeof(g_fb_stamps));
}
#endif

int feat_block_rows(int T) { return (T >= 1 && T <= 64) ? MAXTOK / T : 0; }

hipError_t launch_feat_block(float* X, const void* wqkv, const void* wout, int S, int T, int E, int H, float eps,
                             hipStream_t st) {
  if (S <= 0) return hipSuccess;
  const int R = feat_block_rows(T);
  if (E != FE || H != FH || R < 1) return hipErrorInvalidValue;
  FbArgs a;
  a.X = X, a.wqkv = (const bf16*)wqkv, a.wout = (const bf16*)wout;
  a.S = S, a.T = T, a.R = R, a.Mp = (R * T + 15) / 16 * 16;
  a.eps = eps, a.qscale = kLog2e * 0.17677669529663687f;  // log2(e) / sqrt(32)
  static std::atomic<uint64_t> opted{0};  // > 64 KiB dynamic LDS needs an explicit opt-in
  const hipError_t e = lds_optin(opted, (const void*)feat_block_kernel, (int)feat_block_lds(MAXTOK));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(feat_block_kernel, dim3((S + R - 1) / R), dim3(256), feat_block_lds(a.Mp), st, a);
  return hipGetLastError();
}

}  // namespace mmpfn
