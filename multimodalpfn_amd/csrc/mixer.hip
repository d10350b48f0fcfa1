// Helper kernels of the modality projection heads (transformer.py:33-128):
// row LayerNorm (MGM/MoE input norm, CAP k_norm), the CAP cross-attention core,
// CAP's out_norm(o) + ffn(o) combine and the MoE gate.  The heavy contractions
// (per-head Linear(768,768)+GLU, Linear(384,E), CAP in/out projections, FFN,
// MoE experts) run on the MFMA GEMM in gemm.hip.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

// one wave per row; two-pass mean / biased variance (torch layer_norm).  Rows with
// dim % 4 == 0 and dim <= 4 * 64 * V4 are read once into registers as float4 (V4 per lane);
// others take the strided three-pass loop.
template <typename TO, int V4>
__global__ __launch_bounds__(256) void ln_rows_kernel(const float* __restrict__ in, int64_t rows, int dim, float eps,
                                                      TO* __restrict__ out, const float* __restrict__ g,
                                                      const float* __restrict__ b) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* x = in + row * dim;
  TO* o = out + row * dim;
  if constexpr (V4 > 0) {
    const int n4 = dim >> 2;
    f32x4 v[V4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V4; ++j) {
      const int i4 = lane + 64 * j;
      v[j] = i4 < n4 ? *(const f32x4*)(x + 4 * i4) : f32x4{0.f, 0.f, 0.f, 0.f};
      s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    }
    const float mean = wave_sum(s) / dim;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < V4; ++j)
      if (lane + 64 * j < n4)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[j][e] - mean;
          q += d * d;
        }
    const float inv = 1.0f / sqrtf(wave_sum(q) / dim + eps);
#pragma unroll
    for (int j = 0; j < V4; ++j) {
      const int i4 = lane + 64 * j;
      if (i4 >= n4) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float w = (v[j][e] - mean) * inv;
        if (g) w = w * g[4 * i4 + e] + b[4 * i4 + e];
        o[4 * i4 + e] = from_f32<TO>(w);
      }
    }
  } else {
    float s = 0.f;
    for (int i = lane; i < dim; i += 64) s += x[i];
    const float mean = wave_sum(s) / dim;
    float q = 0.f;
    for (int i = lane; i < dim; i += 64) {
      const float d = x[i] - mean;
      q += d * d;
    }
    const float inv = 1.0f / sqrtf(wave_sum(q) / dim + eps);
    for (int i = lane; i < dim; i += 64) {
      float v = (x[i] - mean) * inv;
      if (g) v = v * g[i] + b[i];
      o[i] = from_f32<TO>(v);
    }
  }
}

// CAP core: per row s, per head h: softmax(q_h k_h^T / sqrt(hd)) v_h with the learned
// queries q [cap][E] (in-projected, shared by all rows) and k/v = kv[s][j][0:E] /
// kv[s][j][E:2E] for the M mixer tokens.  One block per row with one thread per
// (head, query) pair (cap^2 <= 1024; larger cap loops); the row's keys are staged through
// LDS once per chunk of up to 64 keys (all M = 64 at mgm 64; bf16 keys stay bf16 in LDS, 49 KB,
// so three rows' blocks share a CU) and consumed in 32-key
// register sub-chunks by a chunked online softmax in fp32 (exp2 with log2(e) folded into
// the query scale).  HD (head dim = E / cap) is a template parameter so the per-thread
// q / acc arrays stay in registers.
constexpr int CAP_KC = 32;
constexpr int CAP_STAGE = 64;

// HD-wide row of K or V from LDS as fp32 (bf16 rows: 16-B reads when HD % 8 == 0)
template <typename TK, int HD>
__device__ __forceinline__ void cap_row(const TK* r, float (&o)[HD]) {
  if constexpr (sizeof(TK) == 2 && HD % 8 == 0) {
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
      const bf16x8 v = *(const bf16x8*)(r + 8 * c);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[8 * c + i] = (float)v[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < HD; ++i) o[i] = to_f32(r[i]);
  }
}

template <typename TK, typename TO, int HD>
__global__ __launch_bounds__(1024) void cap_attn_kernel(const float* __restrict__ qp, const TK* __restrict__ kv,
                                                        TO* __restrict__ out, int M, int cap, int E, int kcmax) {
  extern __shared__ __attribute__((aligned(16))) unsigned char cap_lds[];
  TK* ks = (TK*)cap_lds;  // [kcmax][2E] in the storage type (bf16: 49 KB at M = 64, E = 192)
  const int s = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const float scale = 1.4426950408889634f / sqrtf((float)HD);
  const TK* kvs = kv + (int64_t)s * M * 2 * E;
  const int pairs = cap * cap;
  for (int pb = 0; pb < pairs; pb += nt) {
    const int pair = pb + tid;
    const bool active = pair < pairs;
    // head-major pairs: a wave's lanes read the K/V rows of ~3 heads (LDS broadcast); the
    // query-major order (coalesced stores) measured 2.6x slower on LDS bank conflicts
    const int h = active ? pair / cap : 0, c = active ? pair % cap : 0;
    float q[HD], acc[HD];
#pragma unroll
    for (int i = 0; i < HD; ++i) {
      q[i] = qp[c * E + h * HD + i] * scale;
      acc[i] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < M; k0 += kcmax) {
      const int kc = min(kcmax, M - k0);
      __syncthreads();
      {  // 16-B copies (2E * sizeof(TK) per key is a multiple of 16: E % 4 == 0 checked at launch)
        const int n16 = kc * 2 * E * (int)sizeof(TK) / 16;
        const u32x4* src = (const u32x4*)(kvs + (int64_t)k0 * 2 * E);
        u32x4* dst = (u32x4*)ks;
        for (int i = tid; i < n16; i += nt) dst[i] = src[i];
      }
      __syncthreads();
      if (!active) continue;
      for (int j0 = 0; j0 < kc; j0 += CAP_KC) {
        const int jc = min(CAP_KC, kc - j0);
        float sc[CAP_KC];
        float cm = -INFINITY;
#pragma unroll
        for (int kk = 0; kk < CAP_KC; ++kk) {
          float a = -INFINITY;
          if (kk < jc) {
            float kr[HD];
            cap_row<TK, HD>(ks + (j0 + kk) * 2 * E + h * HD, kr);
            a = 0.f;
#pragma unroll
            for (int i = 0; i < HD; ++i) a = fmaf(q[i], kr[i], a);
          }
          sc[kk] = a;
          cm = fmaxf(cm, a);
        }
        const float mn = fmaxf(m, cm);
        const float corr = __builtin_amdgcn_exp2f(m - mn);
        l *= corr;
#pragma unroll
        for (int i = 0; i < HD; ++i) acc[i] *= corr;
#pragma unroll
        for (int kk = 0; kk < CAP_KC; ++kk) {
          if (kk < jc) {
            const float pe = __builtin_amdgcn_exp2f(sc[kk] - mn);
            l += pe;
            float vr[HD];
            cap_row<TK, HD>(ks + (j0 + kk) * 2 * E + E + h * HD, vr);
#pragma unroll
            for (int i = 0; i < HD; ++i) acc[i] = fmaf(pe, vr[i], acc[i]);
          }
        }
        m = mn;
      }
    }
    if (active) {
      const float inv = 1.0f / l;
      TO* o = out + ((int64_t)s * cap + c) * E + h * HD;
#pragma unroll
      for (int i = 0; i < HD; ++i) o[i] = (TO)(acc[i] * inv);
    }
  }
}

// CAP core on MFMA (bf16 mode: head dim 8, 24 heads = 24 learned queries, M = 32 MB MGM tokens): one wave
// per table row s, four rows per block, operands straight from HBM / L2 (no LDS):
//   * S^T_h = K_h Q_h^T on v_mfma_f32_32x32x16_bf16, one K step = the 16 dims of a head pair: the A operand
//     (K rows of a 32-key block, row index bits 2 and 3 swapped) serves both heads, the B operand (the
//     constant Q^T, log2(e)/sqrt(8) folded in) is zero outside head h's 8 dims (lane half hh != h & 1);
//   * softmax over the M keys of each query (lane = query: 16 keys per key block here, 16 in lane l ^ 32),
//     P normalised before the product;
//   * O^T_g += V^T_g P_h^T for the 32-dim block g = h / 4: V^T rows outside head h's 8 dims are zeroed, the
//     P^T fragment is the S^T accumulator itself (the row swap makes a lane's 8 values 8 consecutive keys).
// Queries >= cap (lanes r >= 24) compute garbage and are not stored.  Versus one thread per (head, query)
// with the row's K|V staged in LDS (cap_attn_kernel): 16x the MFMA arithmetic of the real work, but no
// scalar dot products.
constexpr int CAPM_NH = 24;  // heads (= cap queries) of the MFMA form, head dim 8: E = 192
template <int MB>
__global__ __launch_bounds__(256) void cap_attn_mfma_kernel(const float* __restrict__ qp, const bf16* __restrict__ K,
                                                            const bf16* __restrict__ VT, bf16* __restrict__ out, int S,
                                                            int cap) {
  constexpr int E = 8 * CAPM_NH, M = 32 * MB;
  const int lane = threadIdx.x & 63, s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;  // wave-uniform; no barriers below
  const int r = lane & 31, hh = lane >> 5;
  const float sc = kLog2e * 0.35355339059327373f;  // log2(e) / sqrt(8)
  const bf16x8 zero8 = {};
  const int pk = (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1);  // key of A row r (bits 2 and 3 swapped)
  const bf16* Ks = K + (int64_t)s * M * E + (int64_t)pk * E + 8 * hh;
  const bf16* Vs = VT + (int64_t)s * E * M + (int64_t)r * M + 8 * hh;
  bf16* orow = out + ((int64_t)s * cap + r) * E + 4 * hh;
#pragma unroll 1  // (six unrolled copies: 24 head bodies, beyond the instruction cache)
  for (int g = 0; g < E / 32; ++g) {
    bf16x8 vf[MB][2];  // V^T block g: dims 32 g + r, keys 32 kb + 16 t + 8 hh .. +7
#pragma unroll
    for (int kb = 0; kb < MB; ++kb)
#pragma unroll
      for (int t = 0; t < 2; ++t) vf[kb][t] = *(const bf16x8*)(Vs + (int64_t)32 * g * M + 32 * kb + 16 * t);
    f32x16 o = {};
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {  // the two head pairs of block g
      const int p = 2 * g + pp;
      // Q^T fragment of the pair: lane (query r, half hh) <- Q[r][16 p + 8 hh .. +7] * log2(e)/sqrt(8) (0: r >= cap)
      bf16x8 qf;
      {
        const float* qr = qp + (r < cap ? r : 0) * E + 16 * p + 8 * hh;
        const f32x4 a = *(const f32x4*)qr, b = *(const f32x4*)(qr + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) qf[j] = (bf16)(r < cap ? a[j] * sc : 0.f), qf[4 + j] = (bf16)(r < cap ? b[j] * sc : 0.f);
      }
      bf16x8 kf[MB];
#pragma unroll
      for (int kb = 0; kb < MB; ++kb) kf[kb] = *(const bf16x8*)(Ks + (int64_t)32 * kb * E + 16 * p);
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const int hq = 2 * pp + hs;  // head 4 g + hq
        const bf16x8 qm = hh == hs ? qf : zero8;
        f32x16 sa[MB];
#pragma unroll
        for (int kb = 0; kb < MB; ++kb) sa[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kb], qm, f32x16{}, 0, 0, 0);
        float m = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < MB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) m = fmaxf(m, sa[kb][i]);
        {
          const auto w = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
          m = fmaxf(__uint_as_float(w[0]), __uint_as_float(w[1]));
        }
        float l = 0.f;
#pragma unroll
        for (int kb = 0; kb < MB; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            sa[kb][i] = __builtin_amdgcn_exp2f(sa[kb][i] - m);
            l += sa[kb][i];
          }
        {
          const auto w = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
          l = __uint_as_float(w[0]) + __uint_as_float(w[1]);
        }
        const float inv = 1.0f / l;
        const bool mine = (r >> 3) == hq;  // V^T row r of block g belongs to head 4 g + hq
#pragma unroll
        for (int kb = 0; kb < MB; ++kb)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            bf16x8 pf;
#pragma unroll
            for (int j = 0; j < 8; ++j) pf[j] = (bf16)(sa[kb][8 * t + j] * inv);
            o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(mine ? vf[kb][t] : zero8, pf, o, 0, 0, 0);
          }
      }
    }
    // O^T block g: lane (query r, half hh), element i = dim 32 g + (i & 3) + 8 (i >> 2) + 4 hh
    if (r < cap)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        bf16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (bf16)o[4 * k + i];
        *(bf16x4*)(orow + 32 * g + 8 * k) = v;
      }
  }
}

// out = LN(o) * g + b + f   (CAP: out_norm(out) + ffn(out), transformer.py:86)
__global__ __launch_bounds__(256) void ln_add_kernel(const float* __restrict__ o, const float* __restrict__ f,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float* __restrict__ out, int64_t rows, int E, float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* x = o + row * E;
  float s = 0.f;
  for (int i = lane; i < E; i += 64) s += x[i];
  const float mean = wave_sum(s) / E;
  float q = 0.f;
  for (int i = lane; i < E; i += 64) {
    const float d = x[i] - mean;
    q += d * d;
  }
  const float inv = 1.0f / sqrtf(wave_sum(q) / E + eps);
  for (int i = lane; i < E; i += 64) out[row * E + i] = ((x[i] - mean) * inv * g[i] + b[i]) + f[row * E + i];
}

// MoE gate: probs[s] = softmax(x[s] W^T + b)  (transformer.py:112-113)
__global__ __launch_bounds__(256) void gate_kernel(const float* __restrict__ x, int64_t ldx, int D,
                                                   const float* __restrict__ w, const float* __restrict__ b, int n,
                                                   float* __restrict__ probs) {
  extern __shared__ float lg[];
  const int s = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float* xr = x + (int64_t)s * ldx;
  for (int i = wave; i < n; i += 4) {
    const float* wr = w + (int64_t)i * D;
    float a = 0.f;
    for (int k = lane; k < D; k += 64) a = fmaf(xr[k], wr[k], a);
    a = wave_sum(a);
    if (lane == 0) lg[i] = a + b[i];
  }
  __syncthreads();
  if (wave == 0) {
    float mx = -INFINITY;
    for (int i = lane; i < n; i += 64) mx = fmaxf(mx, lg[i]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int i = lane; i < n; i += 64) sum += expf(lg[i] - mx);
    sum = wave_sum(sum);
    for (int i = lane; i < n; i += 64) probs[(int64_t)s * n + i] = expf(lg[i] - mx) / sum;
  }
}

__global__ void scale_tokens_kernel(float* __restrict__ tok, const float* __restrict__ probs, int64_t total, int E) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  tok[i] *= probs[i / E];
}

}  // namespace

hipError_t launch_layernorm_rows(const float* in, int64_t rows, int dim, float eps, void* out, bool out_f32,
                                 const float* gamma, const float* beta, hipStream_t st, bool out_f16) {
  if (rows <= 0) return hipSuccess;
  dim3 grid((rows + 3) / 4);
  const int v4 = dim % 4 ? 0 : (dim / 4 + 63) / 64;  // float4 registers per lane
  auto go = [&](auto tag, auto vc) {
    using TO = decltype(tag);
    hipLaunchKernelGGL((ln_rows_kernel<TO, decltype(vc)::value>), grid, dim3(256), 0, st, in, rows, dim, eps,
                       (TO*)out, gamma, beta);
  };
  auto pick = [&](auto tag) {
    if (v4 == 1) go(tag, std::integral_constant<int, 1>{});
    else if (v4 == 2) go(tag, std::integral_constant<int, 2>{});
    else if (v4 == 3) go(tag, std::integral_constant<int, 3>{});
    else if (v4 == 4) go(tag, std::integral_constant<int, 4>{});
    else go(tag, std::integral_constant<int, 0>{});
  };
  if (out_f32) pick(float{});
  else if (out_f16) pick(_Float16{});
  else pick(bf16{});
  return hipGetLastError();
}

template <typename TK, typename TO>
hipError_t launch_cap_t(const float* qp, const TK* kv, TO* out, int S, int M, int cap, int E, hipStream_t st) {
  // the row's keys staged in their storage type, chunks of up to 64 keys within 96 KiB of LDS
  if (E % 4 != 0) return hipErrorInvalidValue;
  const int kcmax = max(1, min(CAP_STAGE, 98304 / (2 * E * (int)sizeof(TK))));
  const size_t lds = (size_t)kcmax * 2 * E * sizeof(TK);
  const int pairs = cap * cap;
  dim3 g(S), b((unsigned)min(1024, (pairs + 63) / 64 * 64));
  switch (E / cap) {
    case 96: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 96>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 48: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 48>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 24: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 24>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 16: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 16>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 12: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 12>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 8: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 8>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 6: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 6>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 4: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 4>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 3: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 3>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 2: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 2>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    case 1: hipLaunchKernelGGL((cap_attn_kernel<TK, TO, 1>), g, b, lds, st, qp, kv, out, M, cap, E, kcmax); break;
    default: return hipErrorInvalidValue;  // cap_heads with E / cap outside the instantiated set
  }
  return hipGetLastError();
}

hipError_t launch_cap_attention(const float* qp, const void* kv, bool kv_f32, void* out, bool out_bf16, int S, int M,
                                int cap, int E, hipStream_t st) {
  if (S <= 0) return hipSuccess;
  if (E % cap != 0) return hipErrorInvalidValue;
  if (kv_f32) return out_bf16 ? launch_cap_t(qp, (const float*)kv, (bf16*)out, S, M, cap, E, st)
                              : launch_cap_t(qp, (const float*)kv, (float*)out, S, M, cap, E, st);
  return out_bf16 ? launch_cap_t(qp, (const bf16*)kv, (bf16*)out, S, M, cap, E, st)
                  : launch_cap_t(qp, (const bf16*)kv, (float*)out, S, M, cap, E, st);
}

hipError_t launch_cap_attention_mfma(const float* qp, const void* K, const void* VT, void* out, int S, int M, int cap,
                                     int E, hipStream_t st) {
  if (S <= 0) return hipSuccess;
  if (E != 8 * CAPM_NH || cap != CAPM_NH || M % 32 != 0 || M > 128 || M <= 0) return hipErrorNotSupported;
  const dim3 grid((unsigned)((S + 3) / 4));
  const bf16 *k = (const bf16*)K, *vt = (const bf16*)VT;
  bf16* o = (bf16*)out;
  switch (M / 32) {
    case 1: hipLaunchKernelGGL((cap_attn_mfma_kernel<1>), grid, dim3(256), 0, st, qp, k, vt, o, S, cap); break;
    case 2: hipLaunchKernelGGL((cap_attn_mfma_kernel<2>), grid, dim3(256), 0, st, qp, k, vt, o, S, cap); break;
    case 3: hipLaunchKernelGGL((cap_attn_mfma_kernel<3>), grid, dim3(256), 0, st, qp, k, vt, o, S, cap); break;
    default: hipLaunchKernelGGL((cap_attn_mfma_kernel<4>), grid, dim3(256), 0, st, qp, k, vt, o, S, cap); break;
  }
  return hipGetLastError();
}

hipError_t launch_ln_add(const float* o, const float* f, const float* g, const float* b, float* out, int64_t rows,
                         int E, float eps, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(ln_add_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, o, f, g, b, out, rows, E, eps);
  return hipGetLastError();
}

hipError_t launch_gate_softmax(const float* x, int64_t ldx, int S, int D, const float* w, const float* b, int n,
                               float* probs, hipStream_t st) {
  if (S <= 0) return hipSuccess;
  hipLaunchKernelGGL(gate_kernel, dim3(S), dim3(256), n * sizeof(float), st, x, ldx, D, w, b, n, probs);
  return hipGetLastError();
}

hipError_t launch_scale_tokens(float* tok, const float* probs, int S, int n, int E, hipStream_t st) {
  const int64_t total = (int64_t)S * n * E;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(scale_tokens_kernel, dim3((total + 255) / 256), dim3(256), 0, st, tok, probs, total, E);
  return hipGetLastError();
}

}  // namespace mmpfn
