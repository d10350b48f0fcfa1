// Input encoders, positional embedding, state assembly and decoder head (gfx950).
//
// x encoder (loading.py:308-371; encoders.py): one block per (feature group, slot) computes
// the column statistics the reference fits on the train rows -- constancy over ALL
// rows (encoders.py:515), NaN/inf fill with the train nanmean (encoders.py:461-493),
// the two-pass 12-sigma soft outlier bounds (encoders.py:133-162), train z-score
// (encoders.py:53-99) and the used-feature rescale (encoders.py:608-655); one more block of
// the same launch takes the label mean.  A second kernel writes the member's whole state:
// the x tokens (statistics applied element-wise, Linear(2*nf -> E), the subspace positional
// embedding, transformer.py:925-933), the mixer tokens + their positional rows and the label
// token, in the state dtype.  Reductions accumulate in fp64.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

__device__ __forceinline__ bool bad(float v) { return isnan(v) || isinf(v); }

__device__ __forceinline__ float soft_clip(float v, float lo, float hi) {
  v = fmaxf(-logf(1.0f + fabsf(v)) + lo, v);  // encoders.py:160
  v = fminf(logf(1.0f + fabsf(v)) + hi, v);   // encoders.py:161
  return v;
}

// NaN-propagating max/min matching torch.maximum / torch.minimum
__device__ __forceinline__ float tmax(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : fmaxf(a, b); }
__device__ __forceinline__ float tmin(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : fminf(a, b); }
__device__ __forceinline__ float soft_clip_t(float v, float lo, float hi) {
  // inside [lo, hi] both steps are the identity (log1p(|v|) >= 0); NaN v / lo / hi take the full form
  if (v >= lo && v <= hi) return v;
  v = tmax(-logf(1.0f + fabsf(v)) + lo, v);
  v = tmin(logf(1.0f + fabsf(v)) + hi, v);
  return v;
}

// Reductions of the statistics kernel: a wave sum identical in every lane (each step pairs lanes
// symmetrically, so both partners add the same two values): DPP quad permutes xor 1 / xor 2, the
// half-row and row mirrors, then the permlane swaps between the 16-lane rows (no LDS round trips)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ double swap_add_d(double v, bool rows32) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto a = rows32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = rows32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double d0 = __longlong_as_double((long long)(((uint64_t)b[0] << 32) | a[0]));
  const double d1 = __longlong_as_double((long long)(((uint64_t)b[1] << 32) | a[1]));
  return d0 + d1;  // {own, partner} in some order: the sum is the same in both lanes
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  v = swap_add_d(v, false);
  return swap_add_d(v, true);
}
// NV sums over a 256-thread block with one barrier; `red` holds two ping-pong sets of 4 * NV doubles (a
// set is rewritten two reductions later, after every thread has passed the barrier of the one between)
struct BlockRed {
  double* red;
  int k = 0;
  template <int NV>
  __device__ __forceinline__ void sum(double (&v)[NV]) {
    double* r = red + (k & 1) * 32;
    ++k;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum_dpp(v[i]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int i = 0; i < NV; ++i) r[4 * i + w] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = (r[4 * i] + r[4 * i + 1]) + (r[4 * i + 2] + r[4 * i + 3]);
  }
};

struct Moments {  // torch_nanmean (clipped count) and torch_nanstd (unbiased)
  float mean_clip, std;
};

// Encoder statistics of one member, one launch: block (g, k) < G * fpg fits slot k of feature group g, the
// last block the label mean (torch.nanmean of the train labels, the NaN fill of the y encoder).  A slot
// block stages its group's fpg columns in LDS ([fpg][S], when they fit), finds the group's non-constant
// columns over all rows (RemoveEmptyFeatures), takes the k-th, and runs the ~9 passes of its statistics:
// 256 threads, each pass ending in one DPP wave reduction + one barrier.  VPT > 0: the selected column is
// held in registers (rows tid + 256 i, S <= 256 VPT), so the passes are unrolled register loops.
template <int VPT>
__global__ __launch_bounds__(256) void enc_stats_kernel(const float* __restrict__ x, int S, int F, int N, int fpg,
                                                        int nslots, float sigma, SlotParams* __restrict__ slots,
                                                        const float* __restrict__ y, int ny, float* __restrict__ ymean,
                                                        int col_lds) {
  __shared__ double red[64];
  extern __shared__ float cols[];  // [fpg][S] when col_lds
  BlockRed br{red};
  const int tid = threadIdx.x;
  if ((int)blockIdx.x == nslots) {  // label mean
    double a[2] = {0.0, 0.0};
#pragma unroll 16  // (independent loads in flight: a rolled loop waits out one memory latency per row)
    for (int s = tid; s < ny; s += 256) {
      const float v = y[s];
      if (!isnan(v)) a[0] += v, a[1] += 1.0;
    }
    br.sum(a);
    if (tid == 0) ymean[0] = (float)(a[0] / a[1]);
    return;
  }
  const int g = blockIdx.x / fpg, k = blockIdx.x - g * fpg;
  auto raw_col = [&](int j, int s) -> float {
    const int c = g * fpg + j;
    if (col_lds) return cols[j * S + s];
    return c < F ? x[(int64_t)s * F + c] : 0.f;  // zero padding column
  };
  if (col_lds) {
    const int n = S * fpg;
#pragma unroll 32  // (all of a typical column's loads in flight at once)
    for (int i = tid; i < n; i += 256) {
      const int s = i / fpg, j = i - s * fpg, c = g * fpg + j;
      cols[j * S + s] = c < F ? x[(int64_t)s * F + c] : 0.f;
    }
    __syncthreads();
  }
  // 1. constancy over all rows of each column of the group
  double eq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) eq[j] = 0.0;
  for (int j = 0; j < fpg; ++j) {
    const float x0 = raw_col(j, 0);
    int e = 0;
    for (int s = 1 + tid; s < S; s += 256) e += raw_col(j, s) == x0;
    eq[j] = (double)e;
  }
  br.sum(eq);
  int jsel = -1;
  for (int j = 0, n = 0; j < fpg; ++j)
    if ((int)(eq[j] + 0.5) != S - 1) {
      if (n == k) jsel = j;
      ++n;
    }
  SlotParams p;
  p.src = jsel >= 0 ? g * fpg + jsel : -1;
  p.fill = 0.f, p.lo = -INFINITY, p.hi = INFINITY, p.mean = 0.f, p.sd = 1.f, p.scale = 0.f;
  if (jsel >= 0) {  // block-uniform
    float xv[VPT > 0 ? VPT : 1];
    if constexpr (VPT > 0) {
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int s = tid + 256 * i;
        xv[i] = s < S ? raw_col(jsel, s) : 0.f;
      }
    }
    // fn(s, raw value) over rows [r0, n) of this thread
    auto for_rows = [&](int r0, int n, auto&& fn) __attribute__((always_inline)) {
      if constexpr (VPT > 0) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int s = tid + 256 * i;
          if (s >= r0 && s < n) fn(xv[i]);
        }
      } else {
        for (int s = r0 + tid; s < n; s += 256) fn(raw_col(jsel, s));
      }
    };
    // nan-skipping moments of f(raw) over rows [0, N); f returns NaN to skip
    auto moments = [&](auto&& f) __attribute__((always_inline)) {
      double a[2] = {0.0, 0.0};  // sum, count
      for_rows(0, N, [&](float r) {
        const float v = f(r);
        if (!isnan(v)) a[0] += (double)v, a[1] += 1.0;
      });
      br.sum(a);
      const double mu = a[0] / a[1];  // unclipped (torch_nanstd)
      double ss[1] = {0.0};
      for_rows(0, N, [&](float r) {
        const float v = f(r);
        if (!isnan(v)) {
          const double dl = mu - (double)v;
          ss[0] += dl * dl;
        }
      });
      br.sum(ss);
      Moments m;
      m.mean_clip = (float)(a[0] / (a[1] < 1.0 ? 1.0 : a[1]));
      m.std = (float)sqrt(ss[0] / (a[1] - 1.0));
      return m;
    };
    {  // NaN handling: torch.nanmean over train rows (inf included)
      double a[2] = {0.0, 0.0};
      for_rows(0, N, [&](float v) {
        if (!isnan(v)) a[0] += (double)v, a[1] += 1.0;
      });
      br.sum(a);
      p.fill = (float)(a[0] / a[1]);
    }
    const float fill = p.fill;
    auto filled = [&](float v) { return bad(v) ? fill : v; };
    if (sigma > 0.f) {
      const Moments a = moments(filled);
      const float lo1 = a.mean_clip - a.std * sigma, hi1 = a.mean_clip + a.std * sigma;
      const Moments b = moments([&](float r) {
        const float v = filled(r);
        return (v > hi1 || v < lo1) ? NAN : v;
      });
      p.lo = b.mean_clip - b.std * sigma;
      p.hi = b.mean_clip + b.std * sigma;
    }
    const float lo = p.lo, hi = p.hi;
    const bool clipping = sigma > 0.f;
    auto clipped = [&](float r) {
      const float v = filled(r);
      return clipping ? soft_clip_t(v, lo, hi) : v;
    };
    const Moments nm = moments(clipped);
    p.mean = nm.mean_clip;
    p.sd = (S == 1 || N == 1) ? 1.0f : nm.std + 1e-20f;
    // used-feature test on the normalised values over all rows
    const float mean = p.mean, sd = p.sd;
    auto normed = [&](float r) { return tmin(tmax((clipped(r) - mean) / sd, -100.f), 100.f); };
    const float u0 = normed(raw_col(jsel, 0));
    int e = 0;
    for_rows(1, S, [&](float r) { e += (normed(r) == u0); });
    double tot[1] = {(double)e};
    br.sum(tot);
    p.scale = (int)(tot[0] + 0.5) != S - 1 ? 1.f : 0.f;  // used flag; the assembly rescales
  }
  if (tid == 0) slots[blockIdx.x] = p;
}

// The member's whole input state X [T][S][E] in one launch, written in the state dtype TX (fp32, or fp16 in
// PREC_F16): rows t < G are the x encoder's tokens (the statistics applied element-wise, Linear(2 nf -> E)
// and the group's positional row; transformer.py:925-933), G <= t < G + C the mixer tokens + their
// positional rows, t = T - 1 the label token (encoders.py target encoder; NaN labels -> train mean,
// indicator -2).  ASM_ROWS rows per block: the per-row encoder inputs (u, NaN / inf indicator; label
// class and indicator) go to LDS once, then each thread writes 16-B pieces of the rows.
constexpr int ASM_ROWS = 32;
constexpr int EMB_EMAX = 256;
struct AsmArgs {
  const float* x;
  int S, F, G, fpg, nf;
  const SlotParams* slots;
  const float* w_enc;  // [E][2 nf]
  const float* pe;     // [G + C][E]
  const float* tok;    // [S][C][E]
  int C;
  const float* y;  // [N] train labels (rows >= N: test rows)
  int N;
  const float* uniq;
  int U;
  const float *yw, *yb, *ymean;
  void* X;
  int E;
  int* flag;
};
template <typename TX>
__global__ __launch_bounds__(256) void assemble_kernel(const AsmArgs a) {
  __shared__ float su[ASM_ROWS][8], si[ASM_ROWS][8];
  __shared__ __attribute__((aligned(16))) float ws[EMB_EMAX * 16];  // [2 nf][E]: a piece's weights are 16-B runs
  const int tid = threadIdx.x, S = a.S, G = a.G, C = a.C, T = G + C + 1, E = a.E, nf = a.nf, fpg = a.fpg;
  const int nrows = T * S, r0 = blockIdx.x * ASM_ROWS;
  const int rn = min(ASM_ROWS, nrows - r0);
  const bool xrows = r0 / S < G;
  if (xrows)
    for (int i = tid; i < E * 2 * nf; i += 256) {
      const int e = i / (2 * nf), k = i - e * 2 * nf;
      ws[k * E + e] = a.w_enc[i];
    }
  for (int it = tid; it < rn * 8; it += 256) {
    const int i = it >> 3, k = it & 7, r = r0 + i, t = r / S, s = r - t * S;
    float u = 0.f, ind = 0.f;
    if (t < G) {
      if (k < fpg) {
        const SlotParams p = a.slots[t * fpg + k];
        float used = 0.f;  // used-feature rescale sqrt(nf / used) of the group (encoders.py:608-655)
        for (int j = 0; j < fpg; ++j) used += a.slots[t * fpg + j].scale;
        const float scale = sqrtf((float)nf / fmaxf(used, 1.f));
        if (p.src >= 0) {
          const float raw = a.x[(int64_t)s * a.F + p.src];
          ind = isnan(raw) ? -2.0f : (isinf(raw) ? (raw > 0 ? 2.0f : 4.0f) : 0.0f);
          float v = bad(raw) ? p.fill : raw;
          v = soft_clip_t(v, p.lo, p.hi);
          v = tmin(tmax((v - p.mean) / p.sd, -100.f), 100.f);
          u = v * scale;
        }
      }
    } else if (t == T - 1 && k == 0) {
      float yv = s < a.N ? a.y[s] : NAN;
      ind = isnan(yv) ? -2.0f : 0.0f;
      if (isnan(yv)) yv = a.ymean[0];
      for (int i2 = 0; i2 < a.U; ++i2) u += (yv > a.uniq[i2]) ? 1.f : 0.f;
    }
    su[i][k] = u, si[i][k] = ind;
  }
  __syncthreads();
  constexpr int PE = 16 / sizeof(TX);  // elements per 16-B piece
  const int npc = E / PE;
  bool nan_x = false, nan_y = false;
  for (int item = tid; item < rn * npc; item += 256) {
    const int i = item / npc, e0 = (item - i * npc) * PE, r = r0 + i, t = r / S, s = r - t * S;
    float o[PE];
    if (t < G) {
#pragma unroll
      for (int c = 0; c < PE; ++c) o[c] = 0.f;
      for (int k = 0; k < nf; ++k) {
        const float u = su[i][k];
#pragma unroll
        for (int c = 0; c < PE; ++c) o[c] = fmaf(u, ws[k * E + e0 + c], o[c]);
      }
      for (int k = 0; k < nf; ++k) {
        const float u = si[i][k];
#pragma unroll
        for (int c = 0; c < PE; ++c) o[c] = fmaf(u, ws[(nf + k) * E + e0 + c], o[c]);
      }
      const float* pr = a.pe + t * E + e0;
#pragma unroll
      for (int c = 0; c < PE; ++c) {
        o[c] += pr[c];
        nan_x |= isnan(o[c]);
      }
    } else if (t < G + C) {
      const float* tr = a.tok + ((int64_t)s * C + (t - G)) * E + e0;
#pragma unroll
      for (int c = 0; c < PE; c += 4) {
        const f32x4 v = *(const f32x4*)(tr + c) + *(const f32x4*)(a.pe + t * E + e0 + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) o[c + q] = v[q], nan_x |= isnan(v[q]);
      }
    } else {
      const float yc = su[i][0], ind = si[i][0];
#pragma unroll
      for (int c = 0; c < PE; ++c) {
        const int e = e0 + c;
        o[c] = fmaf(ind, a.yw[e * 2 + 1], yc * a.yw[e * 2]) + a.yb[e];
        nan_y |= isnan(o[c]);
      }
    }
    TX* dst = (TX*)a.X + (int64_t)r * E + e0;
    if constexpr (PE == 4) {
      *(f32x4*)dst = f32x4{o[0], o[1], o[2], o[3]};
    } else {
      f16x8 h;
#pragma unroll
      for (int c = 0; c < 8; ++c) h[c] = (f16)o[c];
      *(f16x8*)dst = h;
    }
  }
  if (nan_x) atomicOr(a.flag, 1);
  if (nan_y) atomicOr(a.flag, 2);
}

__global__ void pos_emb_kernel(const float* __restrict__ rnd, int n, const float* __restrict__ w,
                               const float* __restrict__ b, float* __restrict__ out, int E) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * E) return;
  const int e = idx % E, k = idx / E;
  const int D = E / 4;
  float a = 0.f;
  for (int j = 0; j < D; ++j) a = fmaf(rnd[k * D + j], w[e * D + j], a);
  out[idx] = a + b[e];
}

// Decoder (transformer.py:388-403,850-853): out = GELU(X W1^T + b1) W2^T + b2 over the Q test rows
// of M members.  Tiled in two launches: dec_hidden_kernel owns a 32-row x 32-hidden tile (X rows
// and the W1 column slice in LDS, one thread per hidden unit and 4 rows, exact-erf GELU) and
// writes that tile's partial outputs [Fh/32][Q][n_out]; dec_sum_kernel adds the partials in a
// fixed order (+ b2).  A per-4-row block streaming all of W1 (0.6 MB) was bound by one CU's
// fill rate (27 us alone, 47 us beside the other lane).
constexpr int DT_R = 32, DT_H = 32, DT_RT = DT_R * DT_H / 256;  // rows per thread (4)
__global__ __launch_bounds__(256) void dec_hidden_kernel(const float* __restrict__ X, int Q, int64_t xm,
                                                         const float* __restrict__ w1t, const float* __restrict__ b1,
                                                         int Fh, const float* __restrict__ w2, int n_out,
                                                         float* __restrict__ part, int E) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;                  // [DT_R][E]
  float* ws = xs + DT_R * E;       // [E][DT_H]
  float* hs = ws + E * DT_H;       // [DT_R][DT_H + 1]
  const int m = blockIdx.z, q0 = blockIdx.x * DT_R, h0 = blockIdx.y * DT_H, tid = threadIdx.x;
  X += m * xm;
  part += (int64_t)m * gridDim.y * Q * n_out;
  const int hw = min(DT_H, Fh - h0);  // hidden units of this tile (the last may be partial)
  for (int i = tid; i < DT_R * E; i += 256) {
    const int r = i / E;
    xs[i] = q0 + r < Q ? X[(int64_t)(q0 + r) * E + (i - r * E)] : 0.f;
  }
  for (int i = tid; i < E * DT_H; i += 256) {
    const int e = i / DT_H;
    const int cc = i - e * DT_H;
    ws[i] = cc < hw ? w1t[(int64_t)e * Fh + h0 + cc] : 0.f;
  }
  __syncthreads();
  const int c = tid & (DT_H - 1), rb = (tid / DT_H) * DT_RT;  // DT_RT rows per thread
  float acc[DT_RT];
#pragma unroll
  for (int r = 0; r < DT_RT; ++r) acc[r] = 0.f;
  for (int e = 0; e < E; e += 4) {  // E % 4 == 0: 16-B row reads
    float w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = ws[(e + i) * DT_H + c];
#pragma unroll
    for (int r = 0; r < DT_RT; ++r) {
      const f32x4 xv = *(const f32x4*)(xs + (rb + r) * E + e);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[r] = fmaf(xv[i], w[i], acc[r]);
    }
  }
  const float bb = c < hw ? b1[h0 + c] : 0.f;
#pragma unroll
  for (int r = 0; r < DT_RT; ++r) hs[(rb + r) * (DT_H + 1) + c] = c < hw ? gelu_erf(acc[r] + bb) : 0.f;
  __syncthreads();
  for (int pr = tid; pr < DT_R * n_out; pr += 256) {
    const int r = pr / n_out, j = pr - r * n_out;
    if (q0 + r >= Q) continue;
    const float* wr = w2 + (int64_t)j * Fh + h0;
    float a = 0.f;
    for (int k = 0; k < hw; ++k) a = fmaf(hs[r * (DT_H + 1) + k], wr[k], a);
    part[((int64_t)blockIdx.y * Q + q0 + r) * n_out + j] = a;
  }
}

__global__ __launch_bounds__(256) void dec_sum_kernel(const float* __restrict__ part, int M, int Q, int nt, int n_out,
                                                      const float* __restrict__ b2, float* __restrict__ out,
                                                      int64_t om) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, per = (int64_t)Q * n_out;
  if (i >= M * per) return;
  const int64_t m = i / per, k = i - m * per;
  const float* pm = part + m * nt * per;
  float a = b2[k % n_out];
  for (int t = 0; t < nt; ++t) a += pm[t * per + k];
  out[m * om + k] = a;
}

// Decoder of the 16-bit modes on MFMA (the reference runs it under its fp16 autocast): one block per 16
// query rows of one member, wave w owning hidden units [w Fh / 4, (w + 1) Fh / 4):
//   H^T = W1 X^T on v_mfma_f32_16x16x32 (A: W1 rows from L2, B: the rows' X fragments, the fp32 state
//   rounded / the fp16 state as is), + b1, exact-erf GELU;
//   out^T = W2p G^T with G^T straight from the H^T accumulators (W2's hidden order permuted as the MLP's,
//   weight_pack.h pack_mlp2_perm; outputs padded to 16 rows), the four waves' partial sums added in LDS.
template <typename TX>
__global__ __launch_bounds__(256) void dec_mfma_kernel(const TX* __restrict__ X, int Q, int64_t xm,
                                                       const void* __restrict__ W1v, const float* __restrict__ b1,
                                                       int Fh, const void* __restrict__ W2v,
                                                       const float* __restrict__ b2, int n_out, float* __restrict__ out,
                                                       int64_t om, int E) {
  constexpr bool F16 = sizeof(TX) == 2;
  typedef typename Op16<F16>::t HT;
  typedef typename Op16<F16>::x8 X8;
  __shared__ f32x4 part[4][64];
  const HT* W1 = (const HT*)W1v;
  const HT* W2 = (const HT*)W2v;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
  const int m = blockIdx.y, q0 = blockIdx.x * 16;
  const TX* xr = X + m * xm + (int64_t)min(q0 + fr, Q - 1) * E + 8 * fg;
  const int hw = Fh / 4, h0 = wave * hw;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};  // out^T tile: lane (row fr, outputs 4 fg + i)
  X8 xb[8];  // the rows' X fragments, every k-step (E <= 256), loaded once
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    if (ks < E / 32) {
      if constexpr (F16) {
        xb[ks] = *(const X8*)(xr + 32 * ks);
      } else {
        const f32x4 a = *(const f32x4*)(xr + 32 * ks), b = *(const f32x4*)(xr + 32 * ks + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) xb[ks][j] = (HT)a[j], xb[ks][4 + j] = (HT)b[j];
      }
    }
  }
  for (int hc = 0; hc < hw; hc += 32) {  // 32 hidden units: tiles t = 0, 1
    X8 wa[8][2];  // the chunk's W1 fragments, all issued before its MFMAs
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (ks < E / 32) wa[ks][t] = *(const X8*)(W1 + (int64_t)(h0 + hc + 16 * t + fr) * E + 32 * ks + 8 * fg);
    const X8 wb = *(const X8*)(W2 + (int64_t)fr * Fh + h0 + hc + 8 * fg);
    f32x4 h[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (ks < E / 32) h[t] = mfma16x(wa[ks][t], xb[ks], h[t]);
    // G^T fragment: lane (row fr, fg) <- hidden hc + 16 (j / 4) + 4 fg + j % 4 (the pack_mlp2_perm order)
    X8 gb;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hid = h0 + hc + 16 * t + 4 * fg + i;
        gb[4 * t + i] = (HT)gelu_erf(h[t][i] + b1[hid]);
      }
    acc = mfma16x(wb, gb, acc);
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    const f32x4 s = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (q0 + fr < Q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = 4 * fg + i;
        if (o < n_out) out[m * om + (int64_t)(q0 + fr) * n_out + o] = s[i] + b2[o];
      }
  }
}

// ensemble aggregation (classifier.py:541-566): per query row, per member
// logits[:, :n_cls] / T (if T != 1) -> class-permutation undo -> softmax -> mean
// (or mean -> softmax), optional class re-weighting, renormalise.
__global__ void aggregate_kernel(const float* __restrict__ logits, int M, int Q, int n_out,
                                 const int* __restrict__ perms, int n_cls, float temp, int avg_before,
                                 const float* __restrict__ cw, float* __restrict__ probs) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  const bool slice = temp != 1.0f;
  const int C = (slice || perms) ? n_cls : n_out;
  float acc[16];
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  for (int m = 0; m < M; ++m) {
    const float* row = logits + ((int64_t)m * Q + q) * n_out;
    float v[16];
    for (int c = 0; c < C; ++c) {
      const int src = perms ? perms[m * n_cls + c] : c;
      v[c] = slice ? row[src] / temp : row[src];
    }
    if (avg_before) {
      for (int c = 0; c < C; ++c) acc[c] += v[c];
    } else {
      float mx = -INFINITY;
      for (int c = 0; c < C; ++c) mx = fmaxf(mx, v[c]);
      float s = 0.f;
      for (int c = 0; c < C; ++c) {
        v[c] = expf(v[c] - mx);
        s += v[c];
      }
      for (int c = 0; c < C; ++c) acc[c] += v[c] / s;
    }
  }
  float out[16];
  if (avg_before) {
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, acc[c] / M);
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
      out[c] = expf(acc[c] / M - mx);
      s += out[c];
    }
    for (int c = 0; c < C; ++c) out[c] /= s;
  } else {
    for (int c = 0; c < C; ++c) out[c] = acc[c] / M;
  }
  if (cw) {
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
      out[c] *= cw[c];
      s += out[c];
    }
    for (int c = 0; c < C; ++c) out[c] /= s;
  }
  for (int c = 0; c < C; ++c) probs[(int64_t)q * C + c] = out[c];
}

}  // namespace

hipError_t launch_aggregate(const float* logits, int M, int Q, int n_out, const int* perms, int n_cls, float temp,
                            int avg_before, const float* class_weights, float* probs, hipStream_t st) {
  if (Q <= 0 || M <= 0) return hipSuccess;
  if (n_out > 16 || n_cls > 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(aggregate_kernel, dim3((Q + 127) / 128), dim3(128), 0, st, logits, M, Q, n_out, perms, n_cls,
                     temp, avg_before, class_weights, probs);
  return hipGetLastError();
}

hipError_t launch_encode_stats(const float* x, int S, int F, int N, int G, int fpg, float sigma, SlotParams* slots,
                               const float* y, int ny, float* ymean, hipStream_t st) {
  if (G < 0 || S <= 0 || (G > 0 && (fpg <= 0 || fpg > 8 || !x)) || !y || !ymean) return hipErrorInvalidValue;
  const int nslots = G * fpg;
  const size_t cb = (size_t)S * fpg * sizeof(float);
  const int col_lds = G > 0 && cb <= 128 * 1024 ? 1 : 0;  // stage the group's columns when they fit
  const size_t lds = col_lds ? cb : 0;
  if (lds > 64 * 1024) {
    static std::atomic<uint64_t> opted16{0}, opted0{0};
    const hipError_t e = S <= 256 * 16 ? lds_optin(opted16, (const void*)enc_stats_kernel<16>, 128 * 1024)
                                       : lds_optin(opted0, (const void*)enc_stats_kernel<0>, 128 * 1024);
    if (e != hipSuccess) return e;
  }
  const dim3 grid((unsigned)(nslots + 1));
  if (S <= 256 * 16)
    hipLaunchKernelGGL((enc_stats_kernel<16>), grid, dim3(256), lds, st, x, S, F, N, fpg, nslots, sigma, slots, y, ny,
                       ymean, col_lds);
  else
    hipLaunchKernelGGL((enc_stats_kernel<0>), grid, dim3(256), lds, st, x, S, F, N, fpg, nslots, sigma, slots, y, ny,
                       ymean, col_lds);
  return hipGetLastError();
}

hipError_t launch_assemble(const float* x, int S, int F, int G, int fpg, int nf, const SlotParams* slots,
                           const float* w_enc, const float* posemb, const float* tok, int C, const float* y, int N,
                           const float* uniq, int U, const float* yw, const float* yb, const float* ymean, void* X,
                           bool half, int E, int* flag, hipStream_t st) {
  if (S <= 0 || G < 0 || C < 0 || U < 0 || N < 0 || N > S) return hipErrorInvalidValue;
  if ((G > 0 && (!x || !slots || fpg <= 0 || fpg > 8 || nf > 8 || nf < fpg)) || (C > 0 && !tok) || (N > 0 && !y))
    return hipErrorInvalidValue;
  if (E > EMB_EMAX || E % (half ? 8 : 4) != 0 || (int64_t)(G + C + 1) * S >= INT32_MAX / 2) return hipErrorInvalidValue;
  AsmArgs a;
  a.x = x, a.S = S, a.F = F, a.G = G, a.fpg = fpg, a.nf = nf, a.slots = slots, a.w_enc = w_enc, a.pe = posemb;
  a.tok = tok, a.C = C, a.y = y, a.N = N, a.uniq = uniq, a.U = U, a.yw = yw, a.yb = yb, a.ymean = ymean;
  a.X = X, a.E = E, a.flag = flag;
  const int nb = (int)(((int64_t)(G + C + 1) * S + ASM_ROWS - 1) / ASM_ROWS);
  if (half)
    hipLaunchKernelGGL((assemble_kernel<f16>), dim3(nb), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((assemble_kernel<float>), dim3(nb), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_pos_emb(const float* rnd, int n, const float* w, const float* b, float* out, int E,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pos_emb_kernel, dim3((n * E + 255) / 256), dim3(256), 0, st, rnd, n, w, b, out, E);
  return hipGetLastError();
}

hipError_t launch_decoder(const float* X, int Q, const float* w1t, const float* b1, int Fh, const float* w2,
                          const float* b2, int n_out, float* out, int E, hipStream_t st, int M, int64_t xm, int64_t om,
                          float* scratch) {
  if (Q <= 0 || M <= 0) return hipSuccess;
  if (Fh <= 0 || !scratch || E % 4 != 0) return hipErrorInvalidValue;
  const size_t lds = (size_t)(DT_R * E + E * DT_H + DT_R * (DT_H + 1)) * sizeof(float);  // 81 KB at E = 192
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int nt = (Fh + DT_H - 1) / DT_H;
  hipLaunchKernelGGL(dec_hidden_kernel, dim3((Q + DT_R - 1) / DT_R, nt, M), dim3(256), lds, st, X, Q, xm, w1t, b1, Fh,
                     w2, n_out, scratch, E);
  const int64_t n = (int64_t)M * Q * n_out;
  hipLaunchKernelGGL(dec_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, scratch, M, Q, nt, n_out, b2,
                     out, om);
  return hipGetLastError();
}

hipError_t launch_decoder_mfma(const void* X, bool x_f16, int Q, const void* W1, const float* b1, int Fh, const void* W2p,
                               const float* b2, int n_out, float* out, int E, hipStream_t st, int M, int64_t xm,
                               int64_t om) {
  if (Q <= 0 || M <= 0) return hipSuccess;
  if (E % 32 != 0 || E > 256 || Fh % 128 != 0 || n_out > 16 || n_out <= 0) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((Q + 15) / 16), (unsigned)M);
  if (x_f16)
    hipLaunchKernelGGL((dec_mfma_kernel<f16>), grid, dim3(256), 0, st, (const f16*)X, Q, xm, W1, b1, Fh, W2p, b2, n_out,
                       out, om, E);
  else
    hipLaunchKernelGGL((dec_mfma_kernel<float>), grid, dim3(256), 0, st, (const float*)X, Q, xm, W1, b1, Fh, W2p, b2,
                       n_out, out, om, E);
  return hipGetLastError();
}

// ---- PREC_F16 state conversions (the encoders and the decoder work in fp32; the layers keep an fp16 state)
namespace {
// out[b][r][:] = in[b][r][:] over nb blocks of rows x E elements with block strides (4 elements per thread)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cvt_rows_kernel(const TI* __restrict__ in, int64_t in_bstride, TO* __restrict__ out,
                                                       int64_t out_bstride, int64_t per_block4, int nb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= per_block4 * nb) return;
  const int64_t b = i / per_block4, j = (i - b * per_block4) * 4;
  const TI* s = in + b * in_bstride + j;
  TO* d = out + b * out_bstride + j;
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = (TO)(float)s[k];
}
// out[s][t][e] (fp32, reference order) = X[t][s][e] (fp16 state)
__global__ __launch_bounds__(256) void state_f16_to_f32_kernel(const f16* __restrict__ X, float* __restrict__ out, int S,
                                                               int T, int E) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = (int64_t)S * T * E;
  if (i >= n) return;
  const int e = (int)(i % E);
  const int64_t st = i / E;
  const int t = (int)(st % T), s = (int)(st / T);
  out[i] = (float)X[((int64_t)t * S + s) * E + e];
}
}  // namespace

hipError_t launch_f32_to_f16(const float* in, int64_t in_bstride, void* out, int64_t out_bstride, int64_t per_block,
                             int nb, hipStream_t st) {
  if (per_block <= 0 || nb <= 0) return hipSuccess;
  if (per_block % 4) return hipErrorInvalidValue;
  const int64_t n4 = per_block / 4 * nb;
  hipLaunchKernelGGL((cvt_rows_kernel<float, f16>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, in,
                     in_bstride, (f16*)out, out_bstride, per_block / 4, nb);
  return hipGetLastError();
}

hipError_t launch_f16_to_f32(const void* in, int64_t in_bstride, float* out, int64_t out_bstride, int64_t per_block,
                             int nb, hipStream_t st) {
  if (per_block <= 0 || nb <= 0) return hipSuccess;
  if (per_block % 4) return hipErrorInvalidValue;
  const int64_t n4 = per_block / 4 * nb;
  hipLaunchKernelGGL((cvt_rows_kernel<f16, float>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                     (const f16*)in, in_bstride, out, out_bstride, per_block / 4, nb);
  return hipGetLastError();
}

hipError_t launch_state_f16_to_f32(const void* X, float* out, int S, int T, int E, hipStream_t st) {
  const int64_t n = (int64_t)S * T * E;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(state_f16_to_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const f16*)X, out, S,
                     T, E);
  return hipGetLastError();
}

}  // namespace mmpfn
