// Input encoders, positional embedding, token assembly and decoder head (gfx950).
//
// x encoder (loading.py:308-371; encoders.py): one block per feature group computes
// the column statistics the reference fits on the train rows -- constancy over ALL
// rows (encoders.py:515), NaN/inf fill with the train nanmean (encoders.py:461-493),
// the two-pass 12-sigma soft outlier bounds (encoders.py:133-162), train z-score
// (encoders.py:53-99) and the used-feature rescale (encoders.py:608-655).  A second
// kernel applies them element-wise, embeds with Linear(2*nf -> E) and adds the
// subspace positional embedding (transformer.py:925-933), writing token g of the
// [T][S][E] state.  Reductions accumulate in fp64.
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
  v = tmax(-logf(1.0f + fabsf(v)) + lo, v);
  v = tmin(logf(1.0f + fabsf(v)) + hi, v);
  return v;
}

struct Moments {  // torch_nanmean (clipped count) and torch_nanstd (unbiased)
  float mean_clip, std;
};

// nan-skipping moments of f(s) over rows [0, n); f returns NaN to skip
template <typename Fn>
__device__ Moments nan_moments(int n, Fn f, double* red) {
  double sum = 0.0, cnt = 0.0;
  for (int s = threadIdx.x; s < n; s += blockDim.x) {
    const float v = f(s);
    if (!isnan(v)) {
      sum += (double)v;
      cnt += 1.0;
    }
  }
  sum = block_sum_d(sum, red);
  cnt = block_sum_d(cnt, red + 16);
  const double mu = sum / cnt;  // unclipped (torch_nanstd)
  double ss = 0.0;
  for (int s = threadIdx.x; s < n; s += blockDim.x) {
    const float v = f(s);
    if (!isnan(v)) {
      const double dl = mu - (double)v;
      ss += dl * dl;
    }
  }
  ss = block_sum_d(ss, red + 32);
  Moments m;
  m.mean_clip = (float)(sum / (cnt < 1.0 ? 1.0 : cnt));
  m.std = (float)sqrt(ss / (cnt - 1.0));
  return m;
}

// 1024 threads (16 waves): each pass over the rows is two strided loads per thread, so the
// ~9 dependent passes per column are short; reduction slots of 16 waves at red + {0,16,32}
__global__ __launch_bounds__(1024) void enc_x_stats_kernel(const float* __restrict__ x, int S, int F, int N, int fpg,
                                                           int nf, float sigma, SlotParams* __restrict__ slots,
                                                           int col_lds) {
  __shared__ double red[48];
  extern __shared__ float colv[];  // col_lds: the slot's column (S rows) staged once for the ~9 passes
  __shared__ int s_cnt[8];
  const int g = blockIdx.x;
  // 1. constancy over all rows (RemoveEmptyFeatures) for each column of the group
  int src_of_slot[8];
  int nsel = 0;
  for (int j = 0; j < fpg; ++j) {
    const int c = g * fpg + j;
    int eq = 0;
    if (c < F) {
      const float x0 = x[c];
      for (int s = 1 + threadIdx.x; s < S; s += blockDim.x) eq += (x[(int64_t)s * F + c] == x0);
    } else {
      for (int s = 1 + threadIdx.x; s < S; s += blockDim.x) eq += 1;  // zero padding column
    }
    const double tot = block_sum_d((double)eq, red);
    const bool sel = (int)(tot + 0.5) != S - 1;
    if (sel) src_of_slot[nsel++] = c;
  }
  for (int k = nsel; k < fpg; ++k) src_of_slot[k] = -1;

  // this block's slot (blockIdx.y): the slots of a group are independent once the group's
  // constant columns are known; the embed kernel sums the groups' used flags
  {
    const int k = blockIdx.y;
    const int c = src_of_slot[k];
    SlotParams p;
    p.src = c;
    p.fill = 0.f;
    p.lo = -INFINITY;
    p.hi = INFINITY;
    p.mean = 0.f;
    p.sd = 1.f;
    p.scale = 1.f;
    if (c >= 0 && col_lds) {
      for (int s = threadIdx.x; s < S; s += blockDim.x) colv[s] = x[(int64_t)s * F + c];
      __syncthreads();
    }
    if (c >= 0) {
      auto raw = [&](int s) { return col_lds ? colv[s] : x[(int64_t)s * F + c]; };
      // NaN handling: torch.nanmean over train rows (inf included)
      {
        double sum = 0.0, cnt = 0.0;
        for (int s = threadIdx.x; s < N; s += blockDim.x) {
          const float v = raw(s);
          if (!isnan(v)) {
            sum += (double)v;
            cnt += 1.0;
          }
        }
        sum = block_sum_d(sum, red);
        cnt = block_sum_d(cnt, red + 16);
        p.fill = (float)(sum / cnt);
      }
      const float fill = p.fill;
      auto filled = [&](int s) {
        const float v = raw(s);
        return bad(v) ? fill : v;
      };
      if (sigma > 0.f) {
        const Moments a = nan_moments(N, filled, red);
        const float lo1 = a.mean_clip - a.std * sigma, hi1 = a.mean_clip + a.std * sigma;
        auto cleaned = [&](int s) {
          const float v = filled(s);
          return (v > hi1 || v < lo1) ? NAN : v;
        };
        const Moments b = nan_moments(N, cleaned, red);
        p.lo = b.mean_clip - b.std * sigma;
        p.hi = b.mean_clip + b.std * sigma;
      }
      const float lo = p.lo, hi = p.hi;
      const bool clipping = sigma > 0.f;
      auto clipped = [&](int s) {
        const float v = filled(s);
        return clipping ? soft_clip_t(v, lo, hi) : v;
      };
      const Moments nm = nan_moments(N, clipped, red);
      p.mean = nm.mean_clip;
      p.sd = (S == 1 || N == 1) ? 1.0f : nm.std + 1e-20f;
      // used-feature test on the normalised values over all rows
      const float mean = p.mean, sd = p.sd;
      auto normed = [&](int s) { return tmin(tmax((clipped(s) - mean) / sd, -100.f), 100.f); };
      const float u0 = normed(0);
      int eq = 0;
      for (int s = 1 + threadIdx.x; s < S; s += blockDim.x) eq += (normed(s) == u0);
      const double tot = block_sum_d((double)eq, red);
      p.scale = (int)(tot + 0.5) != S - 1 ? 1.f : 0.f;  // used flag; the embed kernel rescales
    } else {
      p.scale = 0.f;
    }
    if (threadIdx.x == 0) slots[g * fpg + k] = p;
  }
  (void)s_cnt;
}

// EMB_TOK tokens per block: the per-token model inputs (u, NaN/inf indicators) are computed
// once per (token, slot) into LDS next to the encoder weights; then each thread writes 16-B
// pieces of the embedding (4 columns of one token, consecutive threads -> consecutive columns),
// adding the token's group positional row straight from global memory (one 768-B row per group,
// cache resident).  16 tokens per block (64 measured 31 vs 33 us alone but 53 vs 46 us beside the
// other lane's kernels in the bench: small blocks share the CUs better).
constexpr int EMB_TOK = 16;
constexpr int EMB_EMAX = 256;
__global__ __launch_bounds__(256) void enc_x_embed_kernel(const float* __restrict__ x, int S, int F, int G, int fpg,
                                                          int nf, const SlotParams* __restrict__ slots,
                                                          const float* __restrict__ w, const float* __restrict__ pe,
                                                          float* __restrict__ X, int E, int* flag) {
  __shared__ float su[EMB_TOK][8], si[EMB_TOK][8];
  __shared__ float ws[EMB_EMAX * 16];
  const int tid = threadIdx.x, nin = 2 * nf;
  const int64_t ntok = (int64_t)S * G, tok0 = (int64_t)blockIdx.x * EMB_TOK;
  for (int i = tid; i < E * nin; i += blockDim.x) ws[i] = w[i];
  for (int it = tid; it < EMB_TOK * 8; it += blockDim.x) {
    const int i = it >> 3, k = it & 7;
    const int64_t tok = tok0 + i;
    float u = 0.f, ind = 0.f;
    if (tok < ntok && k < fpg) {
      const int g = (int)tok / S, s = (int)tok - g * S;
      const SlotParams p = slots[g * fpg + k];
      float used = 0.f;  // used-feature rescale sqrt(nf / used) of the group (encoders.py:608-655)
      for (int j = 0; j < fpg; ++j) used += slots[g * fpg + j].scale;
      const float scale = sqrtf((float)nf / fmaxf(used, 1.f));
      if (p.src >= 0) {
        const float raw = x[(int64_t)s * F + p.src];
        ind = isnan(raw) ? -2.0f : (isinf(raw) ? (raw > 0 ? 2.0f : 4.0f) : 0.0f);
        float v = bad(raw) ? p.fill : raw;
        v = soft_clip_t(v, p.lo, p.hi);
        v = tmin(tmax((v - p.mean) / p.sd, -100.f), 100.f);
        u = v * scale;
      }
    }
    su[i][k] = u, si[i][k] = ind;
  }
  __syncthreads();
  const int E4 = E / 4;
  bool nan_seen = false;
  for (int item = tid; item < EMB_TOK * E4; item += blockDim.x) {
    const int i = item / E4, e4 = item - i * E4;
    const int64_t tok = tok0 + i;
    if (tok >= ntok) break;
    const f32x4 pv = *(const f32x4*)(pe + (int)((int)tok / S) * E + e4 * 4);  // S * G < 2^31 (launcher)
    f32x4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int e = e4 * 4 + c;
      const float* wr = ws + e * nin;
      float a = 0.f;
      for (int k = 0; k < nf; ++k) a = fmaf(su[i][k], wr[k], a);
      for (int k = 0; k < nf; ++k) a = fmaf(si[i][k], wr[nf + k], a);
      a += pv[c];
      o[c] = a;
      nan_seen |= isnan(a);
    }
    *(f32x4*)(X + tok * E + e4 * 4) = o;
  }
  if (nan_seen) atomicOr(flag, 1);
}

__global__ void y_stats_kernel(const float* __restrict__ y, int N, float* out) {
  __shared__ double red[16];
  double sum = 0.0, cnt = 0.0;
  for (int s = threadIdx.x; s < N; s += blockDim.x) {
    const float v = y[s];
    if (!isnan(v)) {
      sum += v;
      cnt += 1.0;
    }
  }
  sum = block_sum_d(sum, red);
  cnt = block_sum_d(cnt, red + 4);
  if (threadIdx.x == 0) out[0] = (float)(sum / cnt);
}

__global__ __launch_bounds__(256) void enc_y_embed_kernel(const float* __restrict__ y, int N, int S,
                                                          const float* __restrict__ uniq, int U,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          const float* __restrict__ ymean, float* __restrict__ Xy,
                                                          int E, int* flag) {
  const int E4 = E / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)S * E4) return;
  const int e4 = idx % E4;
  const int s = idx / E4;
  float yv = s < N ? y[s] : NAN;
  const float ind = isnan(yv) ? -2.0f : 0.0f;
  if (isnan(yv)) yv = ymean[0];
  float yc = 0.f;
  for (int i = 0; i < U; ++i) yc += (yv > uniq[i]) ? 1.f : 0.f;
  f32x4 o;
  bool nan_seen = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = e4 * 4 + i;
    const float a = fmaf(ind, w[e * 2 + 1], yc * w[e * 2]) + b[e];
    o[i] = a;
    nan_seen |= isnan(a);
  }
  *(f32x4*)(Xy + (int64_t)s * E + e4 * 4) = o;
  if (nan_seen) atomicOr(flag, 2);
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

__global__ __launch_bounds__(256) void add_tokens_kernel(const float* __restrict__ tok, int S, int C,
                                                         const float* __restrict__ pe, float* __restrict__ X, int E,
                                                         int* flag) {
  const int E4 = E / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)S * C * E4) return;
  const int e4 = idx % E4;
  const int64_t r = idx / E4;  // r = c*S + s  (output order)
  const int s = r % S, c = r / S;
  f32x4 v = *(const f32x4*)(tok + ((int64_t)s * C + c) * E + e4 * 4);
  const f32x4 p = *(const f32x4*)(pe + (int64_t)c * E + e4 * 4);
  v += p;
  *(f32x4*)(X + ((int64_t)c * S + s) * E + e4 * 4) = v;
  if (isnan(v[0]) || isnan(v[1]) || isnan(v[2]) || isnan(v[3])) atomicOr(flag, 1);
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

hipError_t launch_encode_x(const float* x, int S, int F, int N, int G, int fpg, int nf, float sigma,
                           SlotParams* slots, const float* w_enc, const float* posemb, float* X, int E, int* flag,
                           hipStream_t st, bool stats) {
  if (G <= 0) return hipSuccess;
  if (fpg > 8 || nf > 8 || nf < fpg) return hipErrorInvalidValue;
  if (stats) {
    const int col_lds = (size_t)S * sizeof(float) <= 48 * 1024 ? 1 : 0;  // stage the column when it fits
    hipLaunchKernelGGL(enc_x_stats_kernel, dim3(G, fpg), dim3(1024), col_lds ? (size_t)S * sizeof(float) : 0, st, x, S,
                       F, N, fpg, nf, sigma, slots, col_lds);
  }
  if (fpg > 8 || nf > 8 || E > EMB_EMAX || E % 4 != 0 || (int64_t)S * G >= INT32_MAX) return hipErrorInvalidValue;
  const int64_t nblk = ((int64_t)S * G + EMB_TOK - 1) / EMB_TOK;
  hipLaunchKernelGGL(enc_x_embed_kernel, dim3((unsigned)nblk), dim3(256), 0, st, x, S, F, G, fpg, nf, slots, w_enc,
                     posemb, X, E, flag);
  return hipGetLastError();
}

hipError_t launch_encode_y(const float* y_train, int N, int S, const float* uniq, int U, const float* w,
                           const float* b, float* Xy, int E, float* scratch, int* flag, hipStream_t st, bool stats) {
  if (stats) hipLaunchKernelGGL(y_stats_kernel, dim3(1), dim3(256), 0, st, y_train, N, scratch);
  const int64_t n = (int64_t)S * (E / 4);
  hipLaunchKernelGGL(enc_y_embed_kernel, dim3((n + 255) / 256), dim3(256), 0, st, y_train, N, S, uniq, U, w, b,
                     scratch, Xy, E, flag);
  return hipGetLastError();
}

hipError_t launch_pos_emb(const float* rnd, int n, const float* w, const float* b, float* out, int E,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pos_emb_kernel, dim3((n * E + 255) / 256), dim3(256), 0, st, rnd, n, w, b, out, E);
  return hipGetLastError();
}

hipError_t launch_add_tokens(const float* tok, int S, int C, const float* posemb, float* X, int E, int* flag,
                             hipStream_t st) {
  if (C <= 0) return hipSuccess;
  const int64_t n = (int64_t)S * C * (E / 4);
  hipLaunchKernelGGL(add_tokens_kernel, dim3((n + 255) / 256), dim3(256), 0, st, tok, S, C, posemb, X, E, flag);
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
