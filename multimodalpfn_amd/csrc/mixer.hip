// Helper kernels of the modality projection heads (transformer.py:33-128):
// row LayerNorm (MGM/MoE input norm, CAP k_norm), the CAP cross-attention core,
// CAP's out_norm(o) + ffn(o) combine and the MoE gate.  The heavy contractions
// (per-head Linear(768,768)+GLU, Linear(384,E), CAP in/out projections, FFN,
// MoE experts) run on the MFMA GEMM in gemm.hip.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

// one wave per row; two-pass mean / biased variance (torch layer_norm)
template <typename TO>
__global__ __launch_bounds__(256) void ln_rows_kernel(const float* __restrict__ in, int64_t rows, int dim, float eps,
                                                      TO* __restrict__ out, const float* __restrict__ g,
                                                      const float* __restrict__ b) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* x = in + row * dim;
  float s = 0.f;
  for (int i = lane; i < dim; i += 64) s += x[i];
  const float mean = wave_sum(s) / dim;
  float q = 0.f;
  for (int i = lane; i < dim; i += 64) {
    const float d = x[i] - mean;
    q += d * d;
  }
  const float inv = 1.0f / sqrtf(wave_sum(q) / dim + eps);
  TO* o = out + row * dim;
  for (int i = lane; i < dim; i += 64) {
    float v = (x[i] - mean) * inv;
    if (g) v = v * g[i] + b[i];
    o[i] = from_f32<TO>(v);
  }
}

// CAP core: per row s, per head: softmax(q k^T / sqrt(hd)) v with q [cap][E] shared
// by all rows and k/v = kv[s][j][0:E] / kv[s][j][E:2E] (j < M).  One block per row.
template <typename TK>
__global__ __launch_bounds__(256) void cap_attn_kernel(const float* __restrict__ qp, const TK* __restrict__ kv,
                                                       float* __restrict__ out, int M, int cap, int E) {
  extern __shared__ float sc[];  // [cap][M] scores of the current head
  const int s = blockIdx.x;
  const int hd = E / cap;
  const float scale = 1.0f / sqrtf((float)hd);
  const TK* kvs = kv + (int64_t)s * M * 2 * E;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int h = 0; h < cap; ++h) {
    __syncthreads();
    for (int i = threadIdx.x; i < cap * M; i += blockDim.x) {
      const int c = i / M, j = i % M;
      const float* q = qp + c * E + h * hd;
      const TK* k = kvs + (int64_t)j * 2 * E + h * hd;
      float a = 0.f;
      for (int d = 0; d < hd; ++d) a = fmaf(q[d], to_f32(k[d]), a);
      sc[i] = a * scale;
    }
    __syncthreads();
    for (int c = wave; c < cap; c += 4) {
      float* row = sc + c * M;
      float mx = -INFINITY;
      for (int j = lane; j < M; j += 64) mx = fmaxf(mx, row[j]);
      mx = wave_max(mx);
      float sum = 0.f;
      for (int j = lane; j < M; j += 64) {
        const float e = expf(row[j] - mx);
        row[j] = e;
        sum += e;
      }
      sum = wave_sum(sum);
      const float inv = 1.0f / sum;
      for (int j = lane; j < M; j += 64) row[j] *= inv;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < cap * hd; i += blockDim.x) {
      const int c = i / hd, d = i % hd;
      const float* p = sc + c * M;
      const TK* v = kvs + E + h * hd + d;
      float a = 0.f;
      for (int j = 0; j < M; ++j) a = fmaf(p[j], to_f32(v[(int64_t)j * 2 * E]), a);
      out[((int64_t)s * cap + c) * E + h * hd + d] = a;
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
                                 const float* gamma, const float* beta, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  dim3 grid((rows + 3) / 4);
  if (out_f32)
    hipLaunchKernelGGL(ln_rows_kernel<float>, grid, dim3(256), 0, st, in, rows, dim, eps, (float*)out, gamma, beta);
  else
    hipLaunchKernelGGL(ln_rows_kernel<bf16>, grid, dim3(256), 0, st, in, rows, dim, eps, (bf16*)out, gamma, beta);
  return hipGetLastError();
}

hipError_t launch_cap_attention(const float* qp, const void* kv, bool kv_f32, float* out, int S, int M, int cap, int E,
                                hipStream_t st) {
  if (S <= 0) return hipSuccess;
  const size_t lds = (size_t)cap * M * sizeof(float);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  if (kv_f32)
    hipLaunchKernelGGL(cap_attn_kernel<float>, dim3(S), dim3(256), lds, st, qp, (const float*)kv, out, M, cap, E);
  else
    hipLaunchKernelGGL(cap_attn_kernel<bf16>, dim3(S), dim3(256), lds, st, qp, (const bf16*)kv, out, M, cap, E);
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
