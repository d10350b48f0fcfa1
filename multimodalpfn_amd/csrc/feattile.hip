// Tile-resident attention-between-features sublayer for gfx950, fp16 state (PREC_F16):
//   X <- LayerNorm(X + MHA_features(X))        (layer.py:332-339,437-455; multi_head_attention.py:547-736)
//
// One wave owns ONE 16-token tile of a table row (a row of T <= 16 NT tokens is NT waves of one block);
// a block holds R rows.  Against featrow.hip's one-wave-per-row form (the whole row's X^T fragments, every
// head's O^T fragments and the projection accumulators in one wave: 46 spilled VGPRs at T = 36, ~120 MB of
// scratch traffic per two-member launch) a wave keeps only its own tile:
//   xf[ks]     X^T fragments of its 16 tokens (lane (n, g): X[token n][32ks + 8g .. +7]), loaded once, also
//              the residual (the out-projection image's rows are in f16_row_perm order)
//   per head   Q^T / K^T tiles = W_{q,k} . X^T on featrow's permuted weight rows (lane: Q[token n][8g .. +7]),
//              V tile = X . Wv^T (lane: V[token 4g + i][d 16f + n]); its K fragment and V pieces go to LDS, and
//              after the next barrier its query tile attends to the row's NT key tiles read back from LDS -- in
//              exactly the lane layout their producer computed them (K: the A operand of S^T = K Q^T, V: the
//              halves of the A operand V^T of O^T = V^T P^T), so the exchange is lane-linear and conflict-free;
//              heads are software-pipelined (head h's attention beside head h+1's projections, one barrier per
//              head: a first form with two barriers per head ran 116.8 vs featrow's 100.4 us)
//   of[h]      the tile's O^T fragments of every head (6 x 4 VGPRs), out-projection after the last head
//   y[f]       Y^T = Wout . O^T for its 16 tokens (12 tiles), then residual + LayerNorm across the 4 lane groups
// ~150 VGPRs: three waves per SIMD with no spills.  Weights as in featrow.hip (the same LDS images, FR_ST-wide
// rows, by LDS-DMA): per head a 39 KB QKV image double-buffered, two heads ahead of its attention, the 78 KB
// out-projection image over both buffers at the end; K / V exchange double-buffered by head
// parity (4 NT KB per row).  MFMA work per row is featrow's; the lane arithmetic of every value is featrow's
// too, so the two kernels agree bitwise.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int FT_E = 192;
constexpr int FT_H = 6;
constexpr int FT_ST = FEAT_IMG_STRIDE;           // fp16 row stride of every weight image (416 B)
constexpr int FT_QKV_IMG = 96 * FT_ST;           // one head's QKV image (elements)
constexpr int FT_PIECES = FT_QKV_IMG * 2 / 1024; // 1-KB DMA pieces per QKV image (39)

__device__ __forceinline__ f16x8 cat8h(const f32x4& a, const f32x4& b, float s = 1.0f) {
  f16x8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = (_Float16)(a[i] * s), r[4 + i] = (_Float16)(b[i] * s);
  return r;
}
__device__ __forceinline__ f16x4 cvt4h(const f32x4& a) {
  f16x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = (_Float16)a[i];
  return r;
}

typedef __attribute__((address_space(3))) void lds_void;

// rows per block for NT tiles per row (NT R waves: 8 / 12 / 12 / 12)
template <int NT> struct FtRows;
template <> struct FtRows<1> { static constexpr int R = 8; };
template <> struct FtRows<2> { static constexpr int R = 6; };
template <> struct FtRows<3> { static constexpr int R = 4; };
template <> struct FtRows<4> { static constexpr int R = 3; };

template <int NT>
__global__ __launch_bounds__(64 * NT * FtRows<NT>::R, 1) void feat_tiles_kernel(f16* __restrict__ Xs,
                                                                               const f16* __restrict__ pack, int S,
                                                                               int T, int M, float eps) {
  constexpr int R = FtRows<NT>::R, NW = NT * R;
  constexpr int KVB = NT * 64 * 16;          // one row's exchange bytes per head: K (16 B / lane) + V (2 x 8 B / lane)
  constexpr int KVS = R * 2 * KVB;           // one head parity's exchange buffer (K and V of every row)
  __shared__ __attribute__((aligned(1024))) f16 wbuf[2 * FT_QKV_IMG];
  __shared__ __attribute__((aligned(16))) unsigned char kvx[2 * KVS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  const int rl = wave / NT, tt = wave - rl * NT;      // row inside the block, the wave's token tile
  const int row = blockIdx.x * R + rl;
  const bool rowok = row < M * S;                     // wave-uniform: a wave past the last row stores nothing
  const int rc = rowok ? row : M * S - 1;
  const int mem = rc / S, sr = rc - mem * S;
  const int64_t SE = (int64_t)S * FT_E;
  f16* __restrict__ X = Xs + (int64_t)mem * T * SE;

  // LDS-DMA of pieces [p0, p0 + count) of an image: 1-KB piece p by wave p % NW
  auto dma = [&](const f16* src, f16* dst, int pieces) {
    for (int p = wave; p < pieces; p += NW)
      __builtin_amdgcn_global_load_lds((const uint16_t*)src + p * 512 + lane * 8, (lds_void*)((uint16_t*)dst + p * 512),
                                       16, 0, 0);
  };
  dma(pack, wbuf, FT_PIECES);  // head 0 -> buffer 0 (head 1 -> buffer 1 after the first barrier)
  // ---- the tile's tokens (padding tokens t >= T are zero)
  const int t = 16 * tt + n;
  const bool pad = t >= T;
  f16x8 xf[FT_E / 32];
  {
    const f16* xr = X + (int64_t)(pad ? 0 : t) * SE + (int64_t)sr * FT_E + 8 * g;
#pragma unroll
    for (int ks = 0; ks < FT_E / 32; ++ks) {
      xf[ks] = *(const f16x8*)(xr + 32 * ks);
      if (pad) xf[ks] = f16x8{};
    }
  }
  __syncthreads();  // (its vmcnt(0) retires the DMA too)

  constexpr int NKP = (NT + 1) / 2;  // key-tile pairs (K = 32 keys per P.V MFMA)
  f16x8 of[FT_H];                    // the tile's O^T fragments of every head
  // ---- projections of head h (weights in wbuf[h & 1]): Q^T then K^T (C^T tiles) and V (C tile), K = 192 in
  //      6 steps; Q stays in registers, the K fragment and the V pieces go to the exchange buffer of parity h & 1
  auto project = [&](int h, f16x8& qf) __attribute__((always_inline)) {
    const f16* wq = wbuf + (h & 1) * FT_QKV_IMG;  // [96][FT_ST]: Q (permuted) | K (permuted) | V
    unsigned char* kx = kvx + (h & 1) * KVS + rl * 2 * KVB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 qa[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < FT_E / 32; ++ks)
#pragma unroll
        for (int f = 0; f < 2; ++f)
          qa[f] = mfma16x(*(const f16x8*)(wq + (32 * j + 16 * f + n) * FT_ST + 32 * ks + 8 * g), xf[ks], qa[f]);
      if (j == 0) qf = cat8h(qa[0], qa[1]);
      else *(f16x8*)(kx + tt * 1024 + lane * 16) = cat8h(qa[0], qa[1]);  // K fragment of key tile tt
    }
    f32x4 va[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < FT_E / 32; ++ks)
#pragma unroll
      for (int f = 0; f < 2; ++f)
        va[f] = mfma16x(xf[ks], *(const f16x8*)(wq + (64 + 16 * f + n) * FT_ST + 32 * ks + 8 * g), va[f]);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) *(f16x4*)(kx + KVB + (tt * 2 + mt) * 512 + lane * 8) = cvt4h(va[mt]);
  };
  // ---- attention of head h (exchange parity h & 1): S^T[key][query] = K Q^T (log2 units) over the row's key
  //      tiles, softmax over keys, O^T = V^T P^T
  auto attend = [&](int h, const f16x8& qf) __attribute__((always_inline)) {
    const unsigned char* kx = kvx + (h & 1) * KVS + rl * 2 * KVB;
    f32x4 st[NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
      st[kt] = mfma16x(*(const f16x8*)(kx + kt * 1024 + lane * 16), qf, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int i = 0; i < 4; ++i)  // only the last key tile holds padding keys (T > 16 (NT - 1))
      if (16 * (NT - 1) + 4 * g + i >= T) st[NT - 1][i] = -INFINITY;
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) m = fmaxf(m, st[kt][i]);
    m = max_rows4(m);
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __builtin_amdgcn_exp2f(st[kt][i] - m);
        st[kt][i] = e;
        sum += e;
      }
    const float inv = __builtin_amdgcn_rcpf(sum_rows4(sum));
    f32x4 oa[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kp = 0; kp < NKP; ++kp) {
      const f16x8 pb = cat8h(st[2 * kp], 2 * kp + 1 < NT ? st[2 * kp + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f16x4 v0 = *(const f16x4*)(kx + KVB + (2 * kp * 2 + mt) * 512 + lane * 8);
        const f16x4 v1 = 2 * kp + 1 < NT ? *(const f16x4*)(kx + KVB + ((2 * kp + 1) * 2 + mt) * 512 + lane * 8)
                                         : f16x4{};
        const f16x8 vfr = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        oa[mt] = mfma16x(vfr, pb, oa[mt]);
      }
    }
    of[h] = cat8h(oa[0], oa[1], inv);
  };
  // software pipeline over heads, ONE barrier per head: step h runs the attention of head h (its K / V
  // exchanged in step h-1) beside the projections of head h+1 (weights DMA'd during step h-1), and DMAs the
  // image two heads ahead into the weight buffer head h's projections used (step h-1); the barrier ending step h
  // publishes K / V(h+1), lands the next image and frees exchange parity h & 1 for head h+2.  The two work
  // streams of a step are independent, so one wave's projection MFMAs fill the other's softmax latency.
  f16x8 qcur, qnext;
  dma(pack + FT_QKV_IMG, wbuf + FT_QKV_IMG, FT_PIECES);  // head 1 -> buffer 1
  project(0, qcur);
  __syncthreads();  // K / V(0) visible; head 1's image landed
#pragma unroll
  for (int h = 0; h < FT_H; ++h) {
    // the image two heads ahead into buffer h & 1: head h+2's QKV, then the out-projection's halves
    if (h + 2 < FT_H) dma(pack + (h + 2) * FT_QKV_IMG, wbuf + (h & 1) * FT_QKV_IMG, FT_PIECES);
    else dma(pack + FT_H * FT_QKV_IMG + (h + 2 - FT_H) * FT_QKV_IMG, wbuf + (h & 1) * FT_QKV_IMG, FT_PIECES);
    if (h + 1 < FT_H) project(h + 1, qnext);
    attend(h, qcur);
    qcur = qnext;
    __syncthreads();
  }

  // ---- Y^T = Wout . O^T over K = 192 (K-step h = head h), image [192][FT_ST] rows in f16_row_perm order,
  //      then residual (the tile's own X fragments) + LayerNorm per token (lane = token n, 48 of its features)
  f32x4 y[FT_E / 16];
#pragma unroll
  for (int f = 0; f < FT_E / 16; ++f) {
    y[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < FT_H; ++h) y[f] = mfma16x(*(const f16x8*)(wbuf + (16 * f + n) * FT_ST + 32 * h + 8 * g), of[h], y[f]);
  }
  float sm = 0.f;
#pragma unroll
  for (int f = 0; f < FT_E / 16; ++f)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[f][i] += (float)xf[f >> 1][4 * (f & 1) + i];
      sm += y[f][i];
    }
  const float mean = sum_rows4(sm) * (1.0f / FT_E);
  float q = 0.f;
#pragma unroll
  for (int f = 0; f < FT_E / 16; ++f)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dl = y[f][i] - mean;
      q += dl * dl;
    }
  const float rs = 1.0f / sqrtf(sum_rows4(q) * (1.0f / FT_E) + eps);
  if (rowok && !pad) {
    f16* xr = X + (int64_t)t * SE + (int64_t)sr * FT_E + 8 * g;
#pragma unroll
    for (int k = 0; k < FT_E / 32; ++k) {  // features 32k + 8g .. +7 from tiles 2k, 2k+1: one 16-B store each
      f16x8 ov;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        ov[i] = (_Float16)((y[2 * k][i] - mean) * rs), ov[4 + i] = (_Float16)((y[2 * k + 1][i] - mean) * rs);
      *(f16x8*)(xr + 32 * k) = ov;
    }
  }
}

template <int NT>
hipError_t launch_ft(void* X, const void* pk, int S, int T, int M, float eps, hipStream_t st) {
  constexpr int R = FtRows<NT>::R;
  hipLaunchKernelGGL((feat_tiles_kernel<NT>), dim3((M * S + R - 1) / R), dim3(64 * NT * R), 0, st, (f16*)X,
                     (const f16*)pk, S, T, M, eps);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_feat_tiles(void* X, const void* pack, int S, int T, int M, int E, int H, float eps, hipStream_t st) {
  if (S <= 0 || M <= 0) return hipSuccess;
  if (E != FT_E || H != FT_H || T < 1 || T > 64) return hipErrorInvalidValue;
  if (T <= 16) return launch_ft<1>(X, pack, S, T, M, eps, st);
  if (T <= 32) return launch_ft<2>(X, pack, S, T, M, eps, st);
  if (T <= 48) return launch_ft<3>(X, pack, S, T, M, eps, st);
  return launch_ft<4>(X, pack, S, T, M, eps, st);
}

}  // namespace mmpfn
