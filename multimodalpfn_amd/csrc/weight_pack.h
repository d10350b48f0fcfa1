// Host-side weight packing of the bf16 layer kernels (no HIP): the permutations, scales and LDS
// images capi.cpp uploads in mmpfn_finalize_weights.  Header-only and free of HIP types so that
// the host sanitizer check (tests/native/host_check.cpp, g++ -fsanitize=address,undefined) builds
// exactly this code.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace mmpfn {

// featrow.hip: per head [96][FEAT_IMG_STRIDE] (Wq rows permuted & scaled by log2(e)/sqrt(32) | Wk rows
// permuted | Wv), then the out-projection [192][FEAT_IMG_STRIDE] with permuted head columns
constexpr int FEAT_IMG_STRIDE = 208;
constexpr int FEAT_PACK_LAYER = (6 * 96 + 192) * FEAT_IMG_STRIDE;

inline uint16_t f2bf(float f) {  // round-to-nearest-even, NaN preserving
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffff) > 0x7f800000) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

// IEEE binary16, round-to-nearest-even (overflow -> inf, NaN preserved, subnormals kept)
inline uint16_t f2h(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u, a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((a >> 13) & 0x3ffu));  // NaN
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to >= 65520: inf
  if (a < 0x38800000u) {  // below the smallest normal half (2^-14): subnormal or zero
    if (a < 0x33000000u) return (uint16_t)sign;  // < 2^-25: rounds to 0
    const uint32_t m = (a & 0x7fffffu) | 0x800000u;
    const int shift = 126 - (int)(a >> 23);  // 14..24 -> value = m >> shift (in units of 2^-24)
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (r & 1))) ++r;
    return (uint16_t)(sign | r);
  }
  uint32_t r = ((a - 0x38000000u) >> 13);  // rebias 127 -> 15
  const uint32_t rem = a & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1))) ++r;
  return (uint16_t)(sign | r);
}

// w_out [H][d][E] -> W[e][h*d+dd]
inline std::vector<float> transpose_out(const std::vector<float>& w, int HD, int E) {
  std::vector<float> o((size_t)E * HD);
  for (int i = 0; i < HD; ++i)
    for (int e = 0; e < E; ++e) o[(size_t)e * HD + i] = w[(size_t)i * E + e];
  return o;
}

// W2 [E][Fh] with each 32-wide hidden group permuted for mlp_rows_kernel's K order:
// position 8g + j holds hidden 4g + j (j < 4) or 16 + 4g + (j - 4) (j >= 4)
inline std::vector<float> pack_mlp2_perm(const std::vector<float>& w, int E, int Fh) {
  std::vector<float> o(w.size());
  for (int e = 0; e < E; ++e)
    for (int c = 0; c < Fh; c += 32)
      for (int pos = 0; pos < 32; ++pos) {
        const int g = pos >> 3, j = pos & 7;
        const int hid = j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
        o[(size_t)e * Fh + c + pos] = w[(size_t)e * Fh + c + hid];
      }
  return o;
}

// PREC_F16 row layout of a 192-wide output accumulated as Y^T 16x16 tiles: tile f row 4g+i holds
// feature 32(f>>1) + 8g + 4(f&1) + i, so a lane's 48 features are its 6 runs of 8 (16-B fp16 pieces)
inline int f16_row_perm(int r) {
  const int f = r >> 4, rho = r & 15;
  return 32 * (f >> 1) + 8 * (rho >> 2) + 4 * (f & 1) + (rho & 3);
}
// rows of W [E][K] permuted by f16_row_perm (image row r <- W row f16_row_perm(r))
inline std::vector<float> permute_rows_f16(const std::vector<float>& w, int E, int K) {
  std::vector<float> o(w.size());
  for (int r = 0; r < E; ++r) std::memcpy(&o[(size_t)r * K], &w[(size_t)f16_row_perm(r) * K], K * sizeof(float));
  return o;
}

// W1 [Fh][E] with the K (feature) order of mlp_rows_kernel's X fragments: K position
// 32ks + 8g + j holds feature 32ks + 16(j/4) + 4g + (j%4) (the Y^T lane layout, E = 192)
inline std::vector<float> pack_mlp1_perm(const std::vector<float>& w, int E, int Fh) {
  std::vector<float> o(w.size());
  for (int h = 0; h < Fh; ++h)
    for (int k = 0; k < E; ++k) {
      const int ks = k / 32, g = (k % 32) / 8, j = k % 8;
      o[(size_t)h * E + k] = w[(size_t)h * E + 32 * ks + 16 * (j / 4) + 4 * g + (j % 4)];
    }
  return o;
}

// featrow.hip weight pack (FEAT_PACK_LAYER floats, LDS images with FEAT_IMG_STRIDE-wide rows,
// the 16 pad columns zero):
//   per head h, rows [0,32) : Wq row 8(rho>>2) + 4f + (rho&3) for image row 16f + rho, scaled by
//                             log2(e)/sqrt(32) (the feature-attention softmax scale, exp2 domain)
//               rows [32,64): Wk, same row permutation;   rows [64,96): Wv in natural order
//   then [192] rows of the out-projection: Wout[e][32h + perm(c)] at column 32h + c,
//        perm(8g+j) = j<4 ? 4g+j : 16+4g+(j-4)
// qkv: w_qkv [3][H][32][E] (multi_head_attention.py:423-430); wout_t: [E][H*32].  H = 6, E = 192
// (the kernel's and FEAT_PACK_LAYER's shape; the caller checks).
// res_perm (PREC_F16): the out-projection rows in f16_row_perm order, so the Y^T tiles hold the
// features of the lane's X fragments (the residual is added from registers)
inline std::vector<float> pack_feat_rows(const std::vector<float>& qkv, const std::vector<float>& wout_t, int H,
                                         int E, bool res_perm = false) {
  const float c = 1.4426950408889634f / std::sqrt(32.0f);
  const int ST = FEAT_IMG_STRIDE;
  std::vector<float> o((size_t)FEAT_PACK_LAYER, 0.0f);
  for (int h = 0; h < H; ++h) {
    float* ph = o.data() + (size_t)h * 96 * ST;
    for (int r = 0; r < 96; ++r) {
      const int j = r / 32, rr = r % 32, f = rr >> 4, rho = rr & 15;
      const int dd = j < 2 ? 8 * (rho >> 2) + 4 * f + (rho & 3) : rr;
      const float sc = j == 0 ? c : 1.0f;
      const float* src = qkv.data() + ((size_t)(j * H + h) * 32 + dd) * E;
      for (int k = 0; k < E; ++k) ph[(size_t)r * ST + k] = src[k] * sc;
    }
  }
  float* po = o.data() + (size_t)H * 96 * ST;
  for (int e = 0; e < E; ++e) {
    const int src = res_perm ? f16_row_perm(e) : e;
    for (int h = 0; h < H; ++h)
      for (int cc = 0; cc < 32; ++cc) {
        const int g = cc >> 3, jj = cc & 7;
        const int dd = jj < 4 ? 4 * g + jj : 16 + 4 * g + (jj - 4);
        po[(size_t)e * ST + 32 * h + cc] = wout_t[(size_t)src * H * 32 + h * 32 + dd];
      }
  }
  return o;
}

// fold a preceding LayerNorm affine (g, b over K inputs) into Linear (W [N][K], c [N])
inline void fold_ln(std::vector<float>& W, std::vector<float>& c, const float* g, const float* b, int N, int K) {
  for (int n = 0; n < N; ++n) {
    double acc = c[n];
    for (int k = 0; k < K; ++k) {
      acc += (double)W[(size_t)n * K + k] * b[k];
      W[(size_t)n * K + k] *= g[k];
    }
    c[n] = (float)acc;
  }
}

}  // namespace mmpfn
