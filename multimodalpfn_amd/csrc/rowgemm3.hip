// Row-resident projections of width 192 for the fp32 parity mode (split-bf16 "x3") on gfx950:
//   QKV    : rows of X (fp32) . W^T, W [N][192] (N = 576 q|k|v or 192 q), fp32 results scattered
//            into the attention layouts Q [b][h][pos][32], K [b][h][pos][32] (Npad rows) and
//            V^T [b][h][32][Npad]  (layer.py:341-372 item rows; :332-339 feature rows, b = table row)
//   RES_LN : X <- LayerNorm(X + O . Wout^T)  (layer.py:437-455, no affine), O fp32
// Every product is three bf16 MFMAs: hi = bf16(x), lo = bf16(x - hi) of both operands,
// acc += lo.hi + hi.lo + hi.hi (v_mfma_f32_16x16x32_bf16, fp32 accumulate; the W planes are split
// once on the host, capi.cpp upsplit; the rows are split in registers as they arrive).
//
// One 512-thread block per CU (two waves per SIMD).  The block stages one 192-feature panel of W --
// hi and lo planes, 2 x 192 rows of 384 B (XOR-swizzled: conflict-free ds_read_b128) = 144 KB of LDS, filled by LDS-DMA -- and keeps
// it while its waves project 32-row tiles: a wave holds its tile's rows as hi / lo fragments
// (96 VGPRs) and Y^T in 24 accumulators, while the SIMD's other wave loads
// or stores; there is no barrier inside a panel.  Blocks own contiguous ranges of
// the (row set, panel, tile) work list, so a block restages only where its range crosses a panel.
// Per 32-row tile and panel: 32 x 192 x 4 B read, 32 x 192 x 4 B written, 3 x 2 x 32 x 192^2 flop.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int P3E = 192;               // K and panel width
constexpr int P3PL = P3E * P3E;        // one LDS plane (elements): 192 rows of 384 B
constexpr int P3KS = P3E / 32;         // k-steps of 32
constexpr int P3LDS = 2 * P3PL * 2;    // bytes: hi + lo planes (147456)
constexpr int P3TILE = 32;             // rows per wave tile
constexpr int P3W = 8;                 // waves per block (two per SIMD)
constexpr int P3D = 3;                 // W fragment slots read ahead of their MFMAs

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct P3Set {
  const float* A;
  int a_rdiv, a_rmul, a_rmul2, a_roff;
  const bf16* W;  // hi plane; lo plane at W + w_lo
  int64_t w_lo;
  int M, npanel, tiles;
};

struct P3Args {
  P3Set set[2];
  int nset;
  int total;  // work items: sum over sets of npanel * tiles
  float *q, *k, *vt;
  int S, Npad, H;
  float* X;   // RES_LN
  float eps;
};

typedef __attribute__((address_space(3))) void lds_void;

// LDS image of a panel plane: 192 rows of 384 B, 16-B chunk c of row r at slot c ^ ((r >> 1) & 7)
// (conflict-free ds_read_b128 for the 16x16x32 operand fragments)
__device__ __forceinline__ int p3_slot(int r, int c) { return c ^ ((r >> 1) & 7); }

// W rows [0, 192) of a panel (hi plane at Wp, lo plane at Wp + w_lo) -> LDS by LDS-DMA (1 KB per
// wave-instruction, lane l of piece P fills slot P * 64 + l); the caller's barrier retires it
__device__ __forceinline__ void stage_panel3(const bf16* Wp, int64_t w_lo, bf16* wl, int wave, int lane) {
  constexpr int CH = P3E / 8;                 // 16-B chunks per row (24)
  constexpr int PIECES = 2 * P3E * CH / 64;   // 1-KB pieces of both planes (144)
#pragma unroll 1
  for (int pc = wave; pc < PIECES; pc += P3W) {
    const int q = pc * 64 + lane;             // slot over both planes
    const int pl = q / (P3E * CH), rq = q - pl * (P3E * CH);
    const int r = rq / CH, c = p3_slot(r, rq - r * CH);
    __builtin_amdgcn_global_load_lds(Wp + pl * w_lo + r * P3E + c * 8, (lds_void*)(wl + pc * 512), 16, 0, 0);
  }
}

// the tile's fp32 rows: lane (fr, fg) holds row 16 tt + fr, features 32 ks + 8 fg .. + 7
__device__ __forceinline__ void load_rows3(const P3Set& ps, int t, int fr, int fg, f32x4 (&raw)[2][P3KS][2]) {
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int m = min(t * P3TILE + tt * 16 + fr, ps.M - 1);
    const int b = m / ps.a_rdiv;
    const int64_t mr = (int64_t)b * ps.a_rmul + (int64_t)(m - b * ps.a_rdiv) * ps.a_rmul2 + ps.a_roff;
    const float* xr = ps.A + mr * P3E + fg * 8;
#pragma unroll
    for (int ks = 0; ks < P3KS; ++ks) {
      raw[tt][ks][0] = *(const f32x4*)(xr + ks * 32);
      raw[tt][ks][1] = *(const f32x4*)(xr + ks * 32 + 4);
    }
  }
}

__device__ __forceinline__ void split_rows3(const f32x4 (&raw)[2][P3KS][2], bf16x8 (&ah)[2][P3KS],
                                            bf16x8 (&al)[2][P3KS]) {
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int ks = 0; ks < P3KS; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x = raw[tt][ks][h][i];
          const bf16 hi = (bf16)x;
          ah[tt][ks][4 * h + i] = hi;
          al[tt][ks][4 * h + i] = (bf16)(x - (float)hi);
        }
}

// acc[f][tt] = Y^T over K = 192 (features x rows: lane = row 16 tt + fr, features 16 f + 4 fg + i),
// three products per k-step, in a fixed order of 72 "slots" of two W fragments: per k-step six lo-plane
// slots (features 2u, 2u + 1: lo.hi, 4 MFMAs) then six hi-plane slots (hi.lo then hi.hi, 8 MFMAs), so
// an accumulator's dependent MFMAs are >= 4 apart; the fragments of slot q + P3D are read while slot q
// computes (ring of P3D + 1 slots), and sched barriers keep that order.
__device__ __forceinline__ void mma3(const bf16* wl, const bf16x8 (&ah)[2][P3KS], const bf16x8 (&al)[2][P3KS],
                                     int fr, int fg, f32x4 (&acc)[P3E / 16][2]) {
  constexpr int NS = P3KS * 12, R = P3D + 1;
  // slot (4 ks + fg) ^ sw of row 16 x + fr, sw = (fr >> 1) & 7, is 4 ks + fg ^ (sw & 3) + (sw & 4) for
  // even ks and - (sw & 4) for odd ks: two lane bases per plane, the rest immediate offsets
  const int sw = (fr >> 1) & 7, lo3 = fg ^ (sw & 3);
  const bf16* bh[2] = {wl + fr * P3E + ((sw & 4) + lo3) * 8, wl + fr * P3E + (lo3 - (sw & 4)) * 8};
  const bf16* bl[2] = {bh[0] + P3PL, bh[1] + P3PL};
  bf16x8 wf[R][2];
#pragma unroll
  for (int q = 0; q < NS + P3D; ++q) {
    if (q < NS) {  // read slot q's fragments (P3D slots ahead of their use)
      const int ks = q / 12, u = q % 12, f0 = 2 * (u % 6);
      const bf16* base = (u < 6 ? bl : bh)[ks & 1] + f0 * 16 * P3E + ks * 32;
      wf[q % R][0] = *(const bf16x8*)base;
      wf[q % R][1] = *(const bf16x8*)(base + 16 * P3E);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int c = q - P3D;  // slot computed now
    if (c < 0) continue;
    const int ks = c / 12, u = c % 12, f0 = 2 * (u % 6);
    const bf16x8(&w)[2] = wf[c % R];
    if (u < 6) {
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc[f0 + e][tt] = mfma16(w[e], ah[tt][ks], acc[f0 + e][tt]);
    } else {
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc[f0 + e][tt] = mfma16(w[e], al[tt][ks], acc[f0 + e][tt]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc[f0 + e][tt] = mfma16(w[e], ah[tt][ks], acc[f0 + e][tt]);
    }
  }
}

// one panel's tiles [a, b) of a row set, wave w takes a + w, a + w + P3W, ...
template <bool RESLN>
__device__ __forceinline__ void run_tiles3(const P3Args& p, const P3Set& ps, int j, int a, int b, const bf16* wl,
                                           int wave, int fr, int fg) {
  for (int t = a + wave; t < b; t += P3W) {
    bf16x8 ah[2][P3KS], al[2][P3KS];
    {
      f32x4 raw[2][P3KS][2];
      load_rows3(ps, t, fr, fg, raw);
      split_rows3(raw, ah, al);
    }
    f32x4 acc[P3E / 16][2];
#pragma unroll
    for (int f = 0; f < P3E / 16; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    mma3(wl, ah, al, fr, fg, acc);

    if constexpr (RESLN) {
      // Y^T: lane = row 16 tt + fr, features 16 f + 4 fg + i; residual + LayerNorm per row
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int m = t * P3TILE + tt * 16 + fr;
        const bool valid = m < ps.M;
        float* xr = p.X + (int64_t)(valid ? m : ps.M - 1) * P3E + fg * 4;
        float s = 0.f;
#pragma unroll
        for (int f = 0; f < P3E / 16; ++f) {
          const f32x4 xv = *(const f32x4*)(xr + f * 16);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[f][tt][i] += xv[i];
            s += acc[f][tt][i];
          }
        }
        const float mean = sum_rows4(s) * (1.0f / P3E);
        float q = 0.f;
#pragma unroll
        for (int f = 0; f < P3E / 16; ++f)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float dl = acc[f][tt][i] - mean;
            q += dl * dl;
          }
        const float inv = 1.0f / sqrtf(sum_rows4(q) * (1.0f / P3E) + p.eps);
        if (valid) {
#pragma unroll
          for (int f = 0; f < P3E / 16; ++f) {
            f32x4 ov;
#pragma unroll
            for (int i = 0; i < 4; ++i) ov[i] = (acc[f][tt][i] - mean) * inv;
            *(f32x4*)(xr + f * 16) = ov;
          }
        }
      }
    } else {
      // lane = row 16 tt + fr (b = m / rdiv, pos = roff + m % rdiv); features 16 f + 4 fg + i are
      // head f / 2, dims (f % 2) 16 + 4 fg + i.  Q / K: one 16-B store per tile; V^T: four dword
      // stores, the 16 rows of a lane group contiguous (64-B runs) when they share b
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int m = t * P3TILE + tt * 16 + fr;
        if (m < ps.M) {
          const int bb = m / ps.a_rdiv, pos = ps.a_roff + (m - bb * ps.a_rdiv);
          if (j < 2) {
            const int64_t rows = j == 0 ? p.S : p.Npad;
            float* base = (j == 0 ? p.q : p.k) + ((int64_t)bb * p.H * rows + pos) * 32 + fg * 4;
#pragma unroll
            for (int f = 0; f < P3E / 16; ++f) *(f32x4*)(base + (f >> 1) * rows * 32 + (f & 1) * 16) = acc[f][tt];
          } else {
            float* base = p.vt + ((int64_t)bb * p.H * 32 + fg * 4) * p.Npad + pos;
#pragma unroll
            for (int f = 0; f < P3E / 16; ++f)
#pragma unroll
              for (int i = 0; i < 4; ++i) base[(int64_t)(f * 16 + i) * p.Npad] = acc[f][tt][i];
          }
        }
      }
    }
  }
}

template <bool RESLN>
__global__ __launch_bounds__(64 * P3W, 1) void proj3_kernel(const P3Args p) {
  extern __shared__ __attribute__((aligned(16))) bf16 wl3[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int G = gridDim.x;
  const int i0 = (int)((int64_t)p.total * blockIdx.x / G), i1 = (int)((int64_t)p.total * (blockIdx.x + 1) / G);
  int seg = 0;  // first work item of the current (set, panel)
#pragma unroll 1
  for (int s = 0; s < p.nset; ++s) {
    const P3Set ps = s == 0 ? p.set[0] : p.set[1];
    for (int j = 0; j < ps.npanel; ++j) {
      const int a = max(i0, seg), b = min(i1, seg + ps.tiles);
      if (a < b) {  // block-uniform
        __syncthreads();  // the previous panel's last reads
        stage_panel3(ps.W + (int64_t)j * P3E * P3E, ps.w_lo, wl3, wave, lane);
        __syncthreads();
        run_tiles3<RESLN>(p, ps, j, a - seg, b - seg, wl3, wave, fr, fg);
      }
      seg += ps.tiles;
    }
  }
}

int n_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

template <bool RESLN>
hipError_t launch_p3(const P3Args& a, hipStream_t st) {
  static std::atomic<uint64_t> opted{0};
  const hipError_t attr = lds_optin(opted, (const void*)proj3_kernel<RESLN>, P3LDS);
  if (attr != hipSuccess) return attr;
  const int grid = std::min(n_cus(), (a.total + P3W - 1) / P3W);
  hipLaunchKernelGGL(proj3_kernel<RESLN>, dim3(grid), dim3(64 * P3W), P3LDS, st, a);
  return hipGetLastError();
}

bool fill_set(const Proj3Set& s, P3Set& o) {
  if (s.M < 0 || (s.M > 0 && (!s.A || !s.W || s.w_lo <= 0 || s.a_rdiv <= 0))) return false;
  if (s.N != P3E && s.N != 3 * P3E) return false;
  if (s.a_rdiv > INT32_MAX || s.a_rmul > INT32_MAX || s.a_rmul2 > INT32_MAX || s.a_roff > INT32_MAX || s.a_rmul < 0 ||
      s.a_rmul2 < 0 || s.a_roff < 0)
    return false;
  o.A = s.A, o.a_rdiv = (int)s.a_rdiv, o.a_rmul = (int)s.a_rmul, o.a_rmul2 = (int)s.a_rmul2, o.a_roff = (int)s.a_roff;
  o.W = (const bf16*)s.W, o.w_lo = s.w_lo, o.M = s.M, o.npanel = s.N / P3E;
  o.tiles = (s.M + P3TILE - 1) / P3TILE;
  return true;
}

}  // namespace

hipError_t launch_proj3_qkv(const Proj3Set* sets, int nset, void* q, void* k, void* vt, int S, int Npad, int H,
                            hipStream_t st) {
  if (nset < 1 || nset > 2 || H * 32 != P3E) return hipErrorInvalidValue;
  P3Args a{};
  a.nset = nset, a.q = (float*)q, a.k = (float*)k, a.vt = (float*)vt, a.S = S, a.Npad = Npad, a.H = H;
  int64_t total = 0;
  for (int i = 0; i < nset; ++i) {
    if (!fill_set(sets[i], a.set[i])) return hipErrorInvalidValue;
    if (a.set[i].npanel == 3 && sets[i].M > 0 && (!k || !vt)) return hipErrorInvalidValue;
    total += (int64_t)a.set[i].npanel * a.set[i].tiles;
  }
  if (total == 0) return hipSuccess;
  if (total > INT32_MAX / 2) return hipErrorInvalidValue;
  a.total = (int)total;
  return launch_p3<false>(a, st);
}

hipError_t launch_proj3_resln(const float* O, const void* W, int64_t w_lo, int64_t M, float* X, float eps,
                              hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (M > INT32_MAX - P3TILE || !O || !W || !X || w_lo <= 0) return hipErrorInvalidValue;
  P3Args a{};
  Proj3Set s{O, 1, 1, 0, 0, W, w_lo, (int)M, P3E};
  if (!fill_set(s, a.set[0])) return hipErrorInvalidValue;
  a.nset = 1, a.total = a.set[0].tiles, a.X = X, a.eps = eps;
  return launch_p3<true>(a, st);
}

}  // namespace mmpfn
