// Kernels of the modality encoders: the DINOv2 ViT image tower that produces the
// reference's image embeddings (datasets/pad_ufes_20.py:66-107, petfinder.py:100-146:
// vit_base(patch 14).forward_features(x)["x_norm_clstoken"]) and the ELECTRA text tower
// (petfinder.py:150-181: ElectraModel(...).last_hidden_state[:, 0]).  Both are plain
// transformer encoders with head_dim 64; the hot work is five GEMMs per layer and a d = 64
// softmax attention, so this file holds:
//   * gemm_tile_kernel<EPI, ACT>: bf16 C = A . W^T on 256 x 256 tiles (8 waves, 16x16x32 MFMAs)
//     fed by a 4-stage LDS-DMA ring, XCD-ordered, with the epilogues the towers need
//     (bf16 store + bias [+ GELU]; fp32 residual X += gamma * (acc + bias); fp32 store);
//   * attn64_kernel: bf16 flash attention, head_dim 64, S^T = K Q^T with the query on the lane,
//     lazily rescaled running max, row sums on the MFMA pipe (0/1 selector), optional per-key
//     additive mask; attn64_f32_kernel: the fp32 parity-mode counterpart (VALU, one query per
//     thread);
//   * LayerNorm (fp32 in, fp32 and/or bf16 out), im2col of the patch embedding, the bicubic
//     positional-embedding resampling of interpolate_pos_encoding, token assembly, the text
//     embedding sum + LayerNorm, and small residual / gather / cast helpers.
#include "common.h"
#include "modality.h"

namespace mmpfn {

namespace {

// ---------------------------------------------------------------- big-tile GEMM (bf16)
constexpr int TM = 256, TN = 256, TK = 32;
constexpr int TROW = TK * 2;                    // 64-B LDS rows
constexpr int TSTAGE = (TM + TN) * TROW;        // 32 KB per ring stage
#ifndef GT_NST
#define GT_NST 4  // 5 (all 160 KB of LDS): ViT batch 20.52-20.55 vs 20.21 ms, profiles/r04/modality/ab_gemm_tile_variants.txt
#endif
constexpr int TNST = GT_NST;                    // ring stages (4 x 32 KB: two slices in flight)
constexpr int TDMA = (TM + TN) * (TROW / 16) / 512;  // 16-B DMA pieces per thread and slice (4)
constexpr int TMT = TM / 32;                    // 16-row MFMA tiles per wave (8)
constexpr int OST16 = TN + 8;                   // bf16 output staging row stride (elements)
constexpr int OST32 = TN + 4;                   // fp32 output staging row stride (floats), 128 rows per pass
constexpr int imax3(int a, int b, int c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }
constexpr int GT_LDS = imax3(TNST * TSTAGE, TM * OST16 * 2, (TM / 2) * OST32 * 4);

#ifndef GT_GM
#define GT_GM 4  // super-tile (M tiles x N tiles) of the block order
#endif
#ifndef GT_GN
#define GT_GN 8
#endif

__device__ __forceinline__ int gt_slot(int r, int c) { return c ^ ((r >> 1) & 3); }

// "m0" in the clobber list: clang keeps m0 reserved and ignores the entry (-Winline-asm; the ISA is identical with
// and without it), and every m0 use the compiler emits itself is preceded by its own write -- test_codegen checks
// that no m0 read other than these DMA issues exists in the kernels
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void gt_dma16(const void* src, unsigned lds_base) {
  // m0 = the wave's LDS destination; lane i's 16 B land at m0 + 16 i
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_base) : "memory", "m0");
}
#pragma clang diagnostic pop

// C = A[M][K] . W[N][K]^T, 256 x 256 tile per 512-thread block (8 waves as 2 x 4, each 128 x 64 =
// 8 x 4 MFMA-16 tiles).  K moves in 32-wide slices through a 4-stage LDS ring filled by LDS-DMA
// (slice kt+1..kt+3 in flight while kt computes, one barrier per slice); LDS rows are unpadded 64 B
// with 16-B chunk c of row r at slot c ^ ((r >> 1) & 3) (conflict-free ds_read_b128).  Blocks are
// ordered so one XCD runs all M tiles of a W tile back to back (W tile fetched ~once per L2).
template <int EPI, int ACT>
__global__ __launch_bounds__(512, 1) void gemm_tile_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ gamma, void* __restrict__ C,
                                                           int64_t ldc, int M, int N, int K, int mtiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  // Tile order: XCD x (= block % 8) runs a contiguous task range; tasks walk super-tiles of
  // GT_GM M tiles x GT_GN N tiles (N-chunk outer, M-chunk inner, N fastest inside), so the ~32
  // blocks an XCD runs at once share ~GT_GM A panels and ~GT_GN W panels through its L2 (a W-major
  // order would stream every A panel once per N tile).
  int mt, nt;
  {
    const int nb = gridDim.x, ntiles = nb / mtiles;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int per = nb >> 3, extra = nb & 7;
    const int t = xcd * per + min(xcd, extra) + slot;
    const int gn = min(GT_GN, ntiles);
    const int c = min(t / (mtiles * gn), (ntiles - 1) / gn);  // N chunk
    const int w = min(gn, ntiles - c * gn);                     // its width
    const int r = t - c * mtiles * gn;
    const int sidx = r / (GT_GM * w), u = r - sidx * GT_GM * w;
    mt = sidx * GT_GM + u / w;
    nt = c * gn + u % w;
  }
  const int m0 = mt * TM, n0 = nt * TN;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)smem;

  const bf16* src[TDMA];
#pragma unroll
  for (int j = 0; j < TDMA; ++j) {
    const int q = (wave * TDMA + j) * 64 + lane, r = q >> 2, c = gt_slot(r, q & 3);
    src[j] = r < TM ? A + (int64_t)min(m0 + r, M - 1) * K + c * 8 : W + (int64_t)(n0 + r - TM) * K + c * 8;
  }
  auto dma = [&](int kt) {
    const unsigned base = lds0 + (kt % TNST) * TSTAGE + wave * TDMA * 1024;
#pragma unroll
    for (int j = 0; j < TDMA; ++j) gt_dma16(src[j] + kt * TK, __builtin_amdgcn_readfirstlane(base + j * 1024));
  };
  f32x4 acc[TMT][4];
#pragma unroll
  for (int a = 0; a < TMT; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Ping-pong schedule (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_programming.md's 256^2
  // template): the two waves of a SIMD (wm = 0 / 1) run one phase apart, so in every phase one of
  // them issues its MFMAs on a slice's fragments while the other reads the next slice's fragments
  // from LDS.  Phase p: wave group g works on group phase q = p - g: even q reads slice q/2 into
  // registers, odd q computes slice (q-1)/2.  Every wave takes part in every barrier (one per phase).
  // DMA: slice s >= TNST is issued in phase 2(s - TNST) + 2 (its stage was last read, by group 1, in
  // phase 2(s - TNST) + 1); each wave waits for its own pieces of slice j before the barrier that
  // ends phase 2j - 1, so slice j is complete and visible when group 0 reads it in phase 2j.
  const int nk = K / TK;
#pragma unroll
  for (int i = 0; i < TNST; ++i)
    if (i < nk) dma(i);
  {  // slice 0 visible before phase 0
    const int c = min(nk - 1, TNST - 1);
    if (c >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * TDMA) : "memory");
    else if (c == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * TDMA) : "memory");
    else if (c == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * TDMA) : "memory");
    else if (c == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  bf16x8 af[TMT], bw[4];
  auto read = [&](int j) {
    const unsigned char* As = smem + (j % TNST) * TSTAGE;
    const unsigned char* Ws = As + TM * TROW;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rb = wn * 64 + i * 16 + fr;
      bw[i] = *(const bf16x8*)(Ws + rb * TROW + 16 * gt_slot(rb, fg));
    }
#pragma unroll
    for (int i = 0; i < TMT; ++i) {
      const int ra = wm * (TM / 2) + i * 16 + fr;
      af[i] = *(const bf16x8*)(As + ra * TROW + 16 * gt_slot(ra, fg));
    }
  };
  auto compute = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < TMT; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bw[b], acc[a][b], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto issue = [&](int p) {  // even phase p >= 2 issues slice p/2 - 1 + TNST
    const int sidx = (p >> 1) - 1 + TNST;
    if (p >= 2 && sidx < nk) dma(sidx);
  };
  auto wait_for = [&](int j) {  // end of phase 2j - 1: own pieces of slice j landed
    if (j >= nk) return;
    const int c = min(nk - 1, j + TNST - 2) - j;
    if (c >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * TDMA) : "memory");
    else if (c == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * TDMA) : "memory");
    else if (c == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  if (wm == 0) {  // phases 2j: read j | 2j+1: compute j | 2nk: idle
    for (int j = 0; j < nk; ++j) {
      read(j);
      issue(2 * j);
      __syncthreads();
      compute();
      wait_for(j + 1);
      __syncthreads();
    }
    __syncthreads();
  } else {  // phase 0: idle | 2j+1: read j | 2j+2: compute j
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
      read(j);
      wait_for(j + 1);
      __syncthreads();
      compute();
      issue(2 * j + 2);
      __syncthreads();
    }
  }
  __syncthreads();  // the ring is reused for the output tile

  if constexpr (EPI == GT_BF16) {
    // C tile lane layout: row 16a + 4fg + r (of the wave's 128), column 16b + fr (of its 64)
    bf16* Ct = (bf16*)smem;  // [TM][OST16]
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int col = wn * 64 + b * 16 + fr;
      const float bv = bias ? bias[n0 + col] : 0.f;
#pragma unroll
      for (int a = 0; a < TMT; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[a][b][r] + bv;
          // bf16 output: the tanh form (|err| <= 3e-4, below the bf16 rounding of the stored value) at 7 VALU
          // ops + 2 transcendentals, where the erf form took ~15 + 2 in this epilogue (no MFMA to hide behind);
          // the fp32 mode's GEMM keeps the exact erf GELU
          if constexpr (ACT == 1) v = gelu_tanh_fast(v);
          Ct[(wm * (TM / 2) + a * 16 + fg * 4 + r) * OST16 + col] = (bf16)v;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM * (TN / 8) / 512; ++i) {  // TM rows x 32 chunks of 16 B
      const int u = tid + 512 * i, r = u >> 5, ch = u & 31;
      if (m0 + r < M)
        *(u32x4*)((bf16*)C + (int64_t)(m0 + r) * ldc + n0 + ch * 8) = *(const u32x4*)(Ct + r * OST16 + ch * 8);
    }
  } else {
    // fp32 epilogues in two passes of 128 rows (the half tile of the waves with wm == pass)
    float* Cs = (float*)smem;  // [128][OST32]
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (pass) __syncthreads();
      if (wm == pass) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int col = wn * 64 + b * 16 + fr;
          const float bv = bias ? bias[n0 + col] : 0.f;
#pragma unroll
          for (int a = 0; a < TMT; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) Cs[(a * 16 + fg * 4 + r) * OST32 + col] = acc[a][b][r] + bv;
        }
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < (TM / 2) * (TN / 4) / 512; ++i) {  // 128 rows x 64 float4
        const int u = tid + 512 * i, r = u >> 6, c4 = u & 63;
        const int64_t row = m0 + pass * (TM / 2) + r;
        if (row < M) {
          const f32x4 v = *(const f32x4*)(Cs + r * OST32 + 4 * c4);
          float* dst = (float*)C + row * ldc + n0 + 4 * c4;
          if constexpr (EPI == GT_RESID) {
            const f32x4 g = gamma ? *(const f32x4*)(gamma + n0 + 4 * c4) : f32x4{1.f, 1.f, 1.f, 1.f};
            f32x4 x = *(const f32x4*)dst;
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = fmaf(g[e], v[e], x[e]);
            *(f32x4*)dst = x;
          } else {
            *(f32x4*)dst = v;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- attention, head_dim 64 (bf16)
// QKV rows (b * L + t) hold [q(H x 64) | k(H x 64) | v(H x 64)] in bf16 (the QKV GEMM output).
// Block = 4 waves x 32 queries of one (b, h); each 64-key K tile and V^T tile is staged once in
// LDS for the 4 waves (XOR-swizzled 128-B rows).  Per tile and wave: S^T = K Q^T on 8
// v_mfma_f32_32x32x16_bf16 (query on the lane: row statistics need one permlane32 swap), the
// chain starting from the accumulator -m (the running max), p = exp2(s - m) with Q pre-scaled
// by log2(e)/8, O^T += V^T P^T on 8 more, the row sums on 4 v_mfma_f32_16x16x32_bf16 through a
// 0/1 selector.  The max is raised lazily: only when some lane's tile max exceeds the current
// reference by A64_TAU (log2 units) are O and l rescaled -- p <= 2^A64_TAU otherwise, exact in
// fp32.  V^T image: row d, keys of each 16-key group in the order of the P fragment a lane
// builds from its S^T accumulators (position 8hh + j <-> key (j & 3) + 8 (j >> 2) + 4 hh).
constexpr int A64_KT = 64;
constexpr float A64_TAU = 8.0f;
constexpr int A64_STAGE = 2 * 8192 + 256;  // K [64][128 B] | V^T [64][128 B] | key bias [64] f32

__device__ __forceinline__ int a64_off(int row, int c) { return row * 128 + 16 * (c ^ ((row >> 1) & 7)); }
// V image: natural [key][d] rows (128 B, 16-B chunk c of row k at c ^ 4 ((k >> 1) & 1)), written with one
// ds_write_b128 per 8 d's and read transposed by ds_read_b64_tr_b16 (a 4-key x 16-d block per 16 lanes,
// MI355X / cdna_hip_programming.md T10): the swizzle makes the four key rows of a read land on four
// different 16-dword bank ranges, so each 32-lane half is conflict-free
__device__ __forceinline__ int a64v_off(int key, int c) { return key * 128 + 16 * (c ^ (((key >> 1) & 1) << 2)); }
typedef short a64_s4 __attribute__((ext_vector_type(4)));

// NCH query chains of 32 per wave (block = 4 waves x 32 NCH queries): with two, one chain's exps issue
// beside the other chain's MFMAs inside one basic block (the per-chain lazy rescales are decided before it)
#ifndef A64_NCH
#define A64_NCH 2
#endif
template <int NCH>
__global__ __launch_bounds__(256, 2) void attn64_kernel(const bf16* __restrict__ qkv, const float* __restrict__ kbias,
                                                        bf16* __restrict__ out, int L, int H, int q0, int nq,
                                                        int64_t o_bstride, int chunks, int nblocks) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2][A64_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int D = H * 64;
  const int64_t ld = 3 * (int64_t)D;
  int b, h, chunk;
  {  // XCD-contiguous task ranges: the blocks of one (b, h) share an L2
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int task = xcd * (nblocks >> 3) + min(xcd, nblocks & 7) + slot;
    chunk = task % chunks;
    const int bh = task / chunks;
    h = bh % H, b = bh / H;
  }
  const int qw = chunk * (128 * NCH) + wave * (32 * NCH);  // first query (relative to q0) of this wave
  const bool active = qw < nq;                             // wave-uniform
  const bf16* base = qkv + (int64_t)b * L * ld;
  const float c = kLog2e * 0.125f;  // log2(e) / sqrt(64)
  int qi[NCH];
  bf16x8 qf[NCH][4];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    qi[ch] = qw + 32 * ch + r;
    const int qt = q0 + min(qi[ch], nq - 1);
    const bf16* qrow = base + (int64_t)qt * ld + h * 64;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 raw = *(const bf16x8*)(qrow + 16 * ks + 8 * hh);
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[ch][ks][e] = (bf16)((float)raw[e] * c);
    }
  }
  const float* kb = kbias ? kbias + (int64_t)b * L : nullptr;

  // staging: 2 x (one 16-B K chunk + one 16-B V chunk) per thread and tile
  u32x4 rk[2], rv[2];
  float rb = 0.f;
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cidx = tid + 256 * i, key = cidx >> 3, ch = cidx & 7;
      const int kk = k0 + key;
      const bf16* row = base + (int64_t)min(kk, L - 1) * ld + h * 64 + ch * 8;
      rk[i] = *(const u32x4*)(row + D);
      rv[i] = kk < L ? *(const u32x4*)(row + 2 * D) : u32x4{0u, 0u, 0u, 0u};  // V = 0 past L: p = 0 meets no NaN
    }
    if (tid < 64) {
      const int kk = k0 + tid;
      rb = kk < L ? (kb ? kb[kk] : 0.f) : -INFINITY;
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* Ks = lds[buf];
    unsigned char* Vs = Ks + 8192;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cidx = tid + 256 * i, key = cidx >> 3, ch = cidx & 7;
      *(u32x4*)(Ks + a64_off(key, ch)) = rk[i];
      *(u32x4*)(Vs + a64v_off(key, ch)) = rv[i];  // V as stored: [key][d]
    }
    if (tid < 64) ((float*)(Ks + 16384))[tid] = rb;
  };

  bf16x8 sel;  // row-sum selector (A of 16x16x32): D row 0 = queries 0-15, row 1 = queries 16-31
  {
    const int m = lane & 15, kg = lane >> 4;
    const bool one = (m == 0 && (kg & 1) == 0) || (m == 1 && (kg & 1) == 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) sel[j] = (bf16)(one ? 1.0f : 0.0f);
  }
  // the re-run pass's running max, per chain and lane (= per query: lanes l and l + 32 hold one query's two key
  // halves and agree after the permlane swap); a reference shared by two queries can leave one of them with
  // underflowing sums, so each chain keeps its own
  f32x16 o[NCH][2];
  f32x4 lacc[NCH];
  const f32x16 zero16 = {};
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
    for (int i = 0; i < 16; ++i) o[ch][0][i] = o[ch][1][i] = 0.f;
    lacc[ch] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int ntiles = (L + A64_KT - 1) / A64_KT;

  gload(0);
  lstore(0);
  __syncthreads();
  // Pass 1: fixed reference 0 (Q carries log2(e)/8, so p = 2^s) -- no per-tile max, vote or rescale;
  // valid while every row sum stays in [2^-60, 2^100) (then every p <= 2^100: fp32 and bf16 hold it).
  // Otherwise the block re-runs with the lazily raised running max (pass 2, LAZY), as attention_pipe.hip does.
  auto run_pass = [&](auto lazyc) __attribute__((always_inline)) {
    constexpr bool LAZY = decltype(lazyc)::value;
    f32x16 negm[NCH];  // (the re-run pass only: local, so the first pass holds no registers for them)
    float mref[NCH];
    bool have_m[NCH];  // mref set (a tile with an unmasked key seen)
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int i = 0; i < 16; ++i) negm[ch][i] = 0.f;
      mref[ch] = 0.f;
      have_m[ch] = false;
    }
    for (int it = 0; it < ntiles; ++it) {
      const int k0 = it * A64_KT;
      if (it + 1 < ntiles) gload(k0 + A64_KT);
      const unsigned char* Ks = lds[it & 1];
      const unsigned char* Vs = Ks + 8192;
      const float* Bs = (const float*)(Ks + 16384);
      if (active) {
        bf16x8 kf[2][4];
  #pragma unroll
        for (int u = 0; u < 2; ++u)
  #pragma unroll
          for (int ks = 0; ks < 4; ++ks) kf[u][ks] = *(const bf16x8*)(Ks + a64_off(32 * u + r, 2 * ks + hh));
        f32x16 s[NCH][2];
  #pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
  #pragma unroll
          for (int u = 0; u < 2; ++u) {
            s[ch][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[u][0], qf[ch][0], LAZY ? negm[ch] : zero16, 0, 0,
                                                               0);
  #pragma unroll
            for (int ks = 1; ks < 4; ++ks)
              s[ch][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[u][ks], qf[ch][ks], s[ch][u], 0, 0, 0);
          }
        if (kbias != nullptr || (it == ntiles - 1 && (L % A64_KT) != 0)) {  // key bias and keys past L (0 / -inf)
  #pragma unroll
          for (int u = 0; u < 2; ++u)
  #pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float bv = Bs[32 * u + (i & 3) + 8 * (i >> 2) + 4 * hh];
  #pragma unroll
              for (int ch = 0; ch < NCH; ++ch)
                s[ch][u][i] = bv == 0.f ? s[ch][u][i] : (bv == -INFINITY ? -INFINITY : s[ch][u][i] + bv * kLog2e);
            }
        }
        if constexpr (LAZY) {
    #pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            float tm = fmaxf(s[ch][0][0], s[ch][1][0]);
    #pragma unroll
            for (int i = 1; i < 16; ++i) tm = fmaxf(tm, fmaxf(s[ch][0][i], s[ch][1][i]));
            {
              const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tm), __float_as_uint(tm), false, false);
              tm = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
            }
            if (__any(!have_m[ch] || tm > A64_TAU)) {  // wave-uniform lazy rescale
              const float delta = !have_m[ch] ? (tm == -INFINITY ? 0.f : tm) : fmaxf(tm, 0.f);
              have_m[ch] = have_m[ch] || tm != -INFINITY;
              const float alpha = exp2f(-delta);
              // the row sums' selector output: lane l < 16 holds query l's sum (element 0) and query l + 16's
              // (element 1; elements 2, 3 and lanes >= 16 are zero rows), so element 1 takes lane l + 16's factor
              const float alpha16 = __shfl(alpha, (lane & 15) + 16, 64);
              mref[ch] += delta;
    #pragma unroll
              for (int i = 0; i < 16; ++i) {
                o[ch][0][i] *= alpha, o[ch][1][i] *= alpha;
                s[ch][0][i] -= delta;
                s[ch][1][i] -= delta;
                negm[ch][i] = -mref[ch];
              }
              lacc[ch][0] *= alpha;
              lacc[ch][1] *= alpha16;
            }
          }
        }
        // V^T A fragments (lane: d = 32 db + (lane & 31); elements j: keys b + (j & 3) + 8 (j >> 2), b = 16 ks + 4 hh,
        // the P fragment's key order) as two transposed 4-key reads; lane 4q + p of each 16-lane group addresses
        // key b + q (+ 8), d's 16 ((lane >> 4) & 1) + 4p .. +3 of its block (active is wave-uniform: EXEC is full)
        bf16x8 vf[2][4];
        {
          const int q = (lane & 15) >> 2, p4 = lane & 3, dh = (lane >> 4) & 1;
  #pragma unroll
          for (int db = 0; db < 2; ++db)
  #pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              const int kb = 16 * ks + 4 * hh + q, cc = 4 * db + 2 * dh + (p4 >> 1);
              const a64_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (__attribute__((address_space(3))) a64_s4*)(Vs + a64v_off(kb, cc) + 8 * (p4 & 1)));
              const a64_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (__attribute__((address_space(3))) a64_s4*)(Vs + a64v_off(kb + 8, cc) + 8 * (p4 & 1)));
              const bf16x4 l4 = __builtin_bit_cast(bf16x4, lo), h4 = __builtin_bit_cast(bf16x4, hi);
              vf[db][ks] = bf16x8{l4[0], l4[1], l4[2], l4[3], h4[0], h4[1], h4[2], h4[3]};
            }
        }
        // chain by chain (a chain's scores die after its P.V): the next chain's exps issue beside this chain's MFMAs
  #pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
  #pragma unroll
          for (int u = 0; u < 2; ++u)
  #pragma unroll
            for (int sp = 0; sp < 2; ++sp) {
              bf16x8 pb;
  #pragma unroll
              for (int j = 0; j < 8; ++j) pb[j] = (bf16)__builtin_amdgcn_exp2f(s[ch][u][8 * sp + j]);
              const int ks = 2 * u + sp;
              o[ch][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[0][ks], pb, o[ch][0], 0, 0, 0);
              o[ch][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[1][ks], pb, o[ch][1], 0, 0, 0);
              lacc[ch] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pb, lacc[ch], 0, 0, 0);
            }
      }
      if (it + 1 < ntiles) lstore((it + 1) & 1);
      __syncthreads();
    }
  };
  run_pass(std::false_type{});
  {
    bool bad = false;
    if (active)
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const float la = __shfl(lacc[ch][0], lane & 15, 64), lb = __shfl(lacc[ch][1], lane & 15, 64);
        const float ls = r < 16 ? la : lb;
        bad |= !(ls >= 0x1p-60f && ls < 0x1p100f) && qi[ch] < nq;  // also 0 (underflow or every key masked), inf, NaN
      }
    if (__syncthreads_or(bad ? 1 : 0)) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
        for (int i = 0; i < 16; ++i) o[ch][0][i] = o[ch][1][i] = 0.f;
        lacc[ch] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      gload(0);
      lstore(0);
      __syncthreads();
      run_pass(std::true_type{});
    }
  }
  if (!active) return;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const float la = __shfl(lacc[ch][0], lane & 15, 64), lb = __shfl(lacc[ch][1], lane & 15, 64);
    const float ls = r < 16 ? la : lb;
    const float inv = ls > 0.f ? 1.0f / ls : 0.f;  // a query with every key masked gets 0
    if (qi[ch] < nq) {
      bf16* orow = out + ((int64_t)b * o_bstride + qi[ch]) * D + h * 64;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = (bf16)(o[ch][db][4 * g + e] * inv);
          *(bf16x4*)(orow + 32 * db + 8 * g + 4 * hh) = w;
        }
    }
  }
}

// ---------------------------------------------------------------- attention, head_dim 64 (fp32)
// Parity mode: one query per thread, K / V tiles of 32 keys staged in LDS (broadcast reads),
// online softmax in natural-exp units with the reference's 1/sqrt(64) scale on the scores.
__global__ __launch_bounds__(128) void attn64_f32_kernel(const float* __restrict__ qkv,
                                                         const float* __restrict__ kbias, float* __restrict__ out,
                                                         int L, int H, int q0, int nq, int64_t o_bstride,
                                                         int chunks) {
  __shared__ __attribute__((aligned(16))) float Ks[32][64], Vs[32][64], Bs[32];
  const int tid = threadIdx.x;
  const int chunk = blockIdx.x % chunks, bh = blockIdx.x / chunks;
  const int h = bh % H, b = bh / H;
  const int D = H * 64;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = qkv + (int64_t)b * L * ld;
  const int qi = chunk * 128 + tid;
  const int qt = q0 + min(qi, nq - 1);
  float q[64], o[64];
  {
    const float* qrow = base + (int64_t)qt * ld + h * 64;
#pragma unroll
    for (int d = 0; d < 64; d += 4) *(f32x4*)(q + d) = *(const f32x4*)(qrow + d);
  }
#pragma unroll
  for (int d = 0; d < 64; ++d) o[d] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < L; k0 += 32) {
    __syncthreads();
    for (int u = tid; u < 32 * 16; u += 128) {
      const int key = u >> 4, c4 = u & 15, kk = k0 + key;
      const float* row = base + (int64_t)min(kk, L - 1) * ld + h * 64 + 4 * c4;
      *(f32x4*)(&Ks[key][4 * c4]) = *(const f32x4*)(row + D);
      *(f32x4*)(&Vs[key][4 * c4]) = kk < L ? *(const f32x4*)(row + 2 * D) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (tid < 32) {
      const int kk = k0 + tid;
      Bs[tid] = kk < L ? (kbias ? kbias[(int64_t)b * L + kk] : 0.f) : -INFINITY;
    }
    __syncthreads();
    const int nk = min(32, L - k0);
    for (int k = 0; k < nk; ++k) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) s = fmaf(q[d], Ks[k][d], s);
      s = s * 0.125f + Bs[k];
      if (s == -INFINITY) continue;
      if (s > m) {
        const float alpha = expf(m - s);  // m = -inf on the first key: alpha = 0
#pragma unroll
        for (int d = 0; d < 64; ++d) o[d] *= alpha;
        l *= alpha;
        m = s;
      }
      const float p = expf(s - m);
      l += p;
#pragma unroll
      for (int d = 0; d < 64; ++d) o[d] = fmaf(p, Vs[k][d], o[d]);
    }
  }
  if (qi < nq) {
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    float* orow = out + ((int64_t)b * o_bstride + qi) * D + h * 64;
#pragma unroll
    for (int d = 0; d < 64; d += 4) *(f32x4*)(orow + d) = f32x4{o[d] * inv, o[d + 1] * inv, o[d + 2] * inv, o[d + 3] * inv};
  }
}

// ---------------------------------------------------------------- LayerNorm, one wave per row
// fp32 in; fp32 out (may alias in) and / or bf16 out; affine (gamma, beta may be null)
// LN_RPW rows per wave (a block of 4 waves covers 4 * LN_RPW rows)
constexpr int LN_RPW = 1;  // 4 measured slower (148 vs 120 us per ViT LayerNorm): fewer rows in flight
template <int V4>
__global__ __launch_bounds__(256) void ln_dual_kernel(const float* in, int64_t rows, int dim, float eps,
                                                      float* out32, bf16* __restrict__ out16,
                                                      const float* __restrict__ g, const float* __restrict__ bta,
                                                      int64_t in_rstride, int64_t out_rstride) {
  const int lane = threadIdx.x & 63;
  for (int rr = 0; rr < LN_RPW; ++rr) {
  const int64_t row = ((int64_t)blockIdx.x * LN_RPW + rr) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* x = in + row * in_rstride;
  const int n4 = dim >> 2;
  f32x4 v[V4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i4 = lane + 64 * j;
    v[j] = i4 < n4 ? *(const f32x4*)(x + 4 * i4) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  }
  const float mean = wave_sum_dpp_f(s) / dim;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j)
    if (lane + 64 * j < n4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mean;
        q += d * d;
      }
  const float inv = 1.0f / sqrtf(wave_sum_dpp_f(q) / dim + eps);
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i4 = lane + 64 * j;
    if (i4 >= n4) continue;
    // gamma / beta as 16-B loads (dim % 4 == 0), not 4-B loads per element
    const f32x4 gv = g ? *(const f32x4*)(g + 4 * i4) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 bv = bta ? *(const f32x4*)(bta + 4 * i4) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = (v[j][e] - mean) * inv * gv[e] + bv[e];
    if (out32) *(f32x4*)(out32 + row * out_rstride + 4 * i4) = y;
    if (out16) {
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (bf16)y[e];
      *(bf16x4*)(out16 + row * out_rstride + 4 * i4) = w;
    }
  }
  }
}

// ---------------------------------------------------------------- patch embedding helpers
// im2col of Conv2d(C, D, kernel P, stride P): row (b, py, px), column c * P * P + ky * P + kx
// (the conv weight's flattening), zero past C * P * P up to Kpad
template <typename TO>
__global__ void im2col_kernel(const float* __restrict__ img, int B, int C, int Hh, int Ww, int P, int Kpad,
                              TO* __restrict__ out) {
  const int gh = Hh / P, gw = Ww / P;
  const int64_t total = (int64_t)B * gh * gw * Kpad;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(u % Kpad);
    const int64_t rowi = u / Kpad;
    const int px = (int)(rowi % gw), py = (int)((rowi / gw) % gh);
    const int64_t b = rowi / ((int64_t)gw * gh);
    float v = 0.f;
    if (k < C * P * P) {
      const int c = k / (P * P), ky = (k / P) % P, kx = k % P;
      v = img[((b * C + c) * Hh + (py * P + ky)) * Ww + px * P + kx];
    }
    out[u] = from_f32<TO>(v);
  }
}

// torch upsample_bicubic2d (align_corners=False, A = -0.75, border-clamped taps) of the patch
// positional grid [M][M][D] to [oh][ow][D] with source scales sh, sw (input / output)
__device__ __forceinline__ float cubic_conv1(float x, float A) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; }
__device__ __forceinline__ float cubic_conv2(float x, float A) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; }
__device__ __forceinline__ float cubic_interp(float x0, float x1, float x2, float x3, float t) {
  const float A = -0.75f;
  const float c0 = cubic_conv2(t + 1.f, A), c1 = cubic_conv1(t, A), c2 = cubic_conv1(1.f - t, A),
              c3 = cubic_conv2(2.f - t, A);
  return x0 * c0 + x1 * c1 + x2 * c2 + x3 * c3;
}
__global__ void pos_interp_kernel(const float* __restrict__ pos /*[1 + M*M][D]*/, int M, int D, int oh, int ow,
                                  float sh, float sw, float* __restrict__ out /*[1 + oh*ow][D]*/) {
  const int64_t total = (int64_t)(1 + oh * ow) * D;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(u % D);
    const int t = (int)(u / D);
    if (t == 0) {
      out[u] = pos[d];
      continue;
    }
    const int oy = (t - 1) / ow, ox = (t - 1) % ow;
    const float ry = sh * (oy + 0.5f) - 0.5f, rx = sw * (ox + 0.5f) - 0.5f;
    const int iy = (int)floorf(ry), ix = (int)floorf(rx);
    const float ty = ry - iy, tx = rx - ix;
    float rowv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int yy = min(max(iy - 1 + i, 0), M - 1);
      float xs[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int xx = min(max(ix - 1 + j, 0), M - 1);
        xs[j] = pos[(int64_t)(1 + yy * M + xx) * D + d];
      }
      rowv[i] = cubic_interp(xs[0], xs[1], xs[2], xs[3], tx);
    }
    out[u] = cubic_interp(rowv[0], rowv[1], rowv[2], rowv[3], ty);
  }
}

// X[b][0] = cls + pe[0]; X[b][1 + p] = patches[b][p] + pe[1 + p]
__global__ void vit_assemble_kernel(const float* __restrict__ patches, const float* __restrict__ cls,
                                    const float* __restrict__ pe, int B, int np, int D, float* __restrict__ X) {
  const int64_t total = (int64_t)B * (np + 1) * D;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(u % D);
    const int64_t bt = u / D;
    const int t = (int)(bt % (np + 1));
    const int64_t b = bt / (np + 1);
    const float v = t == 0 ? cls[d] : patches[(b * np + t - 1) * D + d];
    X[u] = v + pe[(int64_t)t * D + d];
  }
}

// text embeddings (ElectraEmbeddings.forward): LN((word[id] + type[tt]) + pos[t]), one wave per token
template <int V4>
__global__ __launch_bounds__(256) void text_embed_kernel(const int* __restrict__ ids, const int* __restrict__ types,
                                                         int64_t ntok, int L, int E, const float* __restrict__ wemb,
                                                         const float* __restrict__ pemb,
                                                         const float* __restrict__ temb, const float* __restrict__ g,
                                                         const float* __restrict__ bt, float eps,
                                                         float* __restrict__ out32, bf16* __restrict__ out16,
                                                         int vocab, int ntypes, int* __restrict__ flag) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tok >= ntok) return;
  int id = ids[tok], tt = types ? types[tok] : 0;
  const int t = (int)(tok % L);
  if (id < 0 || id >= vocab || tt < 0 || tt >= ntypes) {  // the reference's embedding lookup raises
    if (lane == 0) atomicOr(flag, 1);
    id = min(max(id, 0), vocab - 1), tt = min(max(tt, 0), ntypes - 1);
  }
  const int n4 = E >> 2;
  f32x4 v[V4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i4 = lane + 64 * j;
    if (i4 < n4) {
      const f32x4 w = *(const f32x4*)(wemb + (int64_t)id * E + 4 * i4);
      const f32x4 ty = *(const f32x4*)(temb + (int64_t)tt * E + 4 * i4);
      const f32x4 p = *(const f32x4*)(pemb + (int64_t)t * E + 4 * i4);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = (w[e] + ty[e]) + p[e];
    } else {
      v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  }
  const float mean = wave_sum(s) / E;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j)
    if (lane + 64 * j < n4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mean;
        q += d * d;
      }
  const float inv = 1.0f / sqrtf(wave_sum(q) / E + eps);
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i4 = lane + 64 * j;
    if (i4 >= n4) continue;
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = (v[j][e] - mean) * inv * g[4 * i4 + e] + bt[4 * i4 + e];
    if (out32) *(f32x4*)(out32 + tok * E + 4 * i4) = y;
    if (out16) {
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (bf16)y[e];
      *(bf16x4*)(out16 + tok * E + 4 * i4) = w;
    }
  }
}

// X += gamma (.) Y (gamma null: 1), rows x dim, both [rows][dim] fp32
__global__ void resid_kernel(float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ g,
                             int64_t n4, int dim) {
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n4; u += (int64_t)gridDim.x * blockDim.x) {
    f32x4 x = ((f32x4*)X)[u];
    const f32x4 y = ((const f32x4*)Y)[u];
    const int c = (int)((u * 4) % dim);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = g ? fmaf(g[c + e], y[e], x[e]) : x[e] + y[e];
    ((f32x4*)X)[u] = x;
  }
}

// out[i] = in[i * in_rstride .. + dim) for rows i (gather one row per batch, e.g. the CLS rows)
template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ in, int64_t in_rstride, int rows, int dim, T* __restrict__ out) {
  const int64_t total = (int64_t)rows * dim;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rr = u / dim;
    out[u] = in[rr * in_rstride + u % dim];
  }
}

// attention_mask [n] int32 (1 keep / 0 exclude) -> additive key bias 0 / -inf
__global__ void mask_bias_kernel(const int* __restrict__ mask, float* __restrict__ out, int64_t n) {
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
    out[u] = mask[u] != 0 ? 0.f : -INFINITY;
}

__global__ void cast_bf16_kernel(const float* __restrict__ in, bf16* __restrict__ out, int64_t n) {
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
    out[u] = (bf16)in[u];
}

inline unsigned grid_for(int64_t n, int threads = 256) {
  const int64_t g = (n + threads - 1) / threads;
  return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

hipError_t launch_gemm_tile(const void* A, const void* W, const float* bias, const float* gamma, void* C,
                            int64_t ldc, int M, int N, int K, int epi, int act, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (N % TN != 0 || K % TK != 0 || K <= 0 || (epi != GT_BF16 && act != 0)) return hipErrorInvalidValue;
  const int mtiles = (M + TM - 1) / TM;
  const int64_t nb = (int64_t)mtiles * (N / TN);
  dim3 g((unsigned)nb), blk(512);
  const bf16 *a = (const bf16*)A, *w = (const bf16*)W;
  switch (epi * 2 + act) {
    case GT_BF16 * 2: hipLaunchKernelGGL((gemm_tile_kernel<GT_BF16, 0>), g, blk, GT_LDS, st, a, w, bias, gamma, C, ldc, M, N, K, mtiles); break;
    case GT_BF16 * 2 + 1: hipLaunchKernelGGL((gemm_tile_kernel<GT_BF16, 1>), g, blk, GT_LDS, st, a, w, bias, gamma, C, ldc, M, N, K, mtiles); break;
    case GT_RESID * 2: hipLaunchKernelGGL((gemm_tile_kernel<GT_RESID, 0>), g, blk, GT_LDS, st, a, w, bias, gamma, C, ldc, M, N, K, mtiles); break;
    case GT_F32 * 2: hipLaunchKernelGGL((gemm_tile_kernel<GT_F32, 0>), g, blk, GT_LDS, st, a, w, bias, gamma, C, ldc, M, N, K, mtiles); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_attn64(const void* qkv, const float* kbias, void* out, int B, int L, int H, int q0, int nq,
                         int64_t o_bstride, int prec, hipStream_t st) {
  if (B <= 0 || nq <= 0) return hipSuccess;
  if (L <= 0 || H <= 0 || q0 < 0 || q0 + nq > L) return hipErrorInvalidValue;
  if (prec == PREC_BF16) {
    const int chunks = (nq + 128 * A64_NCH - 1) / (128 * A64_NCH);
    const int64_t nb = (int64_t)B * H * chunks;
    if (nb > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attn64_kernel<A64_NCH>, dim3((unsigned)nb), dim3(256), 0, st, (const bf16*)qkv, kbias,
                       (bf16*)out, L, H, q0, nq, o_bstride, chunks, (int)nb);
  } else {
    const int chunks = (nq + 127) / 128;
    const int64_t nb = (int64_t)B * H * chunks;
    if (nb > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attn64_f32_kernel, dim3((unsigned)nb), dim3(128), 0, st, (const float*)qkv, kbias, (float*)out,
                       L, H, q0, nq, o_bstride, chunks);
  }
  return hipGetLastError();
}

hipError_t launch_ln_dual(const float* in, int64_t rows, int dim, float eps, float* out32, void* out16,
                          const float* gamma, const float* beta, hipStream_t st, int64_t in_rstride,
                          int64_t out_rstride) {
  if (rows <= 0) return hipSuccess;
  if (dim % 4 != 0 || dim > 1024) return hipErrorInvalidValue;
  if (in_rstride <= 0) in_rstride = dim;
  if (out_rstride <= 0) out_rstride = dim;
  const int v4 = (dim / 4 + 63) / 64;
  dim3 g((unsigned)((rows + 4 * LN_RPW - 1) / (4 * LN_RPW))), b(256);
  switch (v4) {
    case 1: hipLaunchKernelGGL(ln_dual_kernel<1>, g, b, 0, st, in, rows, dim, eps, out32, (bf16*)out16, gamma, beta, in_rstride, out_rstride); break;
    case 2: hipLaunchKernelGGL(ln_dual_kernel<2>, g, b, 0, st, in, rows, dim, eps, out32, (bf16*)out16, gamma, beta, in_rstride, out_rstride); break;
    case 3: hipLaunchKernelGGL(ln_dual_kernel<3>, g, b, 0, st, in, rows, dim, eps, out32, (bf16*)out16, gamma, beta, in_rstride, out_rstride); break;
    default: hipLaunchKernelGGL(ln_dual_kernel<4>, g, b, 0, st, in, rows, dim, eps, out32, (bf16*)out16, gamma, beta, in_rstride, out_rstride); break;
  }
  return hipGetLastError();
}

hipError_t launch_im2col(const float* img, int B, int C, int H, int W, int P, int Kpad, void* out, bool out_f32,
                         hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (H % P || W % P || Kpad < C * P * P) return hipErrorInvalidValue;
  const int64_t n = (int64_t)B * (H / P) * (W / P) * Kpad;
  if (out_f32) hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, img, B, C, H, W, P, Kpad, (float*)out);
  else hipLaunchKernelGGL(im2col_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, img, B, C, H, W, P, Kpad, (bf16*)out);
  return hipGetLastError();
}

hipError_t launch_pos_interp(const float* pos, int M, int D, int oh, int ow, float sh, float sw, float* out,
                             hipStream_t st) {
  const int64_t n = (int64_t)(1 + oh * ow) * D;
  hipLaunchKernelGGL(pos_interp_kernel, dim3(grid_for(n)), dim3(256), 0, st, pos, M, D, oh, ow, sh, sw, out);
  return hipGetLastError();
}

hipError_t launch_vit_assemble(const float* patches, const float* cls, const float* pe, int B, int np, int D,
                               float* X, hipStream_t st) {
  const int64_t n = (int64_t)B * (np + 1) * D;
  hipLaunchKernelGGL(vit_assemble_kernel, dim3(grid_for(n)), dim3(256), 0, st, patches, cls, pe, B, np, D, X);
  return hipGetLastError();
}

hipError_t launch_text_embed(const int* ids, const int* types, int64_t ntok, int L, int E, const float* wemb,
                             const float* pemb, const float* temb, const float* g, const float* b, float eps,
                             float* out32, void* out16, int vocab, int ntypes, int* flag, hipStream_t st) {
  if (ntok <= 0) return hipSuccess;
  if (E % 4 != 0 || E > 1024) return hipErrorInvalidValue;
  const int v4 = (E / 4 + 63) / 64;
  dim3 gr((unsigned)((ntok + 3) / 4)), bl(256);
  switch (v4) {
    case 1: hipLaunchKernelGGL(text_embed_kernel<1>, gr, bl, 0, st, ids, types, ntok, L, E, wemb, pemb, temb, g, b, eps, out32, (bf16*)out16, vocab, ntypes, flag); break;
    case 2: hipLaunchKernelGGL(text_embed_kernel<2>, gr, bl, 0, st, ids, types, ntok, L, E, wemb, pemb, temb, g, b, eps, out32, (bf16*)out16, vocab, ntypes, flag); break;
    case 3: hipLaunchKernelGGL(text_embed_kernel<3>, gr, bl, 0, st, ids, types, ntok, L, E, wemb, pemb, temb, g, b, eps, out32, (bf16*)out16, vocab, ntypes, flag); break;
    default: hipLaunchKernelGGL(text_embed_kernel<4>, gr, bl, 0, st, ids, types, ntok, L, E, wemb, pemb, temb, g, b, eps, out32, (bf16*)out16, vocab, ntypes, flag); break;
  }
  return hipGetLastError();
}

hipError_t launch_resid(float* X, const float* Y, const float* gamma, int64_t rows, int dim, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  if (dim % 4 != 0) return hipErrorInvalidValue;
  const int64_t n4 = rows * dim / 4;
  hipLaunchKernelGGL(resid_kernel, dim3(grid_for(n4)), dim3(256), 0, st, X, Y, gamma, n4, dim);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const void* in, int64_t in_rstride, int rows, int dim, void* out, int elem_bytes,
                              hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  const int64_t n = (int64_t)rows * dim;
  if (elem_bytes == 4)
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (const float*)in, in_rstride, rows, dim, (float*)out);
  else
    hipLaunchKernelGGL(gather_rows_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (const bf16*)in, in_rstride, rows, dim, (bf16*)out);
  return hipGetLastError();
}

hipError_t launch_mask_bias(const int* mask, float* out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mask_bias_kernel, dim3(grid_for(n)), dim3(256), 0, st, mask, out, n);
  return hipGetLastError();
}

hipError_t launch_cast_bf16(const float* in, void* out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, st, in, (bf16*)out, n);
  return hipGetLastError();
}

}  // namespace mmpfn
