// Attention kernels of the PerFeatureEncoderLayer (layer.py:332-395,
// multi_head_attention.py:547-736) for gfx950.
//
// One MFMA flash-attention kernel serves both axes:
//  * sample axis (attn_between_items): batch = token column t, queries = rows s,
//    4 waves x 32 queries per block -- the dominant cost of the forward;
//  * feature axis (attn_between_features): batch = row s, queries = keys = the T
//    tokens of that row, one wave per block.
//
// Sample-axis details:
//    For token column t and head h, query rows s in [s0, s0+nq) attend to keys
//    [0, nk) (the train rows).  Train queries use their own head's K/V; test queries
//    use head 0's K/V for every head (reuse_first_head_kv, layer.py:344-358) via
//    kv_head_fixed = 0.  The scores are computed transposed, S^T = K . Q^T, so the
//    query index lives on the MFMA lane and the keys in accumulator registers: the
//    softmax row reductions are in-register (plus one lane^32 exchange) and the
//    S^T accumulator is fed back as the B operand of O^T += V^T . P^T without any
//    LDS round trip (cdna_hip_programming.md section 3, "accumulator as operand").
//    exp2 with log2(e)/sqrt(d) folded into one FMA; the row sum is kept per half-wave
//    and combined once at the end.
//      bf16 : v_mfma_f32_32x32x16_bf16 (4 per 32x64 score tile + 4 for P.V)
//      f32  : v_mfma_f32_32x32x2_f32 (parity mode; exact fp32 fma chains)
#include <atomic>

#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

// ------------------------------------------------------------------ item attention
constexpr int IA_KT = 64;          // keys per LDS tile

template <bool BF16>
struct IaLds {
  static constexpr int KROW = BF16 ? 80 : 144;    // bytes per key row   (32 d + pad)
  static constexpr int VROW = BF16 ? 136 : 272;   // bytes per V^T row   (64 keys + pad)
  static constexpr int KBYTES = IA_KT * KROW;
  static constexpr int VBYTES = 32 * VROW;
  static constexpr int STAGE = KBYTES + VBYTES;
};

// Softmax bookkeeping (per lane = per query, log2 domain, Q pre-scaled by log2(e)/sqrt(d)):
//   m_ref : reference max; S^T accumulators start from -m_ref (a persistent 16-register
//           vector), so the MFMA chain itself yields s - m_ref and p = exp2(acc) needs no
//           extra VALU op.
//   lazy rescale: m_ref only moves when a tile's max exceeds it by more than TAU
//           (p <= 2^TAU, safe in bf16/fp32) -- wave-uniform branch, rare after the
//           first tiles; the first tile always sets m_ref.
//   row sum (bf16 path): an extra MFMA with an all-ones A operand accumulates
//           sum_k p into every register of lacc, moving the adds off the VALU.
constexpr float IA_TAU = 8.0f;

// hi = bf16(x), lo = bf16(x - hi) of 8 fp32 values (the parity mode's split operands)
__device__ __forceinline__ void split8v(f32x4 a, f32x4 b, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    hi[i] = (bf16)a[i], hi[4 + i] = (bf16)b[i];
    lo[i] = (bf16)(a[i] - (float)hi[i]), lo[4 + i] = (bf16)(b[i] - (float)hi[4 + i]);
  }
}

// MODE 0: fp32-input MFMA (PREC_F32_MFMA), 1: bf16, 2: parity mode on fp32 data with split-bf16 operands
// (three products per contraction, like attn_item3); modes 0 and 2 share the fp32 LDS images
template <int MODE, int NW>
__global__ __launch_bounds__(64 * NW) void attn_item_kernel(const AttnArgs p) {
  constexpr bool BF16 = MODE == 1, X3 = MODE == 2;
  typedef typename std::conditional<BF16, bf16, float>::type TE;
  constexpr int EB = sizeof(TE);
  using L = IaLds<BF16>;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * L::STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  constexpr int NT = 64 * NW;  // threads per block
  // XCD-aware block order: the hardware deals consecutive workgroups round-robin to the 8
  // XCDs; remap so each XCD works through a contiguous run of (query block, head, batch)
  // ids, i.e. the blocks sharing one K/V sequence share that XCD's L2.
  int qblk, h, b;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const int nb = gx * gy * gridDim.z;
    const int pid = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = pid & 7, slot = pid >> 3;
    const int lid = xcd * (nb >> 3) + min(xcd, nb & 7) + slot;
    qblk = lid % gx;
    const int rest = lid / gx;
    h = rest % gy;
    b = rest / gy;
  }
  const int kvh = p.kvh_fixed >= 0 ? p.kvh_fixed : h;
  const int s0 = p.s0, nq = p.nq, nk = p.nk, Npad = p.kpad;
  const TE* Q = (const TE*)p.q + b * p.q_bstride + h * p.q_hstride;
  const TE* Kg = (const TE*)p.k + b * p.kv_bstride + kvh * p.kv_hstride;
  const TE* Vg = (const TE*)p.vt + b * p.kv_bstride + kvh * p.kv_hstride;
  const float c = kLog2e * 0.17677669529663687f;  // log2(e)/sqrt(32)

  const int qi = qblk * (32 * NW) + wave * 32 + r;  // query offset in [0, nq)
  const int64_t qs = s0 + min(qi, nq - 1);

  // ---- Q fragments (B operand of S^T = K Q^T), pre-scaled by c
  bf16x8 qb[2], ql[2];
  float qf[16];
  if constexpr (X3) {
    const float* qrow = (const float*)Q + qs * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f32x4 a = *(const f32x4*)(qrow + 16 * ks + 8 * hh), b = *(const f32x4*)(qrow + 16 * ks + 8 * hh + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] *= c, b[i] *= c;
      split8v(a, b, qb[ks], ql[ks]);
    }
  } else if constexpr (BF16) {
    const bf16* qrow = (const bf16*)Q + qs * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 raw = *(const bf16x8*)(qrow + 16 * ks + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) qb[ks][j] = (bf16)((float)raw[j] * c);
    }
  } else {
    const float* qrow = (const float*)Q + qs * 32 + 16 * hh;
#pragma unroll
    for (int i = 0; i < 16; i += 4) *(f32x4*)(qf + i) = *(const f32x4*)(qrow + i);
#pragma unroll
    for (int i = 0; i < 16; ++i) qf[i] *= c;
  }

  // ---- staging: K tile [64][32], V^T tile [32][64]
  constexpr int KCH = IA_KT * 32 * EB / 16 / NT;  // 16-byte chunks per thread (K)
  constexpr int VCH = 32 * IA_KT * EB / 16 / NT;
  constexpr int VCPR = IA_KT * EB / 16;            // chunks per V^T row
  constexpr int EPC = 16 / EB;                     // elements per chunk
  u32x4 rk[KCH], rv[VCH];
  auto gload = [&](int k0, auto maskc) {
    constexpr bool MASKV = decltype(maskc)::value;
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int cidx = tid + NT * i;  // chunk over the contiguous K tile
      rk[i] = *(const u32x4*)((const unsigned char*)(Kg + (int64_t)k0 * 32) + cidx * 16);
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int cidx = tid + NT * i;
      const int d = cidx / VCPR, ch = cidx % VCPR;
      rv[i] = *(const u32x4*)((const unsigned char*)(Vg + (int64_t)d * Npad + k0) + ch * 16);
      if constexpr (MASKV) {  // zero V for keys >= nk: masked p = 0 must never meet NaN/inf
        const int kfirst = k0 + ch * EPC;
        if constexpr (BF16) {
          bf16x8 e = __builtin_bit_cast(bf16x8, rv[i]);
#pragma unroll
          for (int j = 0; j < EPC; ++j)
            if (kfirst + j >= nk) e[j] = (bf16)0.0f;
          rv[i] = __builtin_bit_cast(u32x4, e);
        } else {
          f32x4 e = __builtin_bit_cast(f32x4, rv[i]);
#pragma unroll
          for (int j = 0; j < EPC; ++j)
            if (kfirst + j >= nk) e[j] = 0.0f;
          rv[i] = __builtin_bit_cast(u32x4, e);
        }
      }
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* Ks = lds + buf * L::STAGE;
    unsigned char* Vs = Ks + L::KBYTES;
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int cidx = tid + NT * i;
      constexpr int CPR = 32 * EB / 16;  // chunks per K row
      const int row = cidx / CPR, ch = cidx % CPR;
      *(u32x4*)(Ks + row * L::KROW + ch * 16) = rk[i];
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int cidx = tid + NT * i;
      const int d = cidx / VCPR, ch = cidx % VCPR;
      unsigned char* dst = Vs + d * L::VROW + ch * 16;
      if constexpr (BF16) {  // 136-byte rows are 8-byte aligned only
        *(u32x2*)dst = u32x2{rv[i].x, rv[i].y};
        *(u32x2*)(dst + 8) = u32x2{rv[i].z, rv[i].w};
      } else {
        *(u32x4*)dst = rv[i];
      }
    }
  };

  f32x16 o, lacc, negm;
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = lacc[i] = negm[i] = 0.f;
  float mref = 0.f, lsum = 0.f;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.0f;

  const int ntiles = (nk + IA_KT - 1) / IA_KT;
  const bool partial = (nk % IA_KT) != 0;

  auto tile = [&](int it, auto maskc, auto firstc) {
    constexpr bool MASK = decltype(maskc)::value;
    constexpr bool FIRST = decltype(firstc)::value;
    const int k0 = it * IA_KT;
    if (it + 1 < ntiles) {
      if (partial && it + 2 == ntiles) gload(k0 + IA_KT, std::true_type{});
      else gload(k0 + IA_KT, std::false_type{});
    }
    const unsigned char* Ks = lds + (it & 1) * L::STAGE;
    const unsigned char* Vs = Ks + L::KBYTES;

    // ---- S^T - m_ref for the two 32-key subtiles
    f32x16 sacc[2];
    if constexpr (X3) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const unsigned char* krow = Ks + (32 * u + r) * L::KROW;
        bf16x8 kh[2], kl[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          split8v(*(const f32x4*)(krow + (16 * ks + 8 * hh) * 4), *(const f32x4*)(krow + (16 * ks + 8 * hh + 4) * 4),
                  kh[ks], kl[ks]);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[0], qb[0], negm, 0, 0, 0);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[1], qb[1], sacc[u], 0, 0, 0);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[0], ql[0], sacc[u], 0, 0, 0);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[1], ql[1], sacc[u], 0, 0, 0);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[0], qb[0], sacc[u], 0, 0, 0);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[1], qb[1], sacc[u], 0, 0, 0);
      }
    } else if constexpr (BF16) {
      // all four K fragments in flight before the first MFMA (the scheduler otherwise
      // serialises read -> wait -> MFMA and exposes the LDS latency four times)
      bf16x8 kf[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const unsigned char* krow = Ks + (32 * u + r) * L::KROW;
        kf[u][0] = *(const bf16x8*)(krow + (8 * hh) * 2);
        kf[u][1] = *(const bf16x8*)(krow + (16 + 8 * hh) * 2);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[u][0], qb[0], negm, 0, 0, 0);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[u][1], qb[1], sacc[u], 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const unsigned char* krow = Ks + (32 * u + r) * L::KROW;
      if constexpr (BF16 || X3) {
      } else {
        float kf[16];
#pragma unroll
        for (int i = 0; i < 16; i += 4) *(f32x4*)(kf + i) = *(const f32x4*)(krow + (16 * hh + i) * 4);
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[0], qf[0], negm, 0, 0, 0);
#pragma unroll
        for (int ks = 1; ks < 16; ++ks)
          sacc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[ks], qf[ks], sacc[u], 0, 0, 0);
      }
    }
    if constexpr (MASK) {  // keys >= nk (last tile only)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + 32 * u + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (key >= nk) sacc[u][i] = -INFINITY;
        }
    }
    // ---- tile max relative to m_ref (lane^32 holds the other 32 keys of this query)
    float tm = fmaxf(sacc[0][0], sacc[1][0]);
#pragma unroll
    for (int i = 1; i < 16; ++i) tm = fmaxf(tm, fmaxf(sacc[0][i], sacc[1][i]));
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tm), __float_as_uint(tm), false, false);
      tm = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    if (FIRST || __any(tm > IA_TAU)) {  // wave-uniform lazy rescale
      const float delta = FIRST ? tm : fmaxf(tm, 0.f);
      if constexpr (!FIRST) {
        const float alpha = exp2f(-delta);
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] *= alpha;
        if constexpr (BF16) {
#pragma unroll
          for (int i = 0; i < 16; ++i) lacc[i] *= alpha;
        } else {
          lsum *= alpha;
        }
      }
      mref += delta;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        negm[i] = -mref;
        sacc[0][i] -= delta;
        sacc[1][i] -= delta;
      }
    }
    // ---- p = exp2(s - m_ref), O^T += V^T . P^T, l += 1 . P^T
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const unsigned char* vrow = Vs + r * L::VROW;
      if constexpr (X3) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          f32x4 pa, pc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pa[j] = exp2f(sacc[u][8 * sp + j]);
            pc[j] = exp2f(sacc[u][8 * sp + 4 + j]);
            lsum += pa[j] + pc[j];
          }
          bf16x8 ph, pl, vh, vl;
          split8v(pa, pc, ph, pl);
          const int kb = 32 * u + 16 * sp + 4 * hh;
          split8v(*(const f32x4*)(vrow + kb * 4), *(const f32x4*)(vrow + (kb + 8) * 4), vh, vl);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph, o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl, o, 0, 0, 0);
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph, o, 0, 0, 0);
        }
      } else if constexpr (BF16) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = (bf16)__builtin_amdgcn_exp2f(sacc[u][8 * sp + j]);
          const int kb = 32 * u + 16 * sp + 4 * hh;
          const u32x2 v0 = *(const u32x2*)(vrow + kb * 2);
          const u32x2 v1 = *(const u32x2*)(vrow + (kb + 8) * 2);
          const bf16x8 va = __builtin_bit_cast(bf16x8, u32x4{v0.x, v0.y, v1.x, v1.y});
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, o, 0, 0, 0);
          lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pb, lacc, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sacc[u][i] = exp2f(sacc[u][i]);
          lsum += sacc[u][i];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 vv = *(const f32x4*)(vrow + (32 * u + 8 * g + 4 * hh) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o = __builtin_amdgcn_mfma_f32_32x32x2f32(vv[e], sacc[u][4 * g + e], o, 0, 0, 0);
        }
      }
    }
    if (it + 1 < ntiles) lstore((it + 1) & 1);
    __syncthreads();
  };

  gload(0, std::bool_constant<true>{});  // masking is a no-op unless the tile is partial
  lstore(0);
  __syncthreads();
  if (ntiles == 1) {
    if (partial) tile(0, std::true_type{}, std::true_type{});
    else tile(0, std::false_type{}, std::true_type{});
  } else {
    tile(0, std::false_type{}, std::true_type{});
    const int nfull = nk / IA_KT;
    for (int it = 1; it < nfull; ++it) tile(it, std::false_type{}, std::false_type{});
    if (partial) tile(nfull, std::true_type{}, std::false_type{});
  }

  // ---- normalise and store O[t][s][h*32 + d]
  float ltot;
  if constexpr (BF16) {
    ltot = lacc[0];
  } else {
    const auto lw = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum), __float_as_uint(lsum), false, false);
    ltot = __uint_as_float(lw[0]) + __uint_as_float(lw[1]);
  }
  const float inv = 1.0f / ltot;
  if (qi < nq) {
    TE* orow = (TE*)p.o + (b * p.o_bstride + qs * p.o_qstride) * (p.H * 32) + h * 32;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 8 * g + 4 * hh;
      if constexpr (BF16) {
        bf16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (bf16)(o[4 * g + e] * inv);
        *(bf16x4*)(orow + d) = w;
      } else {
        f32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = o[4 * g + e] * inv;
        *(f32x4*)(orow + d) = w;
      }
    }
  }
}

// ------------------------------------------------------------------ feature attention, parity mode
// PREC_F32 attention between features (layer.py:332-339): per table row s and head h, the row's T <= 64
// tokens attend to each other.  One wave per (row, head): queries as two 32-token chains, keys as one
// 64-key tile, every operand loaded from the fp32 Q / K / V^T layouts straight into MFMA fragment
// registers and split into bf16 hi + lo (no LDS: a row's tile is read by one wave only).  Exact single-
// tile softmax (row max over the T valid keys), S^T and O^T on three split products each
// (v_mfma_f32_32x32x16_bf16), row sums in fp32 on the VALU.  Keys >= T are masked (K / V padding rows
// are never written by the projection: V is zeroed in registers so p = 0 never meets NaN).
__global__ __launch_bounds__(256, 2) void attn_feat3_kernel(const AttnArgs p, int nrows) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int pair = blockIdx.x * 4 + wave;  // (row, head)
  if (pair >= nrows * p.H) return;         // wave-uniform; no barrier follows
  const int b = pair / p.H, h = pair - b * p.H;
  const int T = p.nk;
  const float* Q = (const float*)p.q + b * p.q_bstride + h * p.q_hstride;
  const float* Kg = (const float*)p.k + b * p.kv_bstride + h * p.kv_hstride;
  const float* Vg = (const float*)p.vt + b * p.kv_bstride + h * p.kv_hstride;
  const float c = kLog2e * 0.17677669529663687f;  // log2(e)/sqrt(32)

  // K (A operand of S^T = K Q^T): lane row 32u + r, dims 16ks + 8hh .. +7; V^T (A operand of O^T = V^T P^T):
  // lane dim r, keys kb .. kb+3, kb+8 .. kb+11 with kb = 32u + 16sp + 4hh (the P^T register order)
  bf16x8 kh[2][2], kl[2][2], vh[2][2], vl[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int key = 32 * u + r;
    const float* kr = Kg + (int64_t)min(key, T - 1) * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      split8v(*(const f32x4*)(kr + 16 * ks + 8 * hh), *(const f32x4*)(kr + 16 * ks + 8 * hh + 4), kh[u][ks], kl[u][ks]);
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      const int kb = 32 * u + 16 * sp + 4 * hh;
      const float* vr = Vg + (int64_t)r * p.kpad;
      f32x4 a = kb < T ? *(const f32x4*)(vr + kb) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 e = kb + 8 < T ? *(const f32x4*)(vr + kb + 8) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kb + j >= T) a[j] = 0.f;
        if (kb + 8 + j >= T) e[j] = 0.f;
      }
      split8v(a, e, vh[u][sp], vl[u][sp]);
    }
  }
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    const int t = 32 * ch + r;
    if (32 * ch >= T) break;  // wave-uniform
    bf16x8 qh[2], ql[2];
    const float* qr = Q + (int64_t)min(t, T - 1) * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f32x4 a = *(const f32x4*)(qr + 16 * ks + 8 * hh), e = *(const f32x4*)(qr + 16 * ks + 8 * hh + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] *= c, e[i] *= c;
      split8v(a, e, qh[ks], ql[ks]);
    }
    f32x16 st[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const f32x16 z = {};
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[u][0], qh[0], z, 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[u][1], qh[1], st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][0], ql[0], st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][1], ql[1], st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][0], qh[0], st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][1], qh[1], st[u], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (32 * u + (i & 3) + 8 * (i >> 2) + 4 * hh >= T) st[u][i] = -INFINITY;
    }
    float m = fmaxf(st[0][0], st[1][0]);
#pragma unroll
    for (int i = 1; i < 16; ++i) m = fmaxf(m, fmaxf(st[0][i], st[1][i]));
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
      m = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    float l = 0.f;
    f32x16 o = {};
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        f32x4 pa, pc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pa[j] = exp2f(st[u][8 * sp + j] - m);
          pc[j] = exp2f(st[u][8 * sp + 4 + j] - m);
          l += pa[j] + pc[j];
        }
        bf16x8 ph, pl;
        split8v(pa, pc, ph, pl);
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl[u][sp], ph, o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh[u][sp], pl, o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh[u][sp], ph, o, 0, 0, 0);
      }
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
      l = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    if (t < T) {
      const float inv = 1.0f / l;
      float* orow = (float*)p.o + (b * p.o_bstride + (int64_t)t * p.o_qstride) * (p.H * 32) + h * 32;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *(f32x4*)(orow + 8 * gq + 4 * hh) =
            f32x4{o[4 * gq] * inv, o[4 * gq + 1] * inv, o[4 * gq + 2] * inv, o[4 * gq + 3] * inv};
    }
  }
}

// ------------------------------------------------------------------ item attention, parity mode
// PREC_F32: the bf16 kernel's task map (attention_pipe.hip) and fixed-reference softmax on fp32 Q / K / V^T, every
// operand split into bf16 hi + lo planes (x = hi + lo to 2^-17): Q in registers, K / V^T as they are
// staged into LDS (two planes per image), and P = exp2(S) in registers.  Per 64-key tile and chain
//   S^T = Kl Qh + Kh Ql + Kh Qh          (6 x v_mfma_f32_32x32x16_bf16 per 32 keys)
//   O^T += Vl Ph + Vh Pl + Vh Ph,  l += 1.(Pl + Ph)  (selector MFMAs over both P planes)
// in fp32 accumulators: each product carries the operands to 2^-16, so the attention matches the
// exact fp32 softmax to ~1e-5 relative at three bf16 MFMAs where fp32-input MFMA takes sixteen.
// Output O is fp32 ([row][H*32], the out-projection's A).
// LDS images of a 64-key tile (unpadded, XOR-swizzled 16-B chunks; conflict-free ds_read_b128 for the
// four 16-lane groups of a wave):
//   K   [64 keys][32 d]  64-B rows : chunk c of row k at k*64 + 16*(c ^ ((k >> 2) & 3))
//   V^T [32 d][64 keys] 128-B rows : chunk c of row d at d*128 + 16*(c ^ ((d >> 1) & 7)), keys inside every
//        16-key group stored in the order 0-3, 8-11, 4-7, 12-15 so that the keys one lane owns in the S^T
//        accumulator (4hh + {0-3, 8-11}) are one 16-B chunk
constexpr int A2_KT = 64;
__device__ __forceinline__ int a2_koff(int row, int c) { return row * 64 + 16 * (c ^ ((row >> 2) & 3)); }
__device__ __forceinline__ int a2_voff(int d, int c) { return d * 128 + 16 * (c ^ ((d >> 1) & 7)); }
constexpr int A3_NCH = 2;
constexpr int A3_QPW = 32 * A3_NCH;
constexpr int A3_QPB = 4 * A3_QPW;
constexpr int A3_STAGE = 4 * 4096;  // K hi | K lo | V^T hi | V^T lo

__device__ __forceinline__ void a3_split8(f32x4 a, f32x4 b, float sc, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x = a[i] * sc, y = b[i] * sc;
    hi[i] = (bf16)x, hi[4 + i] = (bf16)y;
    lo[i] = (bf16)(x - (float)hi[i]), lo[4 + i] = (bf16)(y - (float)hi[4 + i]);
  }
}

// exact two-pass softmax for one query per lane, fp32 K / V^T straight from global memory
__device__ __attribute__((noinline)) void a3_exact_rows(const Attn2Args& p, const float* Kg, const float* Vg,
                                                         const float* qrow, float* orow, bool valid, float c) {
  float q[32], o[32];
#pragma unroll
  for (int d = 0; d < 32; ++d) q[d] = qrow[d] * c, o[d] = 0.f;
  float m = -INFINITY;
  for (int k = 0; k < p.nk; ++k) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) s = fmaf(q[d], Kg[(int64_t)k * 32 + d], s);
    m = fmaxf(m, s);
  }
  float l = 0.f;
  for (int k = 0; k < p.nk; ++k) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) s = fmaf(q[d], Kg[(int64_t)k * 32 + d], s);
    const float e = exp2f(s - m);
    l += e;
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] = fmaf(e, Vg[(int64_t)d * p.Npad + k], o[d]);
  }
  if (valid) {
    const float inv = 1.0f / l;
#pragma unroll
    for (int d = 0; d < 32; d += 4) *(f32x4*)(orow + d) = f32x4{o[d] * inv, o[d + 1] * inv, o[d + 2] * inv, o[d + 3] * inv};
  }
}

// CHEAP: the measured precision budget of DESIGN 5.7 as an opt-in (the launcher picks it when the sequence has
// >= x3_cheap_min_keys keys, default never; profiles/r06/parity_n0_sweep_form*.txt): bit 0, S = K Q^T on ONE fp16 product (Q, K
// rounded to fp16); bit 1, P.V on two products (P rounded to bf16 once, V split: Vl Ph + Vh Ph) and the row sums over
// that same Ph.  CHEAP = 0: every operand split (three products each).
template <int CHEAP>
__global__ __launch_bounds__(256, 2) void attn_item3_kernel(const Attn2Args p) {
  constexpr bool CS = (CHEAP & 1) != 0, CPV = (CHEAP & 2) != 0;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2][A3_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;

  int b, g, chunk;  // task map of attn_pipe_kernel (contiguous task ranges per XCD)
  {
    const int nbk = p.nblocks, pid = blockIdx.x;
    const int xcd = pid & 7, slot = pid >> 3;
    const int task = xcd * (nbk >> 3) + min(xcd, nbk & 7) + slot;
    b = task / p.tasks_per_b;
    const int rem = task - b * p.tasks_per_b;
    g = 0;
    int base = p.tstart[0];
#pragma unroll
    for (int h = 1; h < 9; ++h)
      if (h < p.H && p.tstart[h] <= rem) g = h, base = p.tstart[h];
    chunk = rem - base;
  }
  const int cnt = p.na + (g == p.kvb ? p.H * p.nb : 0);
  const int jw = chunk * A3_QPB + wave * A3_QPW;
  const bool active = jw < cnt;

  const int64_t kvoff = (int64_t)b * p.kv_bstride + (int64_t)g * p.Npad * 32;
  const float* Kg = (const float*)p.k + kvoff;
  const float* Vg = (const float*)p.vt + kvoff;
  const float c = p.q_prescaled ? 1.0f : kLog2e * 0.17677669529663687f;  // log2(e)/sqrt(32)

  int qh[A3_NCH], qsrow[A3_NCH];
  bool qok[A3_NCH];
  bf16x8 qfh[A3_NCH][2], qfl[A3_NCH][2];
  f16x8 qf16[A3_NCH][2];
#pragma unroll
  for (int qb = 0; qb < A3_NCH; ++qb) {
    const int j = jw + 32 * qb + r;
    qok[qb] = j < cnt;
    const int jc = min(j, cnt - 1);
    if (jc < p.na) {
      qh[qb] = g, qsrow[qb] = p.a0 + jc;
    } else {
      const int jj = jc - p.na;
      qh[qb] = jj / p.nb, qsrow[qb] = p.b0 + jj % p.nb;
    }
    const float* qrow = (const float*)p.q + (((int64_t)b * p.H + qh[qb]) * p.S + qsrow[qb]) * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const f32x4 a = *(const f32x4*)(qrow + 16 * ks + 8 * hh), e = *(const f32x4*)(qrow + 16 * ks + 8 * hh + 4);
      if constexpr (CS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) qf16[qb][ks][i] = (_Float16)(a[i] * c), qf16[qb][ks][4 + i] = (_Float16)(e[i] * c);
      } else {
        a3_split8(a, e, c, qfh[qb][ks], qfl[qb][ks]);
      }
    }
  }

  const int ntiles = (p.nk + A2_KT - 1) / A2_KT;
  const bool partial = (p.nk % A2_KT) != 0;

  // staging: 8 fp32 of one K row and 8 fp32 of one V^T row per thread and tile
  const int krow = tid >> 2, kc = tid & 3;
  const int vd = tid >> 3, vc = tid & 7;
  f32x4 rk[2], rv[2];
  auto gload = [&](int t) __attribute__((always_inline)) {
    const int k0 = t * A2_KT;
    const float* ks = Kg + (int64_t)(k0 + krow) * 32 + kc * 8;
    const float* vs = Vg + (int64_t)vd * p.Npad + k0 + vc * 8;
    rk[0] = *(const f32x4*)ks, rk[1] = *(const f32x4*)(ks + 4);
    rv[0] = *(const f32x4*)vs, rv[1] = *(const f32x4*)(vs + 4);
    if (partial && t == ntiles - 1) {  // keys >= nk: V = 0 so that p = 0 never meets NaN / inf padding
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + vc * 8 + j >= p.nk) rv[j >> 2][j & 3] = 0.f;
    }
  };
  const int koff_w = a2_koff(krow, kc);
  const int voff_w0 = a2_voff(vd, vc & ~1) + 8 * (vc & 1), voff_w1 = a2_voff(vd, vc | 1) + 8 * (vc & 1);
  auto lstore = [&](int buf) __attribute__((always_inline)) {
    unsigned char* Ks = lds[buf];
    bf16x8 hi, lo;
    if constexpr (CS) {  // K in fp16, one plane
      f16x8 kk;
#pragma unroll
      for (int i = 0; i < 4; ++i) kk[i] = (_Float16)rk[0][i], kk[4 + i] = (_Float16)rk[1][i];
      *(f16x8*)(Ks + koff_w) = kk;
    } else {
      a3_split8(rk[0], rk[1], 1.0f, hi, lo);
      *(bf16x8*)(Ks + koff_w) = hi;
      *(bf16x8*)(Ks + 4096 + koff_w) = lo;
    }
    a3_split8(rv[0], rv[1], 1.0f, hi, lo);
    const u32x4 vh = __builtin_bit_cast(u32x4, hi), vl = __builtin_bit_cast(u32x4, lo);
    *(u32x2*)(Ks + 8192 + voff_w0) = u32x2{vh.x, vh.y};
    *(u32x2*)(Ks + 8192 + voff_w1) = u32x2{vh.z, vh.w};
    *(u32x2*)(Ks + 12288 + voff_w0) = u32x2{vl.x, vl.y};
    *(u32x2*)(Ks + 12288 + voff_w1) = u32x2{vl.z, vl.w};
  };
  int kro[2][2], vro[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      kro[u][i] = a2_koff(32 * u + r, 2 * i + hh);
      vro[u][i] = 8192 + a2_voff(r, 2 * (2 * u + i) + hh);
    }
  bf16x8 sel;  // row-sum selector (attn_pipe_kernel)
  {
    const int m = lane & 15, kg = lane >> 4;
    const bool one = (m == 0 && (kg & 1) == 0) || (m == 1 && (kg & 1) == 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) sel[j] = (bf16)(one ? 1.0f : 0.0f);
  }
  f32x16 o[A3_NCH];
  f32x4 lacc[A3_NCH];
  float mref[A3_NCH];
#pragma unroll
  for (int qb = 0; qb < A3_NCH; ++qb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) o[qb][i] = 0.f;
    lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    mref[qb] = 0.f;
  }

  auto tile = [&](int it, auto maskc, auto firstc, auto refc) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(maskc)::value;
    constexpr bool FIRST = decltype(firstc)::value;
    constexpr bool REF = decltype(refc)::value;
    const f32x16 zero16 = {};
    const int k0 = it * A2_KT;
    if (it + 1 < ntiles) gload(it + 1);
    const unsigned char* Ks = lds[it & 1];
    if (active) {
      bf16x8 kh[2][2], kl[2][2], vh[2][2], vl[2][2];
      f16x8 k16[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr (CS) {
            k16[u][i] = *(const f16x8*)(Ks + kro[u][i]);
          } else {
            kh[u][i] = *(const bf16x8*)(Ks + kro[u][i]);
            kl[u][i] = *(const bf16x8*)(Ks + 4096 + kro[u][i]);
          }
          vh[u][i] = *(const bf16x8*)(Ks + vro[u][i]);
          vl[u][i] = *(const bf16x8*)(Ks + 4096 + vro[u][i]);
        }
      f32x16 s[A3_NCH][2];
#pragma unroll
      for (int qb = 0; qb < A3_NCH; ++qb)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if constexpr (CS) {
            s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k16[u][0], qf16[qb][0], zero16, 0, 0, 0);
            s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(k16[u][1], qf16[qb][1], s[qb][u], 0, 0, 0);
            continue;
          }
          s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[u][0], qfh[qb][0], zero16, 0, 0, 0);
          s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl[u][1], qfh[qb][1], s[qb][u], 0, 0, 0);
          s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][0], qfl[qb][0], s[qb][u], 0, 0, 0);
          s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][1], qfl[qb][1], s[qb][u], 0, 0, 0);
          s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][0], qfh[qb][0], s[qb][u], 0, 0, 0);
          s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh[u][1], qfh[qb][1], s[qb][u], 0, 0, 0);
        }
      if constexpr (MASK) {
#pragma unroll
        for (int qb = 0; qb < A3_NCH; ++qb)
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (k0 + 32 * u + (i & 3) + 8 * (i >> 2) + 4 * hh >= p.nk) s[qb][u][i] = -INFINITY;
      }
      if constexpr (FIRST) {
#pragma unroll
        for (int qb = 0; qb < A3_NCH; ++qb) {
          float m = fmaxf(s[qb][0][0], s[qb][1][0]);
#pragma unroll
          for (int i = 1; i < 16; ++i) m = fmaxf(m, fmaxf(s[qb][0][i], s[qb][1][i]));
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
          mref[qb] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        }
      }
      if constexpr (REF) {
#pragma unroll
        for (int qb = 0; qb < A3_NCH; ++qb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            s[qb][0][i] -= mref[qb];
            s[qb][1][i] -= mref[qb];
          }
      }
#pragma unroll
      for (int qb = 0; qb < A3_NCH; ++qb)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) {
            bf16x8 ph, pl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float e = __builtin_amdgcn_exp2f(s[qb][u][8 * sp + j]);
              ph[j] = (bf16)e;
              if constexpr (!CPV) pl[j] = (bf16)(e - (float)ph[j]);
            }
            if constexpr (CPV) {
              o[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl[u][sp], ph, o[qb], 0, 0, 0);
              o[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh[u][sp], ph, o[qb], 0, 0, 0);
              lacc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, ph, lacc[qb], 0, 0, 0);
              continue;
            }
            o[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl[u][sp], ph, o[qb], 0, 0, 0);
            o[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh[u][sp], pl, o[qb], 0, 0, 0);
            o[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh[u][sp], ph, o[qb], 0, 0, 0);
            lacc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pl, lacc[qb], 0, 0, 0);
            lacc[qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, ph, lacc[qb], 0, 0, 0);
          }
    }
    if (it + 1 < ntiles) lstore((it + 1) & 1);
    __syncthreads();
  };

  gload(0);
  lstore(0);
  __syncthreads();
  using Y = std::true_type;
  using N = std::false_type;
  auto pass = [&](auto wmc) __attribute__((always_inline)) {
    constexpr bool WM = decltype(wmc)::value;
    using F = std::integral_constant<bool, WM>;
    if (ntiles == 1) {
      if (partial) tile(0, Y{}, F{}, F{});
      else tile(0, N{}, F{}, F{});
    } else {
      tile(0, N{}, F{}, F{});
      const int nfull = p.nk / A2_KT;
      for (int it = 1; it < nfull; ++it) tile(it, N{}, N{}, F{});
      if (partial) tile(nfull, Y{}, N{}, F{});
    }
  };
  auto rowsum = [&](int qb) __attribute__((always_inline)) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(lacc[qb][0]), __float_as_uint(lacc[qb][1]),
                                                    false, false);
    const auto s2 = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);
    return __uint_as_float(s2[0]);
  };
  pass(N{});
  {  // reference-free pass out of [2^-60, 2^100) for any query of the block: re-run with the first tile's max
    bool bad = false;
    if (active)
#pragma unroll
      for (int qb = 0; qb < A3_NCH; ++qb) {
        const unsigned lb = __float_as_uint(rowsum(qb)) & 0x7fffffffu;
        bad |= lb >= 0x71800000u || lb < 0x21800000u;
      }
    if (__syncthreads_or(bad ? 1 : 0)) {
#pragma unroll
      for (int qb = 0; qb < A3_NCH; ++qb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) o[qb][i] = 0.f;
        lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      gload(0);
      lstore(0);
      __syncthreads();
      pass(Y{});
    }
  }
  if (!active) return;
#pragma unroll
  for (int qb = 0; qb < A3_NCH; ++qb) {
    const float ls = rowsum(qb);
    float* orow = (float*)p.o + ((int64_t)b * p.S + qsrow[qb]) * (p.H * 32) + qh[qb] * 32;
    if (__any((__float_as_uint(ls) & 0x7fffffffu) >= 0x71800000u)) {
      const float* qrow = (const float*)p.q + (((int64_t)b * p.H + qh[qb]) * p.S + qsrow[qb]) * 32;
      a3_exact_rows(p, Kg, Vg, qrow, orow, qok[qb] && hh == 0, c);
      continue;
    }
    const float inv = 1.0f / ls;
    if (qok[qb]) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *(f32x4*)(orow + 8 * gq + 4 * hh) = f32x4{o[qb][4 * gq] * inv, o[qb][4 * gq + 1] * inv,
                                                  o[qb][4 * gq + 2] * inv, o[qb][4 * gq + 3] * inv};
    }
  }
}

}  // namespace


namespace {
// parity mode: key count from which the item attention takes a cheap form (attn_item3_kernel<1..3>: fp16 S and / or
// two-product P.V).  Off by default (-1): the sweep of logits error against N on the golden models
// (profiles/r06/parity_n0_sweep_form{1,2,3}.txt, N = 40 .. 1838) found no N from which either form stays 2x under the
// 1e-4 contract (fp16 S: ~1e-4 at every N; two-product P.V: 4.3e-4 at N = 40 falling to 5.8e-5 at 1838), so the
// cheap forms are an opt-in throughput mode (mmpfn_set_parity_attention_min_keys)
#ifndef X3_CHEAP_MIN_KEYS
#define X3_CHEAP_MIN_KEYS (-1)
#endif
#ifndef X3_CHEAP_FORM
#define X3_CHEAP_FORM 3
#endif
std::atomic<int> g_x3_cheap_min_keys{X3_CHEAP_MIN_KEYS};
std::atomic<int> g_x3_cheap_form{X3_CHEAP_FORM};  // attn_item3_kernel's CHEAP bits on those sequences

hipError_t launch_item_attention(const void* q, const void* k, const void* vt, void* out, int S, int T, int H,
                                 int Npad, int nk, int a0, int na, int b0, int nb, int kvb, hipStream_t st,
                                 int64_t kv_bstride, bool q_prescaled, bool x3, const void* vt8 = nullptr,
                                 int f8 = 0, bool qk_f16 = false, bool o_f16 = false) {
  if (na + nb <= 0 || T <= 0) return hipSuccess;
  if (nk <= 0 || Npad % A2_KT != 0 || nk > Npad || H > 8 || H <= 0) return hipErrorInvalidValue;
  if (nb > 0 && (kvb < 0 || kvb >= H)) return hipErrorInvalidValue;
  Attn2Args a;
  a.q = (const bf16*)q, a.k = (const bf16*)k, a.vt = (const bf16*)vt, a.o = (bf16*)out;
  a.S = S, a.H = H, a.Npad = Npad, a.nk = nk;
  a.a0 = a0, a.na = na, a.b0 = b0, a.nb = nb, a.kvb = nb > 0 ? kvb : -1;
  a.kv_bstride = kv_bstride > 0 ? kv_bstride : (int64_t)H * Npad * 32;
  a.q_prescaled = q_prescaled ? 1 : 0;
  a.vt8 = (const unsigned char*)vt8, a.f8 = x3 ? 0 : f8;
  a.qk_f16 = (!x3 && qk_f16) ? 1 : 0;
  a.o_f16 = (!x3 && (qk_f16 || o_f16)) ? 1 : 0;
  if (kv_bstride > 0 && (na > 0 || kvb != 0)) return hipErrorInvalidValue;  // cache layout holds head 0 only
  const int qpb = x3 ? A3_QPB : ATTN_ITEM_QPB;
  int acc = 0;
  for (int g = 0; g < H; ++g) {
    a.tstart[g] = acc;
    const int cnt = na + (g == a.kvb ? H * nb : 0);
    acc += (cnt + qpb - 1) / qpb;
  }
  for (int g = H; g < 9; ++g) a.tstart[g] = acc;
  a.tasks_per_b = acc;
  a.nblocks = acc * T;
  if (a.nblocks == 0) return hipSuccess;
  if (x3) {
    // the budget's cheap forms only on sequences long enough to average their rounding (x3_cheap_min_keys)
    const int mk = g_x3_cheap_min_keys.load(std::memory_order_relaxed);
    const int form = mk >= 0 && nk >= mk ? g_x3_cheap_form.load(std::memory_order_relaxed) : 0;
    if (form == 1) hipLaunchKernelGGL(attn_item3_kernel<1>, dim3(a.nblocks), dim3(256), 0, st, a);
    else if (form == 2) hipLaunchKernelGGL(attn_item3_kernel<2>, dim3(a.nblocks), dim3(256), 0, st, a);
    else if (form == 3) hipLaunchKernelGGL(attn_item3_kernel<3>, dim3(a.nblocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(attn_item3_kernel<0>, dim3(a.nblocks), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  return launch_attn_pipe(a, st);
}

}  // namespace

hipError_t launch_attn_layer(const void* q, const void* k, const void* vt, void* out, int S, int T, int H, int Npad,
                             int nk, int a0, int na, int b0, int nb, int kvb, hipStream_t st, int64_t kv_bstride,
                             bool q_prescaled, const void* vt8, int f8, bool qk_f16, bool o_f16) {
  return launch_item_attention(q, k, vt, out, S, T, H, Npad, nk, a0, na, b0, nb, kvb, st, kv_bstride, q_prescaled,
                               false, vt8, f8, qk_f16, o_f16);
}

int set_x3_cheap_min_keys(int n, int form) {
  if (form >= 1 && form <= 3) g_x3_cheap_form.store(form);
  return g_x3_cheap_min_keys.exchange(n);
}

hipError_t launch_attn_item3(const void* q, const void* k, const void* vt, void* out, int S, int T, int H, int Npad,
                             int nk, int a0, int na, int b0, int nb, int kvb, hipStream_t st, int64_t kv_bstride) {
  return launch_item_attention(q, k, vt, out, S, T, H, Npad, nk, a0, na, b0, nb, kvb, st, kv_bstride, false, true);
}

hipError_t launch_attn(const AttnArgs& a, int batches, int prec, int nw, hipStream_t st) {
  if (a.nq <= 0 || batches <= 0) return hipSuccess;
  if (prec == PREC_F32 && nw == 1 && a.s0 == 0 && a.nq == a.nk && a.nk <= 64 && a.kvh_fixed < 0) {
    // parity-mode feature attention: one wave per (row, head), operands straight to registers
    if (a.kpad % 4 != 0) return hipErrorInvalidValue;
    const int pairs = batches * a.H;
    hipLaunchKernelGGL(attn_feat3_kernel, dim3((pairs + 3) / 4), dim3(256), 0, st, a, batches);
    return hipGetLastError();
  }
  if (a.nk <= 0 || a.kpad % IA_KT != 0 || a.nk > a.kpad) return hipErrorInvalidValue;
  if (nw != 1 && nw != 4) return hipErrorInvalidValue;
  dim3 grid((a.nq + 32 * nw - 1) / (32 * nw), a.H, batches);
  if (prec == PREC_BF16) {
    if (nw == 4) hipLaunchKernelGGL((attn_item_kernel<1, 4>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_item_kernel<1, 1>), grid, dim3(64), 0, st, a);
  } else if (prec == PREC_F32) {  // parity mode: split-bf16 products (the feature attention's path)
    if (nw == 4) hipLaunchKernelGGL((attn_item_kernel<2, 4>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_item_kernel<2, 1>), grid, dim3(64), 0, st, a);
  } else {
    if (nw == 4) hipLaunchKernelGGL((attn_item_kernel<0, 4>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_item_kernel<0, 1>), grid, dim3(64), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_attn_item(const void* q, const void* k, const void* vt, void* out, int S, int T, int H, int Npad,
                            int s0, int nq, int nk, int kv_head_fixed, int prec, hipStream_t st, int64_t kv_bstride) {
  AttnArgs a;
  a.q = q, a.k = k, a.vt = vt, a.o = out;
  a.q_bstride = (int64_t)H * S * 32, a.q_hstride = (int64_t)S * 32;
  a.kv_bstride = kv_bstride > 0 ? kv_bstride : (int64_t)H * Npad * 32, a.kv_hstride = (int64_t)Npad * 32;
  a.kpad = Npad;
  if (kv_bstride > 0 && kv_head_fixed != 0) return hipErrorInvalidValue;
  a.o_bstride = S, a.o_qstride = 1;
  a.s0 = s0, a.nq = nq, a.nk = nk, a.kvh_fixed = kv_head_fixed, a.H = H;
  if (prec == PREC_BF16 || prec == PREC_F32) {
    const bool x3 = prec == PREC_F32;
    if (kv_head_fixed < 0)
      return launch_item_attention(q, k, vt, out, S, T, H, Npad, nk, s0, nq, 0, 0, -1, st, kv_bstride, false, x3);
    return launch_item_attention(q, k, vt, out, S, T, H, Npad, nk, 0, 0, s0, nq, kv_head_fixed, st, kv_bstride, false,
                                 x3);
  }
  return launch_attn(a, T, prec, 4, st);
}

}  // namespace mmpfn
