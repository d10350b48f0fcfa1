// Software-pipelined sample-axis attention for gfx950 (bf16): the item attention of one layer
// (layer.py:341-379 attn_between_items; multi_head_attention.py:693-729) in ONE launch per layer: the
// train rows against their own head's K/V (layer.py:362-372) and the test rows of all heads against
// head 0's K/V (multiquery_item_attention_for_test_set, layer.py:344-358), re-shaped against the SIMD's
// issue model.
//
// At head dim 32 a 64x64 score tile of one wave costs 512 matrix-pipe cycles (16 MFMA-32) but
// 64 v_exp_f32 (8 issue cycles each) + 32 v_cvt_pk_bf16_f32 + the MFMAs' issue holds: the SIMD's
// issue port, not its matrix pipe, binds (~850 cycles per tile-wave).  Round 2's kernel left the two
// waves of a SIMD to overlap that mix (measured ~1.5x the floor: each wave's exps wait on its own
// S MFMAs, its P.V MFMAs on its own conversions).  Here:
//  * inside each wave a three-stage pipeline over (tile, 32-query chain) units:
//    while the exps / conversions of unit j issue, the matrix pipe runs the S MFMAs of unit j+1
//    and the P.V + row-sum MFMAs of unit j-1 -- nothing in a step waits on anything of the same
//    step, and the step is one basic block whose order is pinned by sched_group_barrier;
//  * K / V^T tiles staged once per block in a four-slot LDS ring, the fragments read a step ahead of
//    their MFMAs into two rotating register sets, one s_barrier per tile.  bf16 V^T: by LDS-DMA (each
//    wave one 1-KB K piece and one V^T piece per tile, issued three tiles ahead into XOR-swizzled unpadded
//    slots, the barrier waiting only for the pieces of the tile the next step reads; 3 % faster than
//    register staging); e4m3 V^T: register staging (one 16-B K and one 8-B V^T chunk per
//    thread, written a tile ahead into padded slots);
//  * K rows are read in a permuted order (bits 2 and 3 of the row swapped), so the 8 keys a lane's
//    P fragment holds are 8 consecutive keys: one 16-B V^T read per fragment, no permuted V^T image.
// Softmax: fixed reference 0 (Q carries log2(e)/sqrt(32)), p = exp2(s), row
// sums on the MFMA pipe through a 0/1 selector, the sum range-checked per wave ([2^-60, 2^100)),
// a wave out of range re-running with the first tile's row max, and an exact two-pass backstop.
//
// F8 variants (config E's "fp8 MFMA path", BASELINE.json configs[4]; opt-in): P.V and the row sums on the
// block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 / _16x16x128_ (one MFMA each per chain and 64-key tile
// instead of 4 + 4: 12 instead of 24 MFMA issue holds per tile-wave), V^T in e4m3 (converted once after
// the projection, launch_vt_fp8), P in e4m3 (F8 = 1) or e5m2 (F8 = 2).  S = K Q^T stays bf16.  fp8 has no
// room for the fixed reference 0, so each query gets a power-of-two conversion scale from its first key
// tile's max (the first tile's max lands at 2^ETOP); a later score beyond the format's range converts to
// NaN / inf, which the row-sum check catches, and the wave re-runs on the exact bf16 path.
//
// QF16: Q / K in fp16, so S = K Q^T runs on v_mfma_f32_32x32x16_f16; OF16: the output O in fp16 (the fp16 mode's
// state); V^T and P stay bf16 (P = exp2(s) under the fixed reference needs bf16's exponent range).  The fp16
// mode's forward runs <F8, false, true> -- Q / K in bf16, so every MFMA of the loop is a bf16 one: with fp16 S
// MFMAs between the bf16 P.V / row-sum MFMAs the same launch took 1.7 % longer on identical operand bits
// (DESIGN 5.7); the kernel-level tap with fp16 Q / K (mmpfn_item_attention_layer_ex codes 5-7) runs <F8, true, true>.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

#ifdef MMPFN_STAMPS  // per-phase cycle stamps (diagnostics build only: make dbg; tools/attn_stamps.py)
// 8 consecutive blocks from the grid's middle (consecutive block ids sit on the 8 XCDs), their 4 waves, AP_NST stamps
// each (s_memtime, shader cycles): 0 kernel start, 1 Q fragments loaded, 2 prologue barrier passed (tiles 0-1 in
// LDS), 3 + t after step t's barrier (t < AP_NST - 6), AP_NST - 3 after the loop's drain, AP_NST - 2 after the
// row-sum check (and any re-run), AP_NST - 1 after the output stores
constexpr int AP_NST = 48;
__device__ unsigned long long g_ap_stamps[8 * 4 * AP_NST];
__device__ int g_ap_meta[4];  // gridDim.x, ntiles of the first stamped block, the first stamped block id
#define AP_STAMP(k)                                                                                     \
  do {                                                                                                  \
    const int sb_ = (int)blockIdx.x - (int)(gridDim.x / 2);                                            \
    if (sb_ >= 0 && sb_ < 8 && lane == 0) g_ap_stamps[(sb_ * 4 + wave) * AP_NST + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#elif defined(MMPFN_STAMPS_ALL)  // every wave of the grid: HW_ID, XCC_ID and 36 stamps (diagnostics only)
constexpr int AP_NST = 36, AP_MAXB = 8192;
__device__ unsigned long long g_ap_all[AP_MAXB * 4 * (AP_NST + 2)];
#define AP_STAMP(k)                                                                                     \
  do {                                                                                                  \
    if (lane == 0 && blockIdx.x < AP_MAXB && (k) < AP_NST)                                              \
      g_ap_all[((size_t)blockIdx.x * 4 + wave) * (AP_NST + 2) + 2 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define AP_STAMP(k) \
  do {              \
  } while (0)
#endif

constexpr int P4_KT = 64;    // keys per tile
constexpr int P4_NCH = 2;    // 32-query chains per wave
constexpr int P4_QPW = 32 * P4_NCH;
constexpr int P4_QPB = 4 * P4_QPW;
static_assert(P4_QPB == ATTN_ITEM_QPB, "launch_item_attention's task size");

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) short s16x2;

// fp8 P formats: conversion, MFMA operand format code, where the first tile's max lands (2^ETOP), the
// smallest power of two the format still holds (subnormal) and the underflow guard UFLOW = 2^(EMIN + 6): a
// scaled P' below 2^(EMIN-1) converts to 0 and every subnormal is off by at most that much, so a row's fp8 sum
// L is within nk 2^(EMIN-1) of the sum it stands for; L < nk UFLOW (more than 2^-7 of it possibly lost to the
// format's floor: one large key in the first tile over many keys ~10 octaves below) re-runs the
// wave on the exact bf16 path like an overflow does
template <int F8> struct P8;
// e4m3's ETOP balances the two re-run causes on random q / k (round 6; a CPU model of the kernel's per-query scale
// over N = 1838 / 10 000): 0 sent 94-100 % of the waves back through the underflow guard, 4 sent 25-100 %
// through overflow of the later tiles' maxima; 2 re-runs 16-19 %
#ifndef P8_E4_ETOP
#define P8_E4_ETOP 2
#endif
template <> struct P8<1> {  // e4m3 (max 448 = 2^8.8): >= 6.8 octaves of headroom, 11 below the first max
  static constexpr int FMT = 0, ETOP = P8_E4_ETOP, EMIN = -9, EMAX = 8;
  static constexpr float UFLOW = 0x1p-3f;
  static __device__ __forceinline__ s16x2 cvt(s16x2 old, float a, float b, float sc, bool hi) {
    return hi ? __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(old, a, b, sc, true)
              : __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(old, a, b, sc, false);
  }
};
template <> struct P8<2> {  // e5m2 (max 57344 = 2^15.8): >= 8.8 octaves of headroom, 22 below
  static constexpr int FMT = 1, ETOP = 6, EMIN = -16, EMAX = 15;
  static constexpr float UFLOW = 0x1p-10f;
  static __device__ __forceinline__ s16x2 cvt(s16x2 old, float a, float b, float sc, bool hi) {
    return hi ? __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(old, a, b, sc, true)
              : __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(old, a, b, sc, false);
  }
};

// sched_group_barrier masks (LLVM AMDGPU IGroupLP)
constexpr int SG_VALU = 0x2, SG_MFMA = 0x8, SG_VMEM_READ = 0x20, SG_DS_READ = 0x100, SG_DS_WRITE = 0x200,
              SG_TRANS = 0x400;

// K / V^T staging of the bf16-V^T kernels by LDS-DMA (no staging registers, no ds_write), 0: register staging
#ifndef P4_DMA
#define P4_DMA 1
#endif
// "m0" in the clobber list: clang keeps m0 reserved and ignores the entry (-Winline-asm; the ISA is identical with
// and without it), and every m0 use the compiler emits itself is preceded by its own write -- test_codegen checks
// that no m0 read other than these DMA issues exists in the kernels
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void p4_dma16(uint32_t voff, const void* sbase, unsigned lds_dst) {
  // m0 = the wave's LDS destination; lane i's 16 B (sbase + voff) land at m0 + 16 i.  In inline asm so the
  // compiler's waitcnt pass adds no vmcnt(0) for it; the loop waits for its own pieces at the tile barrier
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// exact two-pass softmax for one query per lane, K / V^T straight from global memory (backstop)
template <typename QT, typename OT>
__device__ __attribute__((noinline)) void p4_exact_rows(const Attn2Args& p, const QT* Kg, const bf16* Vg,
                                                        const QT* qrow, OT* orow, bool valid, float c) {
  float q[32], o[32];
#pragma unroll
  for (int d = 0; d < 32; ++d) q[d] = (float)qrow[d] * c, o[d] = 0.f;
  float m = -INFINITY;
  for (int k = 0; k < p.nk; ++k) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) s = fmaf(q[d], (float)Kg[(int64_t)k * 32 + d], s);
    m = fmaxf(m, s);
  }
  float l = 0.f;
  for (int k = 0; k < p.nk; ++k) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < 32; ++d) s = fmaf(q[d], (float)Kg[(int64_t)k * 32 + d], s);
    const float e = exp2f(s - m);
    l += e;
#pragma unroll
    for (int d = 0; d < 32; ++d) o[d] = fmaf(e, (float)Vg[(int64_t)d * p.Npad + k], o[d]);
  }
  if (valid) {
    const float inv = 1.0f / l;
#pragma unroll
    for (int d = 0; d < 32; ++d) orow[d] = (OT)(o[d] * inv);
  }
}

template <int F8, bool QF16, bool OF16>
__global__ __launch_bounds__(256, 2) void attn_pipe_kernel(const Attn2Args p) {
  typedef typename Op16<QF16>::t QT;    // Q and K elements
  typedef typename Op16<QF16>::x8 Q8;
  typedef typename Op16<OF16>::t OT;    // O elements
  typedef typename Op16<OF16>::x4 O4;
  // LDS slot: K [64][32] bf16 in 80-B rows | V^T [32][64] in 144-B rows (bf16) or 80-B rows (e4m3);
  // DMA (bf16 V^T): K in 64-B rows | V^T in 128-B rows, unpadded and XOR-swizzled (see the fragments below)
  constexpr bool DMA = F8 == 0 && P4_DMA;
  constexpr int KROW = DMA ? 64 : 80;
  constexpr int VROW = F8 ? 80 : (DMA ? 128 : 144);
  constexpr int P4_SLOT_BYTES = 64 * KROW + 32 * VROW;
  __shared__ __attribute__((aligned(1024))) unsigned char ring[4 * P4_SLOT_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  AP_STAMP(0);
#ifdef MMPFN_STAMPS_ALL
  if (lane == 0 && blockIdx.x < AP_MAXB) {
    const size_t b0 = ((size_t)blockIdx.x * 4 + wave) * (AP_NST + 2);
    g_ap_all[b0] = __builtin_amdgcn_s_getreg(4 | (31 << 11));       // HW_REG_HW_ID
    g_ap_all[b0 + 1] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
  }
#endif

  // ---- task: the queries that read KV sequence (column b, kv head g) are the own-head rows [a0, a0+na)
  //      of head g, then, for g == kvb, rows [b0, b0+nb) of all H heads, cut into tasks of 256 (4 waves
  //      x 64); contiguous task ranges per XCD, so one KV sequence stays in one L2
  int b, g, chunk;
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
  const int jw = chunk * P4_QPB + wave * P4_QPW;
  const bool active = jw < cnt;  // wave-uniform; an idle wave only stages its share of every tile

  const int64_t kvoff = (int64_t)b * p.kv_bstride + (int64_t)g * p.Npad * 32;
  const QT* Kg = (const QT*)p.k + kvoff;
  const bf16* Vg = p.vt + kvoff;
  const unsigned char* Vg8 = p.vt8 + kvoff;  // F8: e4m3 V^T, same element layout
  const float c = kLog2e * 0.17677669529663687f;  // log2(e)/sqrt(32)

  // the lane's query of chain qb: head and table row (recomputed after the tile loop rather than kept live)
  struct QRow {
    int h, s;
    bool ok;
  };
  auto qrow_of = [&](int qb) __attribute__((always_inline)) {
    const int j = jw + 32 * qb + r;
    const int jc = min(j, cnt - 1);
    QRow q;
    q.ok = j < cnt;
    if (jc < p.na) {
      q.h = g, q.s = p.a0 + jc;
    } else {
      const int jj = jc - p.na;
      q.h = jj / p.nb, q.s = p.b0 + jj % p.nb;
    }
    return q;
  };
  Q8 qf[P4_NCH][2];
#pragma unroll
  for (int qb = 0; qb < P4_NCH; ++qb) {
    const QRow q = qrow_of(qb);
    const QT* qrow = (const QT*)p.q + (((int64_t)b * p.H + q.h) * p.S + q.s) * 32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const Q8 raw = *(const Q8*)(qrow + 16 * ks + 8 * hh);
      if (p.q_prescaled) {
        qf[qb][ks] = raw;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[qb][ks][e] = (QT)((float)raw[e] * c);
      }
    }
  }

  AP_STAMP(1);
  const int ntiles = (p.nk + P4_KT - 1) / P4_KT;
  const int nfull = p.nk / P4_KT;
#ifdef MMPFN_STAMPS
  if (blockIdx.x == gridDim.x / 2 && tid == 0) g_ap_meta[0] = gridDim.x, g_ap_meta[1] = ntiles, g_ap_meta[2] = blockIdx.x;
#endif
  const bool partial = nfull != ntiles;
  // key-tile order of the fast pass: the partial last tile first -- staged by the prologue with its keys
  // >= nk zeroed (K rows 0: s = 0, p = 1 exactly; V^T 0: nothing added to O) -- then tiles 0 .. nfull-1,
  // so every tile runs in the pipelined loop; each row sum then holds exactly npad extra ones
  const int poff = partial ? 1 : 0;
  auto tile_of = [&](int i) __attribute__((always_inline)) { return (partial && i == 0) ? nfull : i - poff; };

  // ---- fragments:
  //   K   A operand of S^T = K Q^T : lane (r, hh) <- K[key 32u + pk(r)][16ks + 8hh .. +7], pk swapping
  //       bits 2 and 3, so the S^T accumulator rows (i&3) + 8(i>>2) + 4hh of P fragment (u, sp) are the
  //       keys 32u + 16sp + 8hh + 0..7
  //   V^T A operand of O^T = V^T P^T: lane (r = d, hh) <- V^T[d][32u + 16sp + 8hh .. +7]
  const int pkr = (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1);
  // LDS ring: slot = K [64][32] in 80-B rows | V^T [32][64] in 144-B rows: the padded strides make the
  // ds_read_b128 of every 16-lane group conflict-free (row * 20 and d * 36 dwords are distinct mod 64
  // over 16 rows), and every fragment of a lane sits at one base + an immediate offset
  //   F8: V^T A operand of the 32x32x64 MFMA: lane (r = d, hh) <- V^T[d][logical k 32hh .. 32hh+31], logical
  //       k 32hh + 8j + b = key 16j + 8hh + b (the keys of the P bytes, see expc): an e4m3 V^T row is stored
  //       with key group g (8 keys) at byte 32 (g & 1) + 8 (g >> 1), so a lane reads 32 contiguous bytes
  //   DMA: the LDS-DMA writes a wave's 1 KB lane-linearly, so the padding goes and 16-B unit u of K row R sits at
  //       u ^ ((R >> 2) & 3), of V^T row d at u ^ ((d >> 1) & 7): the 16 rows of a ds_read_b128 lane group (16
  //       distinct rows mod 16, pk permuting only inside them) then cover all 16 16-B slots of the 256-B bank row
  constexpr int VBASE = 64 * KROW;
  const int kb = (32 * 0 + pkr) * KROW + 16 * hh, vb = VBASE + r * VROW + (F8 ? 32 : 16) * hh;
  int kro[2][2], vro[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (DMA) {
        kro[u][i] = (32 * u + pkr) * KROW + 16 * ((2 * i + hh) ^ ((pkr >> 2) & 3));
        vro[u][i] = VBASE + r * VROW + 16 * ((4 * u + 2 * i + hh) ^ ((r >> 1) & 7));
      } else {
        kro[u][i] = kb + 32 * u * KROW + 32 * i;
        vro[u][i] = vb + 64 * u + 32 * i;
      }
    }
  auto readk = [&](Q8(&kf)[2][2], const unsigned char* slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) kf[u][ks] = *(const Q8*)(slot + kro[u][ks]);
  };
  using VFrag = std::conditional_t<F8 != 0, i32x8, bf16x8[2][2]>;  // V^T fragments of one tile
  using PFrag = std::conditional_t<F8 != 0, i32x8, bf16x8[2][2]>;  // P^T fragments of one (tile, chain)
  using VStage = std::conditional_t<F8 != 0, u32x2, u32x4>;        // a thread's V^T staging share
  auto readv = [&](VFrag& vf, const unsigned char* slot) __attribute__((always_inline)) {
    if constexpr (F8 != 0) {
      const u32x4 a = *(const u32x4*)(slot + vb), c = *(const u32x4*)(slot + vb + 16);
      vf = i32x8{(int)a.x, (int)a.y, (int)a.z, (int)a.w, (int)c.x, (int)c.y, (int)c.z, (int)c.w};
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) vf[u][sp] = *(const bf16x8*)(slot + vro[u][sp]);
    }
  };
  // staging: thread tid holds K row tid >> 2 chunk tid & 3 and V^T row tid >> 3 key group tid & 7 of a tile
  const int krow = tid >> 2, kc = tid & 3, vd = tid >> 3, vc = tid & 7;
  const int kso = krow * 32 + kc * 8, vso = vd * p.Npad + vc * 8;  // 32-bit lane offsets on wave-uniform bases
  const int kw = krow * KROW + 16 * (DMA ? kc ^ ((krow >> 2) & 3) : kc);
  const int vw = F8    ? VBASE + vd * VROW + 32 * (vc & 1) + 8 * (vc >> 1)
                 : DMA ? VBASE + vd * VROW + 16 * (vc ^ ((vd >> 1) & 7))
                       : VBASE + vd * VROW + 16 * vc;
  // DMA: wave w fills K rows 16w .. 16w+15 and V^T rows 8w .. 8w+7 of a slot (one 1-KB piece each); lane i lands at
  // 16 i of its piece, so it fetches the logical unit the swizzle puts there
  uint32_t kdo = 0, vdo = 0;
  if constexpr (DMA) {
    const int R = 16 * wave + (lane >> 2), d = 8 * wave + (lane >> 3);
    kdo = (uint32_t)(R * 32 + 8 * ((lane & 3) ^ ((R >> 2) & 3))) * 2;
    vdo = (uint32_t)(d * p.Npad + 8 * ((lane & 7) ^ ((d >> 1) & 7))) * 2;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)ring;
  auto dma = [&](int t, int slot) __attribute__((always_inline)) {  // tile t -> ring slot (wave-uniform)
    p4_dma16(kdo, Kg + (int64_t)t * (P4_KT * 32), __builtin_amdgcn_readfirstlane(lds0 + slot * P4_SLOT_BYTES + wave * 1024));
    p4_dma16(vdo, Vg + t * P4_KT,
             __builtin_amdgcn_readfirstlane(lds0 + slot * P4_SLOT_BYTES + VBASE + wave * 1024));
  };
  // staging registers: P4_LEAD = 1: one set, tile t+3 loaded in step t and written to LDS in step t+1;
  // P4_LEAD = 2: two sets (tile j in set j & 1), tile t+4 loaded in step t, written in step t+2, so a load has
  // two steps to land instead of one (ablation: the K / V^T global loads cost ~40 us of a 258 us launch)
#ifndef P4_LEAD
#define P4_LEAD 2
#endif
  constexpr int LEAD = P4_LEAD;
  static_assert(LEAD == 1 || LEAD == 2, "staging lead");
  u32x4 rk[LEAD];
  VStage rv[LEAD];
  auto gload = [&](int t, u32x4& k, VStage& v) __attribute__((always_inline)) {
    k = *(const u32x4*)(Kg + (int64_t)t * (P4_KT * 32) + kso);
    if constexpr (F8 != 0) v = *(const u32x2*)(Vg8 + t * P4_KT + vso);
    else v = *(const u32x4*)(Vg + t * P4_KT + vso);
  };
  auto lstore = [&](unsigned char* slot, const u32x4& k, const VStage& v) __attribute__((always_inline)) {
    *(u32x4*)(slot + kw) = k;
    *(VStage*)(slot + vw) = v;
  };
  auto mask_pad = [&](u32x4& k, VStage& v) {  // this thread's staging share of tile nfull, keys >= nk -> 0
    const int k0 = nfull * P4_KT;
    if (k0 + krow >= p.nk) k = u32x4{0u, 0u, 0u, 0u};
    if constexpr (F8 != 0) {
      uint64_t e = __builtin_bit_cast(uint64_t, v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + vc * 8 + j >= p.nk) e &= ~((uint64_t)0xff << (8 * j));
      v = __builtin_bit_cast(u32x2, e);
    } else {
      bf16x8 e = __builtin_bit_cast(bf16x8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + vc * 8 + j >= p.nk) e[j] = (bf16)0.0f;
      v = __builtin_bit_cast(u32x4, e);
    }
  };
  // one barrier per tile: the LDS writes done (lgkmcnt(0)), global loads left in flight; DMA: also the wave's
  // pieces of the tile the next step reads (all but the two issued this step: vmcnt(2))
  auto lds_barrier = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(DMA ? 0x0072 : 0xC07F);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // direct fragment loads (the non-pipelined tile below)
  auto loadk = [&](Q8(&kf)[2][2], int t) __attribute__((always_inline)) {
    const QT* s = Kg + ((int64_t)t * P4_KT + pkr) * 32 + 8 * hh;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) kf[u][ks] = *(const Q8*)(s + u * 32 * 32 + 16 * ks);
  };
  auto loadv = [&](bf16x8(&vf)[2][2], int t) __attribute__((always_inline)) {
    const bf16* s = Vg + (int64_t)r * p.Npad + t * P4_KT + 8 * hh;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) vf[u][sp] = *(const bf16x8*)(s + 32 * u + 16 * sp);
  };

  // row-sum selector (A of v_mfma_f32_16x16x32_bf16): D row 0 sums the P fragment's k-groups 0 and 2
  // (queries 0-15 of the chain), row 1 k-groups 1 and 3 (queries 16-31)
  // (F8: A of v_mfma_scale_f32_16x16x128_f8f6f4 in e4m3, the same rows over k-groups of 32)
  bf16x8 sel;
  i32x8 sel8;
  {
    const int m = lane & 15, kg = lane >> 4;
    const bool one = (m == 0 && (kg & 1) == 0) || (m == 1 && (kg & 1) == 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) sel[j] = (bf16)(one ? 1.0f : 0.0f), sel8[j] = one ? 0x38383838 : 0;  // e4m3 1.0
  }

  f32x16 o[P4_NCH];
  f32x4 lacc[P4_NCH];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int qb = 0; qb < P4_NCH; ++qb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) o[qb][i] = 0.f;
      lacc[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  zero_acc();
  // the fast pass's row sums start at -npad: the partial tile (processed first) adds one p = 1 per padded
  // key, so they cancel in its own MFMAs and every later tile accumulates at the scale of the true sum
  const float padsum = (float)(ntiles * P4_KT - p.nk);
#pragma unroll
  for (int qb = 0; qb < P4_NCH; ++qb) lacc[qb] = f32x4{-padsum, -padsum, -padsum, -padsum};

  const f32x16 zero16 = {};
  auto smm = [&](f32x16(&s)[2], const Q8(&kf)[2][2], int qb) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      s[u] = mfma32(kf[u][0], qf[qb][0], zero16);
      s[u] = mfma32(kf[u][1], qf[qb][1], s[u]);
    }
  };
  // bf16 P.V of one (tile, chain): the re-run tile of every variant
  auto expc16 = [&](bf16x8(&pb)[2][2], const f32x16(&s)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[u][sp][j] = (bf16)__builtin_amdgcn_exp2f(s[u][8 * sp + j]);
  };
  auto pv16 = [&](int qb, const bf16x8(&pb)[2][2], const bf16x8(&vf)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        o[qb] = mfma32(vf[u][sp], pb[u][sp], o[qb]);
        lacc[qb] = mfma16(sel, pb[u][sp], lacc[qb]);
      }
  };
  // F8: per-chain conversion scale of the lane's query (P' = exp2(s) / scale), set from the first tile
  // and P'(0), the value every padded key adds to the row sum
  float scl[P4_NCH] = {1.0f, 1.0f}, padv[P4_NCH] = {1.0f, 1.0f};
  // bf16: P^T fragment (u, sp) = keys 32u + 16sp + 8hh + 0..7 (bf16x8 each).  F8: one i32x8 per chain,
  // byte 16u + i of the lane = s[u][i], i.e. logical k 32hh + 16u + i = key 32u + 16 (i >> 3) + 8hh + (i & 7)
  auto expc = [&](PFrag& pb, const f32x16(&s)[2], int qb) __attribute__((always_inline)) {
    if constexpr (F8 != 0) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          // (the low half is converted into the register of its own first input, which dies there: both
          // halves get written, and any other `old` operand costs a v_mov per word)
          const float e0 = __builtin_amdgcn_exp2f(s[u][4 * w]);
          s16x2 x = P8<F8>::cvt(__builtin_bit_cast(s16x2, e0), e0, __builtin_amdgcn_exp2f(s[u][4 * w + 1]), scl[qb],
                                false);
          x = P8<F8>::cvt(x, __builtin_amdgcn_exp2f(s[u][4 * w + 2]), __builtin_amdgcn_exp2f(s[u][4 * w + 3]), scl[qb],
                          true);
          pb[4 * u + w] = __builtin_bit_cast(int, x);
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[u][sp][j] = (bf16)__builtin_amdgcn_exp2f(s[u][8 * sp + j]);
    }
  };
  auto pv = [&](int qb, const PFrag& pb, const VFrag& vf) __attribute__((always_inline)) {
    if constexpr (F8 != 0) {
      o[qb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pb, o[qb], 0, P8<F8>::FMT, 0, 127, 0, 127);
      lacc[qb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(sel8, pb, lacc[qb], 0, P8<F8>::FMT, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          o[qb] = mfma32(vf[u][sp], pb[u][sp], o[qb]);
          lacc[qb] = mfma16(sel, pb[u][sp], lacc[qb]);
        }
    }
  };
  // the order of one pipeline step: 12 MFMAs (S0-S3 32x32, then P.V 32x32 / row-sum 16x16 pairs), 32
  // exps, 16 conversions and the step's LDS / global traffic.  An MFMA holds vector issue for 8 cycles;
  // a filler is free while the gap's issue sum fits the MFMA (32 / 16 cycles) and costs extra once it
  // overflows (MI355X_MICROARCH.md constants), so each gap carries exactly its budget (P4_PIN 1: three
  // exps per 32x32, one per 16x16) and the conversions + remaining exps follow in an MFMA-free tail
#ifndef P4_PIN
#define P4_PIN 1
#endif
  auto pin_step = [&](bool mem) __attribute__((always_inline)) {
#if P4_PIN == 0
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      if (mem) __builtin_amdgcn_sched_group_barrier(SG_DS_READ, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_VALU, 1, 0);
      if (mem && i == 1) __builtin_amdgcn_sched_group_barrier(SG_DS_WRITE, 2, 0);
      if (mem && i == 2) __builtin_amdgcn_sched_group_barrier(SG_VMEM_READ, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_VALU, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_VALU, 2, 0);
    }
#else
    if constexpr (F8 != 0) {
      // S MFMAs (32 cycles): 3 exps each; P.V 32x32x64 (64 cycles): 7; row sum 16x16x128 (32 cycles): 3
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
        if (mem && i < 2) __builtin_amdgcn_sched_group_barrier(SG_DS_READ, 3, 0);
        __builtin_amdgcn_sched_group_barrier(SG_TRANS, 3, 0);
      }
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 7, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 10, 0);
      __builtin_amdgcn_sched_group_barrier(SG_VALU, 16, 0);
      if (mem) {
        __builtin_amdgcn_sched_group_barrier(SG_DS_WRITE, 2, 0);
        __builtin_amdgcn_sched_group_barrier(SG_VMEM_READ, 2, 0);
      }
      return;
    }
    // S MFMAs: 3 exps each (the LDS reads of the next fragments ride in the first two gaps)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      if (mem && i < 2) __builtin_amdgcn_sched_group_barrier(SG_DS_READ, 4, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 3, 0);
    }
    // P.V (32x32) + row-sum (16x16) pairs: 3 + 1 exps
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, 3, 0);
      __builtin_amdgcn_sched_group_barrier(SG_MFMA, 1, 0);
      __builtin_amdgcn_sched_group_barrier(SG_TRANS, P4_PIN == 2 ? 0 : 1, 0);
    }
    // tail: the remaining exps and the 16 conversions, then the staging traffic
    __builtin_amdgcn_sched_group_barrier(SG_TRANS, P4_PIN == 2 ? 8 : 4, 0);
    __builtin_amdgcn_sched_group_barrier(SG_VALU, 16, 0);
    if (mem && !DMA) {
      __builtin_amdgcn_sched_group_barrier(SG_DS_WRITE, 2, 0);
      __builtin_amdgcn_sched_group_barrier(SG_VMEM_READ, 2, 0);
    }
#endif
  };

  // ---- fast pass: fixed reference 0 over the full tiles, pipelined by (tile, chain) units
  //   step (t, 0): S(t, chain 1) | exp S(t, chain 0) | P.V(t-1, chain 1); reads kf(t+1), vf(t) from LDS,
  //                writes tile t+2 (staged) to LDS, loads tile t+3 into the staging registers
  //   step (t, 1): S(t+1, chain 0) | exp S(t, chain 1) | P.V(t, chain 0); then the tile's barrier
  // kf(t) in register set t % 2, vf(t) in set (t + 1) % 2
  if (ntiles > 0) {
    Q8 kf[2][2][2];
    VFrag vf[2];
    f32x16 sa[2], sb[2];
    PFrag pa, pz;
    {  // tiles 0 and 1 in flight together, then tile 2 into the staging registers
      u32x4 rk1;
      VStage rv1;
      gload(tile_of(0), rk[0], rv[0]);
      gload(tile_of(min(1, ntiles - 1)), rk1, rv1);
      if constexpr (DMA) dma(tile_of(min(2, ntiles - 1)), 2);  // (the partial tile, if any, is tile 0: masked here)
      if (partial) mask_pad(rk[0], rv[0]);
      lstore(ring, rk[0], rv[0]);
      lstore(ring + P4_SLOT_BYTES, rk1, rv1);
    }
    if constexpr (!DMA) {
      gload(tile_of(min(2, ntiles - 1)), rk[0], rv[0]);
      if constexpr (LEAD == 2) gload(tile_of(min(3, ntiles - 1)), rk[1], rv[1]);
    }
    lds_barrier();
    AP_STAMP(2);
    if (!active) {
      // a wave without queries (a kv sequence's last, partial task) stages its share of every tile and
      // meets every barrier, but issues none of the loop's MFMAs / exps: they would take issue slots
      // from the other block's wave on its SIMD
      if constexpr (DMA) {
        for (int t = 0; t < ntiles; ++t) {
          dma(tile_of(min(t + 3, ntiles - 1)), (t + 3) & 3);
          lds_barrier();
        }
        __builtin_amdgcn_s_waitcnt(0x0070);  // the last pieces landed before the wave ends
        return;
      }
      for (int t = 0; t < ntiles; t += LEAD) {
        lstore(ring + ((t + 2) & 3) * P4_SLOT_BYTES, rk[0], rv[0]);
        gload(tile_of(min(t + 2 + LEAD, ntiles - 1)), rk[0], rv[0]);
        lds_barrier();
        if (LEAD == 2 && t + 1 < ntiles) {
          lstore(ring + ((t + 3) & 3) * P4_SLOT_BYTES, rk[LEAD - 1], rv[LEAD - 1]);
          gload(tile_of(min(t + 5, ntiles - 1)), rk[LEAD - 1], rv[LEAD - 1]);
          lds_barrier();
        }
      }
      return;  // no barrier follows the fast pass
    }
    readk(kf[0], ring);
    if constexpr (F8 != 0) {
      vf[0] = i32x8{0, 0, 0, 0, 0, 0, 0, 0}, pz = vf[0];
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int j = 0; j < 8; ++j) vf[0][u][sp][j] = pz[u][sp][j] = (bf16)0.0f;
    }
    smm(sa, kf[0], 0);
    if constexpr (F8 != 0) {
      // the lane's query reference: max over the real keys of the first tile in processing order (both
      // chains; chain 1's scores are recomputed by the loop), P' = exp2(s) / 2^e, e = floor(max) - ETOP.  The
      // row sums start at -npad P'(0): the padded keys (s = 0) add exactly that, as fp8 (0 once 2^-e
      // underflows); with padded keys e >= -EMAX keeps P'(0) inside the format (a row whose first-tile max is
      // that far below 0 keeps fewer octaves under its max; a total underflow fails the row-sum check)
      f32x16 s1[2];
      smm(s1, kf[0], 1);
      const int k0 = tile_of(0) * P4_KT;
#pragma unroll
      for (int qb = 0; qb < P4_NCH; ++qb) {
        const f32x16(&s)[2] = qb == 0 ? sa : s1;
        float m = -INFINITY;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (k0 + 32 * u + 16 * (i >> 3) + 8 * hh + (i & 7) < p.nk) m = fmaxf(m, s[u][i]);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
        m = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        const float elo = partial ? -(float)P8<F8>::EMAX : -100.f;
        const int e = (int)fminf(fmaxf(floorf(m) - (float)P8<F8>::ETOP, elo), 100.f);
        scl[qb] = __int_as_float((e + 127) << 23);
        padv[qb] = -e >= P8<F8>::EMIN ? __int_as_float((127 - e) << 23) : 0.f;
      }
      const float ps = -(float)(ntiles * P4_KT - p.nk);
#pragma unroll
      for (int qb = 0; qb < P4_NCH; ++qb) {
        const float own = ps * padv[qb], hi = __shfl(own, (lane & 15) + 16, 64);
        lacc[qb] = f32x4{own, hi, own, hi};
      }
    }
    // tile t in ring slot t % 4 (compile-time slots: every LDS address is a base + an immediate)
    auto iter = [&](auto phc, int t) __attribute__((always_inline)) {
      constexpr int L = decltype(phc)::value, A = L & 1, B = A ^ 1;
      constexpr int S0 = L * P4_SLOT_BYTES, S1 = ((L + 1) & 3) * P4_SLOT_BYTES, S2 = ((L + 2) & 3) * P4_SLOT_BYTES;
      readk(kf[B], ring + S1);
      readv(vf[B], ring + S0);
      constexpr int RS = LEAD == 2 ? A : 0;  // staging set of tile t+2 (and of t+2+LEAD, loaded next)
      if constexpr (!DMA) {
        lstore(ring + S2, rk[RS], rv[RS]);
        gload(tile_of(min(t + 2 + LEAD, ntiles - 1)), rk[RS], rv[RS]);
      }
      smm(sb, kf[A], 1);
      expc(pa, sa, 0);
      pv(1, pz, vf[A]);
      pin_step(true);
      // DMA: tile t+3 into the slot tile t-1 left (its last reads done before the previous barrier); it has
      // this step and the next to land
      if constexpr (DMA) dma(tile_of(min(t + 3, ntiles - 1)), (L + 3) & 3);
      smm(sa, kf[B], 0);
      expc(pz, sb, 1);
      pv(0, pa, vf[B]);
      pin_step(false);
      lds_barrier();
#if defined(MMPFN_STAMPS) || defined(MMPFN_STAMPS_ALL)
      if (t < AP_NST - 6) AP_STAMP(3 + t);
#endif
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    int t = 0;
    for (; t + 4 <= ntiles; t += 4) {
      iter(I0{}, t);
      iter(I1{}, t + 1);
      iter(I2{}, t + 2);
      iter(I3{}, t + 3);
    }
    if (t < ntiles) iter(I0{}, t++);
    if (t < ntiles) iter(I1{}, t++);
    if (t < ntiles) iter(I2{}, t++);
    // drain: P.V of the last tile's chain 1 (vf(ntiles - 1) sits in set ntiles % 2)
    if (ntiles & 1) pv(1, pz, vf[1]);
    else pv(1, pz, vf[0]);
  }
  AP_STAMP(AP_NST - 3);

  if (!active) return;
  // ---- one tile, not pipelined, straight from global memory: every tile of the rare re-run with a
  //      reference (REF: s - mref; FIRST: mref = this tile's row max)
  float mref[P4_NCH] = {0.f, 0.f};
  auto tile1 = [&](int t, bool first, bool ref) {
    const int k0 = t * P4_KT;
    Q8 kf[2][2];
    bf16x8 vf[2][2];
    loadk(kf, t);
    loadv(vf, t);
    const bool mask = k0 + P4_KT > p.nk;
    if (mask) {  // keys >= nk: V = 0 so that p = 0 never meets NaN / inf padding
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (k0 + 32 * u + 16 * sp + 8 * hh + j >= p.nk) vf[u][sp][j] = (bf16)0.0f;
    }
#pragma unroll
    for (int qb = 0; qb < P4_NCH; ++qb) {
      f32x16 s[2];
      smm(s, kf, qb);
      if (mask) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (k0 + 32 * u + (i & 3) + 4 * ((i >> 2) & 1) + 8 * hh + 16 * (i >> 3) >= p.nk) s[u][i] = -INFINITY;
      }
      if (first) {
        float m = fmaxf(s[0][0], s[1][0]);
#pragma unroll
        for (int i = 1; i < 16; ++i) m = fmaxf(m, fmaxf(s[0][i], s[1][i]));
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
        mref[qb] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      if (ref) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[0][i] -= mref[qb], s[1][i] -= mref[qb];
      }
      bf16x8 pb[2][2];
      expc16(pb, s);
      pv16(qb, pb, vf);
    }
  };

  // the row sum of chain qb on the query's lanes (D rows 0 / 1 of lacc sit in lanes 0-15, registers 0 / 1)
  auto rowsum = [&](int qb) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(lacc[qb][0]), __float_as_uint(lacc[qb][1]),
                                                    false, false);
    const auto s2 = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);
    return __uint_as_float(s2[0]);
  };
  {  // reference-free pass out of [2^-60, 2^100) (tested on the bits; built with -fno-honor-nans) for
     // any query of the wave: re-run the wave with the first tile's row max
    // (also when a row sum is below 2^-12 npad: the cancelled ones left a few roundings at ulp(npad) in it)
    bool bad = false;
#pragma unroll
    for (int qb = 0; qb < P4_NCH; ++qb) {
      const float rs = rowsum(qb);
      const unsigned lb = __float_as_uint(rs) & 0x7fffffffu;
      // (F8: the padded keys' ones are P'(0) each; a score past the format's range is NaN / inf here)
      bad |= lb >= 0x71800000u || lb < 0x21800000u || rs < padsum * padv[qb] * 0x1p-12f;
      if constexpr (F8 != 0) bad |= rs < (float)p.nk * P8<F8>::UFLOW;  // the format's floor (UFLOW above)
    }
    if (__any(bad)) {
      zero_acc();
      for (int t = 0; t < ntiles; ++t) tile1(t, t == 0, true);
    }
  }
  AP_STAMP(AP_NST - 2);

  // ---- row sums to the query's lanes, overflow backstop, normalise, store
#pragma unroll
  for (int qb = 0; qb < P4_NCH; ++qb) {
    const float ls = rowsum(qb);
    const QRow q = qrow_of(qb);
    OT* orow = (OT*)p.o + ((int64_t)b * p.S + q.s) * (p.H * 32) + q.h * 32;
    if (__any((__float_as_uint(ls) & 0x7fffffffu) >= 0x71800000u)) {
      const QT* qrow = (const QT*)p.q + (((int64_t)b * p.H + q.h) * p.S + q.s) * 32;
      p4_exact_rows(p, Kg, Vg, qrow, orow, q.ok && hh == 0, p.q_prescaled ? 1.0f : c);
      continue;
    }
    const float inv = 1.0f / ls;
    // lane (r, hh) holds d = 8 gq + 4 hh + 0..3: lanes 0-31 store d 8g .. 8g+7, lanes 32-63 d 8g+8 .. +15
    u32x2 w[4];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      O4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (OT)(o[qb][4 * gq + e] * inv);
      w[gq] = __builtin_bit_cast(u32x2, v);
    }
#pragma unroll
    for (int gg = 0; gg < 4; gg += 2) {
      const auto sx = __builtin_amdgcn_permlane32_swap(w[gg].x, w[gg + 1].x, false, false);
      const auto sy = __builtin_amdgcn_permlane32_swap(w[gg].y, w[gg + 1].y, false, false);
      const u32x4 st = hh == 0 ? u32x4{w[gg].x, w[gg].y, sx[1], sy[1]} : u32x4{sx[0], sy[0], w[gg + 1].x, w[gg + 1].y};
      if (q.ok) *(u32x4*)(orow + 8 * gg + 8 * hh) = st;
    }
  }
  AP_STAMP(AP_NST - 1);
}

}  // namespace

namespace {
template <bool QF16, bool OF16>
hipError_t launch_pipe(const Attn2Args& a, hipStream_t st) {
  if (a.f8 == 1) {
    if (!a.vt8) return hipErrorInvalidValue;
    hipLaunchKernelGGL((attn_pipe_kernel<1, QF16, OF16>), dim3(a.nblocks), dim3(256), 0, st, a);
  } else if (a.f8 == 2) {
    if (!a.vt8) return hipErrorInvalidValue;
    hipLaunchKernelGGL((attn_pipe_kernel<2, QF16, OF16>), dim3(a.nblocks), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_pipe_kernel<0, QF16, OF16>), dim3(a.nblocks), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}
}  // namespace

#ifdef MMPFN_STAMPS
extern "C" int mmpfn_dbg_attn_stamps(unsigned long long* stamps, int* meta) {
  hipError_t e = hipMemcpyFromSymbol(stamps, HIP_SYMBOL(g_ap_stamps), sizeof(g_ap_stamps));
  if (e == hipSuccess) e = hipMemcpyFromSymbol(meta, HIP_SYMBOL(g_ap_meta), sizeof(g_ap_meta));
  return (int)e;
}
#endif

#ifdef MMPFN_STAMPS_ALL
extern "C" int mmpfn_dbg_attn_stamps_all(unsigned long long* out, int nblocks) {
  const size_t n = (size_t)(nblocks < AP_MAXB ? nblocks : AP_MAXB) * 4 * (AP_NST + 2) * sizeof(unsigned long long);
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ap_all), n);
}
#endif

hipError_t launch_attn_pipe(const Attn2Args& a, hipStream_t st) {
  if (a.qk_f16) return launch_pipe<true, true>(a, st);
  return a.o_f16 ? launch_pipe<false, true>(a, st) : launch_pipe<false, false>(a, st);
}

namespace {
// bf16 -> e4m3 (saturating at +-448: a value past the range must not turn V into NaN), 8 elements per
// thread, for the F8 attention's V^T operand
__global__ void vt_fp8_kernel(const u32x4* __restrict__ in, u32x2* __restrict__ out, int64_t n8) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const bf16x8 v = __builtin_bit_cast(bf16x8, in[i]);
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf((float)v[j], -448.f), 448.f);
  s16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s16x2{0, 0}, f[0], f[1], 1.0f, false);
  lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(lo, f[2], f[3], 1.0f, true);
  s16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s16x2{0, 0}, f[4], f[5], 1.0f, false);
  hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(hi, f[6], f[7], 1.0f, true);
  out[i] = u32x2{__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
}
}  // namespace

hipError_t launch_vt_fp8(const void* vt, void* vt8, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n % 8) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(vt_fp8_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, (const u32x4*)vt, (u32x2*)vt8,
                     n8);
  return hipGetLastError();
}

}  // namespace mmpfn
