// Row-resident MLP sublayer on 32x32x16 MFMAs (bf16 performance mode):
//   X <- LayerNorm(X + GELU(X W1^T) W2^T)           (mlp.py:93-104, layer.py:437-455)
// optionally after the fused item-attention out-projection (RES): X <- LayerNorm(X + O Wout^T)
//
// The design of mlp_rows.hip (32 rows per wave resident in registers, weights streamed through
// three-slot LDS-DMA rings, GELU of chunk c beside the up-projection of chunk c+1, the residual
// inside the output accumulators) with every contraction on v_mfma_f32_32x32x16_bf16: the same
// flops in half as many MFMA instructions, so half the issue slots the MFMAs hold from the VALU
// (MI355X_MICROARCH.md: 8 per MFMA of either shape).  The kernel is bound by its vector issue:
// 16 GELUs (two transcendentals each) per lane and 32-hidden chunk beside 48 16x16x32 MFMAs.
//
// Lane layouts (lane l: token r = l % 32 of the wave's 32 rows, half hh = l / 32):
//   Y^T accumulators y[o] (o = 0..5, 32 features each): register i = feature 32o + (i&3) + 8(i>>2) + 4hh
//   X'^T B fragments af[ks] (k-step ks of 16 features): registers 8(ks&1) .. +7 of y[ks>>1], i.e.
//       K position 16ks + 8hh + m <-> feature 32(ks>>1) + 16(ks&1) + (m&3) + 8(m>>2) + 4hh
//       (W1's columns are permuted to that order on the host: capi.cpp pack_mlp1_perm32)
//   H^T accumulator of a 32-hidden chunk: register i = hidden (i&3) + 8(i>>2) + 4hh; its GELU,
//       registers 8j .. 8j+7, is the B fragment of down-projection k-step j, whose K position
//       16j + 8hh + m <-> hidden 16j + (m&3) + 8(m>>2) + 4hh (W2's chunk columns permuted alike:
//       capi.cpp pack_mlp2_perm32)
// LDS images (unpadded, 16-B units XOR-swizzled, conflict-free ds_read_b128 for the 32x32 operand):
//   W1 slot [32 hidden][384 B] and the Wout halves [96 out][384 B]: unit u of row r at u ^ ((r >> 1) & 7)
//   W2 slot [192 out][64 B]: unit u of row r at u ^ ((r >> 2) & 3)
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int QE = 192;                    // model width
constexpr int QHC = 32;                    // hidden chunk
constexpr int QSLOT = QHC * QE * 2;        // one W1 or W2 chunk image: 12 KB
constexpr int QNSLOT = 3;                  // ring depth per matrix
constexpr int QW2RING = QNSLOT * QSLOT;    // byte offset of the W2 ring
constexpr int QLDS = 2 * QNSLOT * QSLOT;   // 72 KB per block: two blocks per CU
constexpr int QMP = QSLOT / 1024 / 4;      // 1-KB DMA pieces per wave, matrix and chunk (3)
typedef __attribute__((ext_vector_type(2))) float float2_t;

__device__ __forceinline__ void q_dma16(uint32_t voff, const void* sbase, unsigned lds_dst) {
  // m0 = the wave's LDS destination; lane i's 16 B (sbase + voff) land at m0 + 16 i
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory");
}

template <typename F, int... I>
__device__ __forceinline__ void q_static_for_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void q_static_for(F&& f) {
  q_static_for_(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <bool RES>
__global__ __launch_bounds__(256, 2) void mlp32_kernel(float* __restrict__ X, const bf16* __restrict__ W1,
                                                       const bf16* __restrict__ W2p, int M, int Fh, float eps,
                                                       const bf16* __restrict__ O, const bf16* __restrict__ Wout) {
  constexpr int RROWS = 128;  // 4 waves x 32 rows
  __shared__ __attribute__((aligned(1024))) bf16 lds[QLDS / 2];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * RROWS + wave * 32;
  const int nchunks = Fh / QHC;
  const int64_t mrow = min(m0 + r, (int64_t)M - 1);  // the lane's token (clamped: tail rows recompute, no store)

  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  uint32_t o1[QMP], o2[QMP];
#pragma unroll
  for (int j = 0; j < QMP; ++j) {
    const int q = (wave * QMP + j) * 64 + lane;  // unit index inside a slot image
    const int r1 = q / 24, u1 = (q % 24) ^ ((r1 >> 1) & 7);
    o1[j] = (uint32_t)(r1 * QE + u1 * 8) * 2;
    const int r2 = q >> 2, u2 = (q & 3) ^ ((r2 >> 2) & 3);
    o2[j] = (uint32_t)(r2 * Fh + u2 * 8) * 2;
  }
  auto dma_w1 = [&](int c, int slot) {  // W1 rows c*32 .. +31 (columns in the af K order)
    const bf16* base = W1 + (int64_t)c * QHC * QE;
#pragma unroll
    for (int j = 0; j < QMP; ++j)
      q_dma16(o1[j], base, __builtin_amdgcn_readfirstlane(lds0 + slot * QSLOT + (wave * QMP + j) * 1024));
  };
  auto dma_w2 = [&](int c, int slot) {  // W2 columns c*32 .. +31 (permuted), all 192 rows
    const bf16* base = W2p + c * QHC;
#pragma unroll
    for (int j = 0; j < QMP; ++j)
      q_dma16(o2[j], base, __builtin_amdgcn_readfirstlane(lds0 + QW2RING + slot * QSLOT + (wave * QMP + j) * 1024));
  };
  // fragment reads (bytes inside a slot): W1 row r, unit 2ks + hh; W2 row 32o + r, unit 2j + hh
  // unit u = 8a + b sits at 8a + (b ^ swizzle): a lane offset per (ks & 3) / j, the rest immediate
  const int s1 = (r >> 1) & 7, s2 = (r >> 2) & 3;
  uint32_t f1[4], f2[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) f1[k] = r * 384 + (((2 * k + hh) ^ s1) << 4);
#pragma unroll
  for (int j = 0; j < 2; ++j) f2[j] = QW2RING + r * 64 + (((2 * j + hh) ^ s2) << 4);
  const unsigned char* ldsb = (const unsigned char*)lds;
  auto w1frag = [&](int slot, int ks) {
    return *(const bf16x8*)(ldsb + slot * QSLOT + 128 * (ks >> 2) + f1[ks & 3]);
  };
  auto w2frag = [&](int slot, int o, int j) {
    return *(const bf16x8*)(ldsb + slot * QSLOT + 32 * o * 64 + f2[j]);
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;

  f32x16 y[QE / 32];
  bf16x8 af[QE / 16];
  auto to_af = [&]() {
#pragma unroll
    for (int ks = 0; ks < QE / 16; ++ks) {
      bf16x8 b;
#pragma unroll
      for (int m = 0; m < 8; ++m) b[m] = (bf16)y[ks >> 1][8 * (ks & 1) + m];
      af[ks] = b;
    }
  };
  auto load_x = [&]() {  // y <- the fp32 residual rows, Y^T layout
    const float* xr = X + mrow * QE + 4 * hh;
#pragma unroll
    for (int o = 0; o < QE / 32; ++o)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = *(const f32x4*)(xr + 32 * o + 8 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) y[o][4 * g + i] = v[i];
      }
  };
  auto layernorm = [&]() {  // in place on y: the token's 192 features = this lane's 96 + lane^32's 96
    float sm = 0.f;
#pragma unroll
    for (int o = 0; o < QE / 32; ++o)
#pragma unroll
      for (int i = 0; i < 16; ++i) sm += y[o][i];
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(sm), __float_as_uint(sm), false, false);
      sm = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    const float mean = sm * (1.0f / QE);
    float q = 0.f;
#pragma unroll
    for (int o = 0; o < QE / 32; ++o)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float dl = y[o][i] - mean;
        q += dl * dl;
      }
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(q), __float_as_uint(q), false, false);
      q = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    const float inv = 1.0f / sqrtf(q * (1.0f / QE) + eps);
#pragma unroll
    for (int o = 0; o < QE / 32; ++o)
#pragma unroll
      for (int i = 0; i < 16; ++i) y[o][i] = (y[o][i] - mean) * inv;
  };
  auto wait_vm = [](auto nc) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(nc)::value) : "memory"); };
  using std::integral_constant;
  const bool deep = nchunks >= 3;

  if constexpr (RES) {
    // X <- LayerNorm(X + O . Wout^T): Wout [192 out][192 in] by LDS-DMA in two 96-row halves (half 0 over the
    // W1 ring, half 1 over the W2 ring), the accumulators starting from the residual X
    {
      uint32_t ow[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int q = (wave * 9 + j) * 64 + lane, rr = q / 24, u = (q % 24) ^ ((rr >> 1) & 7);
        ow[j] = (uint32_t)(rr * QE + u * 8) * 2;
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (hf == 1) load_x();
#pragma unroll
        for (int j = 0; j < 9; ++j)
          q_dma16(ow[j], Wout + hf * 96 * QE,
                  __builtin_amdgcn_readfirstlane(lds0 + hf * QNSLOT * QSLOT + (wave * 9 + j) * 1024));
        if (hf == 0) {
          const bf16* orow = O + mrow * QE + 8 * hh;
#pragma unroll
          for (int ks = 0; ks < QE / 16; ++ks) af[ks] = *(const bf16x8*)(orow + 16 * ks);  // O^T fragments
        }
      }
    }
    auto outproj = [&](auto hc) {  // y[3 hf .. 3 hf + 2] += Wout half hf . O^T
      constexpr int HF = decltype(hc)::value;
#pragma unroll
      for (int ks = 0; ks < QE / 16; ++ks)
#pragma unroll
        for (int ol = 0; ol < 3; ++ol) {
          const bf16x8 w = *(const bf16x8*)(ldsb + HF * QNSLOT * QSLOT + 32 * ol * 384 + 128 * (ks >> 2) + f1[ks & 3]);
          y[3 * HF + ol] = mfma32(w, af[ks], y[3 * HF + ol]);
        }
    };
    wait_vm(integral_constant<int, 9>{});  // half 0 (and O, X) landed; half 1 may fly
    __syncthreads();
    outproj(integral_constant<int, 0>{});
    __syncthreads();  // the W1 ring is free
    dma_w1(0, 0);
    if (nchunks > 1) dma_w1(1, 1);
    if (deep) dma_w1(2, 2);
    if (deep) wait_vm(integral_constant<int, 3 * QMP>{});
    else wait_vm(integral_constant<int, 0>{});
    __syncthreads();
    outproj(integral_constant<int, 1>{});
    __syncthreads();  // the W2 ring is free
    dma_w2(0, 0);
    if (nchunks > 1) dma_w2(1, 1);
    layernorm();
    to_af();
    if (deep) wait_vm(integral_constant<int, 4 * QMP>{});  // W1(0) landed
    else wait_vm(integral_constant<int, 0>{});
  } else {
    dma_w1(0, 0);
    if (nchunks > 1) dma_w1(1, 1);
    load_x();
    to_af();
    dma_w2(0, 0);
    if (deep) dma_w1(2, 2);
    if (nchunks > 1) dma_w2(1, 1);
    if (deep) wait_vm(integral_constant<int, 4 * QMP>{});  // W1(0) landed (X, older, too)
    else wait_vm(integral_constant<int, 0>{});
  }
  __syncthreads();

  // up-projection H^T = W1c . X'^T of the chunk in W1 slot SL; with G, the previous chunk's GELU (hs -> hb)
  // rides in its k-steps (one element pair per k-step for 8 of the 12)
  auto gelu_pair = [&](auto qc, const f32x16& hs, bf16x8 (&hb)[2]) {
    constexpr int q = decltype(qc)::value, i = 2 * q;  // registers i, i+1 -> hb[i >> 3][i & 7 ..]
    const bf16x2 pr = __builtin_convertvector((float2_t){gelu_tanh_fast(hs[i]), gelu_tanh_fast(hs[i + 1])}, bf16x2);
    hb[i >> 3][i & 7] = pr[0];
    hb[i >> 3][(i & 7) + 1] = pr[1];
  };
  auto hmma = [&](auto slc, f32x16& h, auto gc, const f32x16& hs, bf16x8 (&hb)[2]) {
    constexpr bool G = decltype(gc)::value;
    constexpr int SL = decltype(slc)::value;
    h = f32x16{};
    constexpr int PU = 2;  // k-steps of W1 fragments in flight ahead of their MFMAs
    bf16x8 wa[PU];
#pragma unroll
    for (int i = 0; i < PU; ++i) wa[i] = w1frag(SL, i);
#pragma unroll
    for (int ks = 0; ks < QE / 16; ++ks) {
      __builtin_amdgcn_sched_barrier(0);
      h = mfma32(wa[ks % PU], af[ks], h);
      if (ks + PU < QE / 16) wa[ks % PU] = w1frag(SL, ks + PU);
      if constexpr (G) {  // 8 pairs over the 12 k-steps
        q_static_for<8>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if (q * 12 / 8 == ks) gelu_pair(qc, hs, hb);
        });
      }
    }
  };
  f32x16 h;
  {
    bf16x8 unused[2];
    hmma(S0{}, h, std::false_type{}, h, unused);
  }
  if (deep) wait_vm(integral_constant<int, QMP>{});  // W1(1) and W2(0) landed
  else wait_vm(integral_constant<int, 0>{});
  __syncthreads();

  auto chunk = [&](int c, auto parc) {
    const bool MORE = c + 1 < nchunks;
    constexpr int PAR = decltype(parc)::value;
    const bool d1 = c + 3 < nchunks, d2 = c + 2 < nchunks;
    if (d1) dma_w1(c + 3, PAR);
    if (d2) dma_w2(c + 2, (PAR + 2) % 3);
    bf16x8 hb[2];
    {
      f32x16 hn;
      hmma(std::integral_constant<int, (PAR + 1) % 3>{}, hn, std::true_type{}, h, hb);
      h = hn;
    }
    // Y^T [192][32 rows] += W2c(perm) . GELU(H^T): 6 output tiles x 2 k-steps, fragments 3 ahead
    {
      constexpr int PF = 3;
      bf16x8 wb[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) wb[i] = w2frag(PAR, i >> 1, i & 1);
#pragma unroll
      for (int t = 0; t < 12; ++t) {
        __builtin_amdgcn_sched_barrier(0);
        y[t >> 1] = mfma32(wb[t % PF], hb[t & 1], y[t >> 1]);
        if (t + PF < 12) wb[t % PF] = w2frag(PAR, (t + PF) >> 1, (t + PF) & 1);
      }
    }
    if (MORE) {
      if (d1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * QMP) : "memory");
      else if (d2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QMP) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };
  for (int c = 0; c < nchunks; c += 3) {
    chunk(c, S0{});
    if (c + 1 < nchunks) chunk(c + 1, S1{});
    if (c + 2 < nchunks) chunk(c + 2, S2{});
  }

  layernorm();
  if (m0 + r < M) {
    float* xr = X + (m0 + r) * QE + 4 * hh;
#pragma unroll
    for (int o = 0; o < QE / 32; ++o)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(f32x4*)(xr + 32 * o + 8 * g) = f32x4{y[o][4 * g], y[o][4 * g + 1], y[o][4 * g + 2], y[o][4 * g + 3]};
  }
}

}  // namespace

hipError_t launch_mlp32(float* X, const void* W1perm, const void* W2perm, int64_t M, int E, int Fh, float eps,
                        hipStream_t st, const void* O, const void* Wout) {
  if (M <= 0) return hipSuccess;
  if (E != QE || Fh % QHC != 0) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((M + 127) / 128)), block(256);
  if (O)
    hipLaunchKernelGGL(mlp32_kernel<true>, grid, block, 0, st, X, (const bf16*)W1perm, (const bf16*)W2perm, (int)M,
                       Fh, eps, (const bf16*)O, (const bf16*)Wout);
  else
    hipLaunchKernelGGL(mlp32_kernel<false>, grid, block, 0, st, X, (const bf16*)W1perm, (const bf16*)W2perm, (int)M,
                       Fh, eps, nullptr, nullptr);
  return hipGetLastError();
}

}  // namespace mmpfn
