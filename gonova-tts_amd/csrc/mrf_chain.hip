// Fused HiFi-GAN resblock: the three ResBlock pairs of one resblock (dilations 1, 3, 5) in
// one launch, for the resblocks whose pair kernels are HBM-bound (k = 3 at C = 32 / 64,
// k = 7 at C = 32):
//
//   h0 = x;  for p in 0..2:  t = lrelu(conv_{k,d_p}(lrelu(h_p)) + b1_p)
//                            h_{p+1} = conv_{k,1}(t) + b2_p + h_p
//   y = ((accum ? y : 0) + h_3) * scale                       (oracle: vocoder.resblock)
//
// Three pair launches move [rows][C] through HBM six times (read h, write h' per pair, the
// first pair's halo from L2); here a block reads its x tile once (with the resblock's whole
// receptive-field halo H0 = a2 * sum(d_p + 1) rows per side) and writes its BN output rows
// once.  At C = 32 a row is 64 bytes and a k = 3 pair only 12 kFLOP per row, so the pair
// kernels ran near the HBM rate; the chain trades that traffic for the halo recompute
// (every conv computes only the rows its successor needs, in 16-row tiles).
//
// LDS: two [NRA][C] tiles in the pair kernel's swizzled layout (mrf_tile.h):
//   Hs: h_p, the residual (raw, in place: each h_{p+1} row is written by the thread that
//       read h_p there);
//   GT: G = lrelu(h_p) (conv1's operand), overwritten by T after conv1, overwritten by the
//       next G after conv2 (barriers between), and by the last conv2's output for the
//       row pass.
// Rows are in block coordinates: LDS row r <-> utterance row n0 - H0 + r; rows outside the
// utterance are zero in G and T after every conv (the unfused convs' zero padding).
// Arithmetic and rounding order match the pair path (mrf_pair.hip) exactly, so the chain's
// output is bit-identical to three pair launches.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "mrf_tile.h"

namespace tts {

template <int C, int K>
struct ChainGeom;
// Rows per block and blocks per CU (LDS 2 * NRA * C * 2 bytes per block, registers sized for
// OCC blocks) per (C, k); tuned by same-box A/B (tools/ab.sh).
#ifndef TTS_CHAIN_BN32_3
#define TTS_CHAIN_BN32_3 256
#endif
#ifndef TTS_CHAIN_BN32_7
#define TTS_CHAIN_BN32_7 320
#endif
#ifndef TTS_CHAIN_BN64_3
#define TTS_CHAIN_BN64_3 160
#endif
#ifndef TTS_CHAIN_BN64_7
#define TTS_CHAIN_BN64_7 128
#endif
#ifndef TTS_CHAIN_OCC64_7
#define TTS_CHAIN_OCC64_7 2
#endif
#ifndef TTS_CHAIN_C64K7
#define TTS_CHAIN_C64K7 0          // chain the k = 7 resblock at C = 64 too
#endif
#ifndef TTS_CHAIN_OCC32_3
#define TTS_CHAIN_OCC32_3 3
#endif
#ifndef TTS_CHAIN_OCC32_7
#define TTS_CHAIN_OCC32_7 3
#endif
#ifndef TTS_CHAIN_OCC64_3
#define TTS_CHAIN_OCC64_3 3
#endif
// Measured (same-box A/B, tools/ab.sh): smaller tiles at 4-5 blocks per CU (BN 192/192/96) and a
// third LDS tile that halves the block barriers (2 per pair; LDS then allows 2-3 blocks per CU)
// were both slower (chains 2.15 -> 2.23-2.72 ms per C2 step): the halo recompute and the
// occupancy loss cost more than the barriers.  At C = 32 the per-tile epilogue (bias, lrelu,
// residual, LDS writes) is as long as the tile's 3 MFMAs, so these kernels run at 30-45 % MFMA.
template <>
struct ChainGeom<32, 3> { static constexpr int BN = TTS_CHAIN_BN32_3, OCC = TTS_CHAIN_OCC32_3; };
template <>
struct ChainGeom<32, 7> { static constexpr int BN = TTS_CHAIN_BN32_7, OCC = TTS_CHAIN_OCC32_7; };
#ifndef TTS_CHAIN_C32K11
#define TTS_CHAIN_C32K11 0         // chain the k = 11 resblock at C = 32 too
#endif
#ifndef TTS_CHAIN_BN32_11
#define TTS_CHAIN_BN32_11 256
#endif
template <>
struct ChainGeom<32, 11> { static constexpr int BN = TTS_CHAIN_BN32_11, OCC = 3; };
template <>
struct ChainGeom<64, 3> { static constexpr int BN = TTS_CHAIN_BN64_3, OCC = TTS_CHAIN_OCC64_3; };
template <>
struct ChainGeom<64, 7> { static constexpr int BN = TTS_CHAIN_BN64_7, OCC = TTS_CHAIN_OCC64_7; };

#ifndef TTS_CHAIN_C128K3
#define TTS_CHAIN_C128K3 0         // chain the k = 3 resblock at C = 128 too
#endif
#ifndef TTS_CHAIN_BN128_3
#define TTS_CHAIN_BN128_3 96
#endif
#ifndef TTS_CHAIN_OCC128_3
#define TTS_CHAIN_OCC128_3 2
#endif
template <>
struct ChainGeom<128, 3> { static constexpr int BN = TTS_CHAIN_BN128_3, OCC = TTS_CHAIN_OCC128_3; };

constexpr int CHAIN_D0 = 1, CHAIN_D1 = 3, CHAIN_D2 = 5;  // HiFi-GAN V1/V2 dilations

// tile height by dtype: the bf16 C = 64 k = 3 chain keeps 128 rows (at 160 its f32 epilogue
// arithmetic spills past 168 VGPRs; the f16 form fits: 142)
#ifndef TTS_CHAIN_BN64_3_BF16
#define TTS_CHAIN_BN64_3_BF16 128
#endif
#ifndef TTS_CHAIN_D64_BF16
#define TTS_CHAIN_D64_BF16 3
#endif
template <typename T, int C, int K>
constexpr int chain_bn() {
  return C == 64 && K == 3 && !__is_same(T, half_t) ? TTS_CHAIN_BN64_3_BF16 : ChainGeom<C, K>::BN;
}

template <int C, int K, int BNV = ChainGeom<C, K>::BN>
struct ChainPlan {
  static constexpr int BN = BNV;
  static constexpr int A = (K - 1) / 2;
  static constexpr int DIL[3] = {CHAIN_D0, CHAIN_D1, CHAIN_D2};
  // first row each pair's output must cover (s[3] = H0)
  static constexpr int s(int p) { return p == 0 ? 0 : s(p - 1) + A * (DIL[p - 1] + 1); }
  static constexpr int H0 = s(3);
  static constexpr int NR = BN + 2 * H0;
  static constexpr int lo1(int p) { return s(p) + A * DIL[p]; }
  static constexpr int nt1(int p) { return (NR - 2 * lo1(p) + 15) / 16; }
  static constexpr int lo2(int p) { return s(p + 1); }
  static constexpr int nt2(int p) { return (NR - 2 * lo2(p) + 15) / 16; }
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  // rows touched: staging [0, NR); conv1 reads up to lo1 + 16*nt1 + A*d, conv2 up to lo2 + 16*nt2 + A
  static constexpr int top(int p) {
    return cmax(lo1(p) + 16 * nt1(p) + A * DIL[p], lo2(p) + 16 * nt2(p) + A);
  }
  static constexpr int NRA = cmax(NR, cmax(top(0), cmax(top(1), top(2))));
};

template <typename T, int C, int K>
static size_t chain_lds_bytes() {
  return (size_t)2 * ChainPlan<C, K, chain_bn<T, C, K>()>::NRA * PairGeom<C>::RS;
}

// 4 x T: (y + h), rounded as epi_row does for the intermediate h' (scale 1, no accumulate)
template <typename T>
__device__ inline uint2 epi_add4(uint2 y, uint2 h) {
  if constexpr (__is_same(T, half_t)) {
    const half4 v = *reinterpret_cast<const half4*>(&y) + *reinterpret_cast<const half4*>(&h);
    return *reinterpret_cast<const uint2*>(&v);
  } else {
    return uint2{bf16x2_pack(bf16x2_unpack(y.x) + bf16x2_unpack(h.x)),
                 bf16x2_pack(bf16x2_unpack(y.y) + bf16x2_unpack(h.y))};
  }
}
template <typename T>
__device__ inline uint2 lrelu4(uint2 v, float slope) {  // 4 x T, 0 <= slope <= 1 (lrelu_unit on 4 lanes)
  if constexpr (__is_same(T, half_t)) {
    half4 h = *reinterpret_cast<const half4*>(&v);
    h = __builtin_elementwise_max(h, h * (half_t)slope);
    return *reinterpret_cast<const uint2*>(&h);
  } else {
    return uint2{lrelu_bf16x2(v.x, slope), lrelu_bf16x2(v.y, slope)};
  }
}

template <typename T, int C, int K>
__global__ __launch_bounds__(256, (ChainGeom<C, K>::OCC)) void mrf_chain_kernel(MrfChainParams p) {
  using G = PairGeom<C>;
  using P = ChainPlan<C, K, chain_bn<T, C, K>()>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int BN = P::BN, WM = C / 32, WN = 4 / WM, RS = G::RS, A = P::A;  // 32 channels per wave
  // weight ring depth (k-steps ahead): one shallower for the tall bf16 C = 64 tile, whose f32
  // epilogue arithmetic otherwise pushes it past 168 VGPRs (same k-step order: bit-identical)
  constexpr int D = !__is_same(T, half_t) && C == 64 && BN > 128 ? TTS_CHAIN_D64_BF16 : G::D;
  constexpr int NTHR = 256, MT = 2, KS = C / 32, S = K * KS, VPR = C / 8;
  constexpr int H0 = P::H0, NR = P::NR, NRA = P::NRA;
  // bf16 (f32 epilogue arithmetic) on the tall C = 64 tile: the MRF-sum rows are loaded after
  // the last epilogue instead of during it (held across it they push the kernel past 168 VGPRs)
  constexpr bool SIN_LATE = !__is_same(T, half_t) && C == 64 && BN > 128;
  static_assert(WM * WN * 64 == NTHR && WM * 32 == C, "wave grid");
  static_assert(BN % 16 == 0 && (NR - 2 * P::lo2(2)) == BN, "last conv covers exactly the output rows");
  auto swz = [](int r) { return ((r * G::SW_MUL) >> G::SW_S) & G::SW_M; };
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Hs = smem;
  char* GT = smem + NRA * RS;

  int b, tile0;
  if (!xcd_tile((p.T + BN - 1) / BN, p.B, b, tile0)) return;
  const int n0 = tile0 * BN;
  const int len = min(p.len[b], p.T);
  if (n0 >= len) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = WM == 1 ? 0 : wave % WM, wn = WN == 1 ? 0 : wave / WM;
  const int l15 = lane & 15, lq = lane >> 4;
  const int r0g = n0 - H0;             // utterance row of LDS row 0
  const float slope = p.slope;
  const int ch0 = 32 * wm + 4 * lq;    // + 16*mt: this lane's 4 output channels
  // per-lane swizzle tables of the 8 row phases (every conv's rows and taps are compile-time
  // offsets from l15): B-fragment chunks and epilogue bytes without per-step swizzle arithmetic
  int sw8[8], ep8[8];
  pair_sw8<C>(sw8, l15, lq);
  pair_ep8<C>(ep8, l15, lq);
  const int lrow = (16 * wn + l15) * RS;  // the lane's row in its wave's tile 0, LDS row 0 based
  // Interior blocks (every LDS row inside the utterance) store the epilogues unmasked; only the
  // first and last blocks of an utterance zero the rows outside it (the unfused convs' padding)
  const bool edge = r0g < 0 || r0g + NRA > len;
  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;
  constexpr int TU = 16 * WN * RS;     // bytes from a wave's tile u to its tile u + 1

  Frag ring[D][MT];
  auto preload = [&](const void* w) __attribute__((always_inline)) {
    const char* wp = reinterpret_cast<const char*>(w) + (long long)(2 * wm) * S * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (i < S)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) ring[i][mt] = *reinterpret_cast<const Frag*>(wp + ((long long)mt * S + i) * 1024);
  };
  // the running conv's bias: the accumulators start at it (TTS_BIAS_ACC); each is loaded
  // before the weight preload of its conv (in-order vmcnt)
  f32x4 bias[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) bias[mt] = *reinterpret_cast<const f32x4*>(p.b1[0] + ch0 + 16 * mt);
  preload(p.w1[0]);

  // ---- stage h (Hs) and g = lrelu(h) (GT), zero outside the utterance ----
  {
    const int cc = tid % VPR, rr0 = tid / VPR;
    constexpr int rstep = NTHR / VPR;
    const T* xc = X + cc * 8;
    for (int rb = rr0; rb < NR; rb += PAIR_SU * rstep) {
      uint4 v[PAIR_SU];
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int gr = min(max(r0g + min(rb + i * rstep, NR - 1), 0), len - 1);
        v[i] = *reinterpret_cast<const uint4*>(xc + (long long)gr * C);
      }
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int r = rb + i * rstep;
        const int gr = r0g + r;
        const bool in = gr >= 0 && gr < len;
        const uint4 h = in ? v[i] : uint4{0u, 0u, 0u, 0u};
        const uint4 g = lrelu_unit<T>(h, slope);  // consumed unconditionally (waitcnt)
        if (r < NR) {
          const int o = r * RS + ((cc ^ swz(r)) << 4);
          *reinterpret_cast<uint4*>(Hs + o) = h;
          *reinterpret_cast<uint4*>(GT + o) = g;
        }
      }
    }
  }
  __syncthreads();

  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.T * C;
  constexpr int NIT = (BN * VPR + NTHR - 1) / NTHR;  // row-pass pieces per thread (the last may be partial)
  uint4 sin[NIT];
  // the MRF-sum rows the row pass adds (no records when not accumulating)
  auto load_sin = [&]() __attribute__((always_inline)) {
    const auto yrsrc = __builtin_amdgcn_make_buffer_rsrc(Y, 0, p.accum ? len * C * (int)sizeof(T) : 0, 0x00020000);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NTHR;
      const int e = min(n0 + idx / VPR, len - 1) * C + (idx % VPR) * 8;
      sin[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yrsrc, e * (int)sizeof(T), 0, 0));
    }
  };
  auto pair = [&](auto PI) __attribute__((always_inline)) {
    constexpr int Q = decltype(PI)::value;
    constexpr int DQ = P::DIL[Q];
    constexpr int LO1 = P::lo1(Q), NT1 = P::nt1(Q), NU1 = (NT1 + WN - 1) / WN;
    constexpr int LO2 = P::lo2(Q), NT2 = P::nt2(Q), NU2 = (NT2 + WN - 1) / WN;
    const char* w1 = reinterpret_cast<const char*>(p.w1[Q]) + (long long)(2 * wm) * S * 1024 + lane * 16;
    const char* w2 = reinterpret_cast<const char*>(p.w2[Q]) + (long long)(2 * wm) * S * 1024 + lane * 16;

    // conv1: T rows [LO1, LO1 + 16 NT1) read G rows (row - A*DQ) + tap*DQ
    {
      f32x4 acc1[NU1][MT];
#pragma unroll
      for (int u = 0; u < NU1; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc1[u][mt] = acc_init(bias[mt]);
      constexpr int RB1 = LO1 - A * DQ;
      pair_conv<T, C, S, NU1, D, MT, false, TU, RB1, DQ>(acc1, ring, w1, GT + RB1 * RS + lrow, DQ * RS, DQ, RB1 + l15, lq,
                                                         16 * (min(wn + WN * (NU1 - 1), NT1 - 1) - wn) * RS, sw8);
      __builtin_amdgcn_sched_barrier(0);
      const f32x4 b1v[MT] = {bias[0], bias[1]};  // conv1's bias for its epilogue (no-op with TTS_BIAS_ACC)
      // conv2's bias before the weight preload: in-order vmcnt
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) bias[mt] = *reinterpret_cast<const f32x4*>(p.b2[Q] + ch0 + 16 * mt);
      preload(p.w2[Q]);  // conv2's first steps in flight during the epilogue
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();  // T overwrites G
      auto epi1 = [&](auto EDGE) __attribute__((always_inline)) {
        int eo[MT];  // the lane's bytes in the wave's tile 0 (tile u: + u * TU)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) eo[mt] = LO1 * RS + lrow + (ep8[LO1 & 7] ^ ((2 * wm + mt) << 5));
        const int gr0 = r0g + LO1 + 16 * wn + l15;
#pragma unroll
        for (int u = 0; u < NU1; ++u)
          if (NT1 % WN == 0 || wn + WN * u < NT1) {
            const bool valid = !decltype(EDGE)::value || (unsigned)(gr0 + 16 * WN * u) < (unsigned)len;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              uint2 pk = epi_conv1<T>(acc1[u][mt], b1v[mt], slope);
              if (!valid) pk = uint2{0u, 0u};
              *reinterpret_cast<uint2*>(GT + eo[mt] + u * TU) = pk;
            }
          }
      };
      if (edge) epi1(std::true_type{}); else epi1(std::false_type{});
      __syncthreads();
    }
    // conv2: output rows [LO2, LO2 + 16 NT2) read T rows (row - A) + tap
    {
      f32x4 acc2[NU2][MT];
#pragma unroll
      for (int u = 0; u < NU2; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc2[u][mt] = acc_init(bias[mt]);
      constexpr int RB2 = LO2 - A;
      pair_conv<T, C, S, NU2, D, MT, false, TU, RB2, 1>(acc2, ring, w2, GT + RB2 * RS + lrow, RS, 1, RB2 + l15, lq,
                                                        16 * (min(wn + WN * (NU2 - 1), NT2 - 1) - wn) * RS, sw8);
      __builtin_amdgcn_sched_barrier(0);
      const f32x4 b2v[MT] = {bias[0], bias[1]};  // conv2's bias for its epilogue (no-op with TTS_BIAS_ACC)
      if constexpr (Q < 2) {
        // the next pair's conv1 bias before its weight preload: in-order vmcnt
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) bias[mt] = *reinterpret_cast<const f32x4*>(p.b1[Q + 1] + ch0 + 16 * mt);
        preload(p.w1[Q + 1]);
      } else if constexpr (!SIN_LATE) {  // MRF-sum rows in flight during the last epilogue
        load_sin();
      }
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();  // T no longer read
      auto epi2 = [&](auto EDGE) __attribute__((always_inline)) {
        int eo[MT];  // the lane's bytes in the wave's tile 0 (tile u: + u * TU)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) eo[mt] = LO2 * RS + lrow + (ep8[LO2 & 7] ^ ((2 * wm + mt) << 5));
        const int gr0 = r0g + LO2 + 16 * wn + l15;
#pragma unroll
        for (int u = 0; u < NU2; ++u)
          if (NT2 % WN == 0 || wn + WN * u < NT2) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              const int o = eo[mt] + u * TU;
              const uint2 y = epi_conv2<T>(acc2[u][mt], b2v[mt]);
              if constexpr (Q < 2) {
                const bool valid = !decltype(EDGE)::value || (unsigned)(gr0 + 16 * WN * u) < (unsigned)len;
                const uint2 h = epi_add4<T>(y, *reinterpret_cast<const uint2*>(Hs + o));
                *reinterpret_cast<uint2*>(Hs + o) = h;
                *reinterpret_cast<uint2*>(GT + o) = valid ? lrelu4<T>(h, slope) : uint2{0u, 0u};
              } else {
                *reinterpret_cast<uint2*>(GT + o) = y;  // row pass: epi_row(y, h, S)
              }
            }
          }
      };
      if (edge) epi2(std::true_type{}); else epi2(std::false_type{});
      __syncthreads();
    }
  };
  pair(std::integral_constant<int, 0>{});
  pair(std::integral_constant<int, 1>{});
  pair(std::integral_constant<int, 2>{});
  if constexpr (SIN_LATE) load_sin();

  // ---- row pass: y = ((accum ? S : 0) + (y2 + h2)) * scale over rows [n0, n0 + BN) ----
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = tid + it * NTHR;
    const int o = idx / VPR, c8 = idx % VPR;
    const int gr = n0 + o;
    if ((BN * VPR % NTHR != 0 && idx >= BN * VPR) || gr >= len) continue;
    const int r = H0 + o;
    const int off = r * RS + ((c8 ^ swz(r)) << 4);
    T* dst = Y + (long long)gr * C + c8 * 8;
    const uint4 y = *reinterpret_cast<const uint4*>(GT + off);
    const uint4 h = *reinterpret_cast<const uint4*>(Hs + off);
    store16<TTS_ROW_STORE>(Y, (int)((dst - Y) * (long long)sizeof(T)), epi_row<T>(y, h, p.accum, sin[it], p.scale));
  }
}

template <typename T, int C, int K>
static hipError_t launch_chain_t(const MrfChainParams& p, hipStream_t s) {
  constexpr int BN = chain_bn<T, C, K>();
  const size_t lds = chain_lds_bytes<T, C, K>();
  static_assert(2 * ChainPlan<C, K, BN>::NRA * PairGeom<C>::RS * ChainGeom<C, K>::OCC <= 160 * 1024, "LDS for OCC blocks per CU");
  dim3 grid(xcd_grid((p.T + BN - 1) / BN, p.B));
  hipLaunchKernelGGL((mrf_chain_kernel<T, C, K>), grid, dim3(256), lds, s, p);
  return hipGetLastError();
}

bool mrf_chain_supported(int dtype, int C, int k, const int* dil, int npair) {
  if (!(dtype == DT_F16 || dtype == DT_BF16) || npair != 3) return false;
  if (dil[0] != CHAIN_D0 || dil[1] != CHAIN_D1 || dil[2] != CHAIN_D2) return false;
  return (C == 32 && (k == 3 || k == 7 || (TTS_CHAIN_C32K11 && k == 11))) ||
         (C == 64 && (k == 3 || (TTS_CHAIN_C64K7 && k == 7))) || (TTS_CHAIN_C128K3 && C == 128 && k == 3);
}

hipError_t mrf_chain_launch(int dtype, int C, int k, const MrfChainParams& p, hipStream_t s) {
  if (!(p.slope >= 0.f && p.slope <= 1.f)) return hipErrorInvalidValue;  // lrelu_unit / epi_conv1
  const bool f16 = dtype == DT_F16;
  if (C == 32 && k == 3) return f16 ? launch_chain_t<half_t, 32, 3>(p, s) : launch_chain_t<bf16_t, 32, 3>(p, s);
  if (C == 32 && k == 7) return f16 ? launch_chain_t<half_t, 32, 7>(p, s) : launch_chain_t<bf16_t, 32, 7>(p, s);
#if TTS_CHAIN_C32K11
  if (C == 32 && k == 11) return f16 ? launch_chain_t<half_t, 32, 11>(p, s) : launch_chain_t<bf16_t, 32, 11>(p, s);
#endif
  if (C == 64 && k == 3) return f16 ? launch_chain_t<half_t, 64, 3>(p, s) : launch_chain_t<bf16_t, 64, 3>(p, s);
#if TTS_CHAIN_C128K3
  if (C == 128 && k == 3) return f16 ? launch_chain_t<half_t, 128, 3>(p, s) : launch_chain_t<bf16_t, 128, 3>(p, s);
#endif
#if TTS_CHAIN_C64K7
  if (C == 64 && k == 7) return f16 ? launch_chain_t<half_t, 64, 7>(p, s) : launch_chain_t<bf16_t, 64, 7>(p, s);
#endif
  return hipErrorInvalidValue;
}

}  // namespace tts
