// Fused HiFi-GAN ResBlock pair, one launch per (dilation) pair of an MRF stage:
//
//   t  = lrelu( conv_{k,d}( lrelu(h) ) + b1 )          (oracle: vocoder.resblock, one q)
//   h' = conv_{k,1}( t ) + b2 + h
//   out = h'                      (accum = 0)       next pair's input
//   S   = (S + h') * scale        (accum = 1)       MRF sum over resblocks (scale 1/3 last)
//
// A block owns BN output rows.  It stages its input tile once from HBM as g = lrelu(h)
// (rows n0-a1-a2 .. n0+BN+a1+a2, a1 = d(k-1)/2, a2 = (k-1)/2; zero outside the utterance)
// in LDS ("G"), computes conv1 for the BN + 2*a2 rows conv2 needs, writes t over G ("T",
// after a barrier: both tiles at once would not leave 3 blocks per CU), runs conv2 for
// the BN output rows, stages the output tile in LDS and leaves through 16-byte row pieces,
// adding the residual h from the input rows (L2-hot: the block just staged them) and, for
// the last pair of a resblock, the running MRF sum.  HBM traffic per pair: read h once
// (+ halo, mostly L2), write h' once (S: read + write).
//
// Why pairs, not whole stages (round 1's mrf_fused kernel, removed) or single convs (conv_xres): a whole-stage
// tile must carry the receptive-field halo of all three pairs of a resblock (60 rows per
// side at k=11) and recompute it in every conv -- 55 % (C=64) / 71 % (C=32) of its issued
// MFMA work was useful; a pair recomputes only conv1's 2*a2 <= 10 extra rows.  Against two
// single-conv launches a pair saves t's HBM round trip and the residual pass.
//
// Tile size: weights are streamed from L2 per block, so a block's L2 traffic is dominated
// by its 2*k*C*C weight elements; BN = 512 / 256 / 128 rows at C = 32 / 64 / 128 keeps
// that near 1.4 KB per row (measured: at BN = 128, C = 64 the L2 request rate sat at the
// per-CU L2 limit).
//
// MFMA: v_mfma_f32_16x16x32_{f16,bf16}, M = output channels (2 x 16 per wave), N = time
// rows in 16-row tiles (fine tiles keep the 8 + 1 conv1 tiles per wave balanced),
// K = taps x C.  Weights are fragment-packed on the host (frag_pack16, runtime.h) so each
// wave's A fragment is one contiguous 1 KiB load, streamed through a 4-step register ring
// (no barriers inside a conv).  Activation tiles are XOR-swizzled (PairGeom).
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "mrf_tile.h"
#include "switches.h"

#ifndef TTS_PAIR_C256
#define TTS_PAIR_C256 1  // stage 0 (C = 256) as pair launches; 0: single convs (conv_xres)
#endif
#ifndef TTS_PAIR_MTO_MIN
#define TTS_PAIR_MTO_MIN 64  // pair_conv's M-tile-outer MFMA order from this channel count up
#endif

#include <algorithm>

#ifndef TTS_PAIR_STAMP
#define TTS_PAIR_STAMP 0  // diagnostic builds only: per-block phase timestamps (tools/pair_stamps.py)
#endif

namespace tts {

#define HIP_RETURN_IF_ERR(expr)         \
  do {                                  \
    const hipError_t e_ = (expr);       \
    if (e_ != hipSuccess) return e_;    \
  } while (0)

#if TTS_PAIR_STAMP
// Phase timestamps of the pair launches whose (C, k, d) match g_pair_stamp_target (the last such
// launch of the workload wins), one record of 16 words per block: s_memtime at entry / input tile
// staged / conv1 done / T written / conv2 done / output tile staged / row pass issued,
// s_memrealtime at entry and end, and the hardware ids (XCC, SE, CU).  Never built into the product library.
__device__ int g_pair_stamp_target[3];
__device__ unsigned long long g_pair_stamp[1 << 21];
#endif

// conv_post fused into the vocoder's last pair (POST): the block computes PAIR_PO extra output
// rows per side so conv_post's halo (post_k <= 2*PAIR_PO + 1 taps) is in the block
constexpr int PAIR_PO = 8;

// Short-tile geometry: BN / DIV output rows per block, everything else as PairGeom<C>.  The
// launcher picks it when the full-height grid leaves most CUs idle (the streamed vocoder's
// stage 0 at batch 8: 48 blocks for 256 CUs; see pair_div).  A row's
// arithmetic (k-step order, roundings) does not depend on the tile height, so the output is
// bit-identical to the full-height launch (tests/test_vocoder_gpu.py).
// Full-height output rows per block by (C, k).  A multiple of 16 spends most of a conv1 tile on
// the 2*a2 halo rows (k = 3 at C = 256: five 16-row tiles for 66 rows, conv2 four for 64): a height
// that makes conv1's BN + 2*a2 rows a whole number of tiles leaves the rounding to conv2 (k = 3
// at C = 256: 78 rows, ten tiles in all for 78 rows instead of nine for 64; the weight stream
// per row drops by the same 18 %).  At C = 64 (two waves along the rows) the height also makes
// conv1's tile count even, so no wave repeats a tile.  Any height works: a row's arithmetic does
// not depend on it.  Same-box A/B (profiles/r03i_ab_tile_heights.txt): C = 256 k = 3 / 7 pairs
// 976 -> 1011 / 1087 -> 1142 TF/s, C = 128 k = 3 996 -> 1039, C = 32 k = 11 963 -> 980.  Round 4
// (profiles/r04o_ab_c256_tile_heights.txt): at C = 256 the k = 7 / 11 pairs stream 2*k*C*C*2 =
// 1.8 / 2.9 MB of weights per block from L2, so taller tiles (106 / 86 rows, as tall as the LDS of
// two blocks per CU and 256 VGPRs allow) cut the weight bytes per row by 30 / 25 %: k = 7 pairs
// 356 -> 341 us, k = 11 574 -> 558 us (stage-0 pairs -99 us per C2 step), bit-identical; k = 3 at
// 110 rows (profiles/r04q_ab_c256_k3_tile_heights.txt): 169 -> 157 us per pair.
#ifndef TTS_PBN_256_3
#define TTS_PBN_256_3 110  // conv1 7 tiles (112 rows), 254 VGPRs; round 3: 78 (5 tiles)
#endif
#ifndef TTS_PBN_256_7
#define TTS_PBN_256_7 106  // conv1 7 tiles (112 rows); round 3: 74 (5 tiles)
#endif
#ifndef TTS_PBN_256_11
#define TTS_PBN_256_11 86  // conv1 6 tiles (96 rows); the G tile of d = 5 (146 rows, 75 KB) still fits two blocks per CU
#endif
#ifndef TTS_PBN_128_3
#define TTS_PBN_128_3 142
#endif
#ifndef TTS_PBN_128_11
#define TTS_PBN_128_11 128
#endif
#ifndef TTS_PBN_32_11
#define TTS_PBN_32_11 502
#endif
#ifndef TTS_PBN_128_7
#define TTS_PBN_128_7 138
#endif
#ifndef TTS_PBN_64_7
#define TTS_PBN_64_7 282
#endif
#ifndef TTS_PBN_64_11
#define TTS_PBN_64_11 278
#endif
template <int C, int K>
constexpr int pair_bn() {
  if (C == 256 && K == 3) return TTS_PBN_256_3;
  if (C == 256 && K == 7) return TTS_PBN_256_7;
  if (C == 256 && K == 11) return TTS_PBN_256_11;
  if (C == 128 && K == 3) return TTS_PBN_128_3;
  if (C == 32 && K == 11) return TTS_PBN_32_11;
  if (C == 128 && K == 7) return TTS_PBN_128_7;
  if (C == 128 && K == 11) return TTS_PBN_128_11;
  if (C == 64 && K == 7) return TTS_PBN_64_7;
  if (C == 64 && K == 11) return TTS_PBN_64_11;
  return PairGeom<C>::BN;
}

#ifndef TTS_P256K11_D
#define TTS_P256K11_D 2  // weight-ring depth of the full-height C = 256 k = 11 pairs (the others: TTS_P256_D)
#endif
#ifndef TTS_P32K11_OCC
#define TTS_P32K11_OCC 3
#endif
#ifndef TTS_PAIR_SHORT_D256
#define TTS_PAIR_SHORT_D256 4  // weight-ring depth (k-steps) of the C = 256 short tiles (full height: 2)
#endif
// A/B builds only: the row pass's residual rows loaded into registers right after the input tile
// is staged (L2-hot then) and held through both convs, instead of re-read at the end (where they
// have left the 4 MB L2: the 1.48x FETCH of profiles/r05z_pmc_traffic_c2.json).  The registers
// cost the third block per CU (OCC 2); C = 256 (already two blocks, 254 VGPRs) and conv_post
// keep the re-read.  Measured in profiles/r05o_ab_resreg.txt.
#ifndef TTS_PAIR_RESREG
#define TTS_PAIR_RESREG 0
#endif
#ifndef TTS_PAIR_RESREG_ONLYC
#define TTS_PAIR_RESREG_ONLYC 0  // A/B builds: only pairs of this channel count (0: every C <= 128)
#endif
#ifndef TTS_PAIR_RESREG_OCC
#define TTS_PAIR_RESREG_OCC 2    // blocks per CU the RESREG register budget is sized for
#endif
template <int C, int DIV, int K = 0, bool POST = false>
struct PairGeomS : PairGeom<C> {
  static constexpr bool RESREG = TTS_PAIR_RESREG && C <= 128 && !POST &&
                                 (TTS_PAIR_RESREG_ONLYC == 0 || C == TTS_PAIR_RESREG_ONLYC);
  static constexpr int BN = DIV == 1 && K > 0 && !POST ? pair_bn<C, K>() : PairGeom<C>::BN / DIV;
  // short tiles do few MFMAs per k-step (one row tile per wave), so the weight ring's L2 round
  // trips are exposed unless it runs further ahead; the depth only moves loads earlier (same
  // k-step order: bit-identical).  C = 256, D 2 -> 4 (profiles/r04t_ab_short_ring.txt): the C5
  // chunk's stage-0 pairs 337 -> 266 us, C5 3.44 -> 3.36 ms (8: 270 us)
  static constexpr int D = DIV > 1 && C == 256 ? TTS_PAIR_SHORT_D256
                           : DIV == 1 && C == 256 && K == 11 ? TTS_P256K11_D
                                                             : PairGeom<C>::D;
  // blocks per CU the register budget is sized for (the C = 32 k = 11 pairs without conv_post
  // may take a fourth: TTS_P32K11_OCC; the HiFi-GAN V3 C = 64 k = 5 pair spills at three)
  static constexpr int OCC = RESREG                                  ? TTS_PAIR_RESREG_OCC
                             : C == 32 && K == 11 && !POST && DIV == 1 ? TTS_P32K11_OCC
                             : C == 64 && K == 5                    ? 2
                                                                    : PairGeom<C>::OCC;
};

// LDS bytes of one launch (G tile incl. conv1 overrun rows, T tile; >= output staging tile of
// 16 * NT2 rows: conv2's last tile may run past the BO output rows)
template <int C, int DIV = 1, int K = 0, bool POST = false>
static size_t pair_lds_bytes(int k, int d, bool post) {
  using G = PairGeomS<C, DIV, K, POST>;
  const int a1 = (k - 1) / 2 * d, a2 = (k - 1) / 2;
  const int bo = G::BN + (post ? 2 * PAIR_PO : 0);
  const int nt1 = (bo + 2 * a2 + 15) / 16;
  const int nt2 = (bo + 15) / 16;

  const size_t g = (size_t)(16 * nt1 + 2 * a1) * G::RS;
  const size_t t = (size_t)16 * nt1 * G::RS;
  return std::max(std::max(g, t), (size_t)16 * nt2 * (C * 2 + 16));
}

// OUTACT: the stored rows are LeakyReLU(p.out_slope) of the row pass's values (a stage's last
// pair, whose MRF sum only the next upsampler reads; MrfPairParams::out_act)
template <typename T, int C, int K, bool POST = false, int DIV = 1, bool OUTACT = false>
__global__ __launch_bounds__((64 * PairGeom<C>::WM * PairGeom<C>::WN), (PairGeomS<C, DIV, K, POST>::OCC)) void mrf_pair_kernel(
    MrfPairParams p) {
  using G = PairGeomS<C, DIV, K, POST>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int BN = G::BN, WM = G::WM, WN = G::WN, RS = G::RS;
  constexpr int D = G::D;              // weight ring depth (k-steps)
  auto swz = [](int r) { return ((r * G::SW_MUL) >> G::SW_S) & G::SW_M; };  // chunk XOR of row r
  constexpr int NTHR = 64 * WM * WN;    // 4 waves; 8 at C = 256 with 128-row tiles
  constexpr int KS = C / 32;           // k-steps (of 32 channels) per tap
  constexpr int MT = G::MT;            // 16-channel M tiles per wave
  constexpr int S = K * KS;            // k-steps per conv
  constexpr int A2 = (K - 1) / 2;
  constexpr int PO = POST ? PAIR_PO : 0;  // extra output rows per side (conv_post's halo)
  constexpr int BO = BN + 2 * PO;      // output rows: block row o <-> utterance row n0 - PO + o
  constexpr int RT = BO + 2 * A2;      // conv1 rows conv2 needs
  constexpr int NT1 = (RT + 15) / 16;  // conv1 tiles (block)
  constexpr int NU1 = (NT1 + WN - 1) / WN;  // conv1 tiles per wave (the last may be a repeat)
  constexpr int NT2 = (BO + 15) / 16;  // conv2 tiles (block; the last may run past BO: not stored)
  static_assert(NT2 <= NT1, "conv2's overrun rows (past BO) read inside the G / T region");
  constexpr int NU2 = (NT2 + WN - 1) / WN;  // conv2 tiles per wave (the last may be a repeat)
  static_assert(!POST || (C == 32 && BN == 512 && NTHR == 256), "conv_post fusion: C = 32, two samples per thread");
  constexpr int VPR = C / 8;           // 16-byte pieces per row
  constexpr int YS16 = C * 2 + 16;     // output tile staging row stride
  static_assert(WM * WN * 64 == NTHR && WM * 16 * MT == C, "wave grid");
  static_assert(NTHR % VPR == 0, "staging");
  static_assert(2 * A2 <= 16, "conv1 overrun within one tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];

#if TTS_PAIR_STAMP
  unsigned long long stp[7] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0, 0, 0};
  const unsigned long long rtp0 = __builtin_amdgcn_s_memrealtime();
  const bool stamp_on = C == g_pair_stamp_target[0] && p.k == g_pair_stamp_target[1] && p.d == g_pair_stamp_target[2];
#define TTS_PSTAMP(i_) stp[i_] = __builtin_amdgcn_s_memtime()
#else
#define TTS_PSTAMP(i_) (void)0
#endif
  int b, tile0;
  if (!xcd_tile((p.T + BN - 1) / BN, p.B, b, tile0)) return;
  const int n0 = tile0 * BN;
  const int len = min(p.len[b], p.T);
  const int tid = threadIdx.x;
  if (n0 >= len) {
    if constexpr (POST) {  // conv_post's grid covered every row: zeros past the utterance
      if (n0 + tid < p.T) p.wav[b * p.swb + n0 + tid] = 0.f;
      if (n0 + tid + 256 < p.T) p.wav[b * p.swb + n0 + tid + 256] = 0.f;
    }
    return;
  }
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = WM == 1 ? 0 : wave % WM, wn = WN == 1 ? 0 : wave / WM;
  const int l15 = lane & 15, lq = lane >> 4;
  const int d = p.d;
  const int a1 = A2 * d;
  const int RG = BO + 2 * (a1 + A2);
  char* Gs = smem;
  char* Ts = smem;                     // T overwrites G after conv1
  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;
  const float slope = p.slope;
  const int ch0 = 16 * MT * wm + 4 * lq;  // + 16*mt: this lane's 4 output channels

  // weights: [C/16][k][KS][64][8] -> step s of m-tile mb at (mb*S + s) KiB
  const char* w1 = reinterpret_cast<const char*>(p.w1) + (long long)(MT * wm) * S * 1024 + lane * 16;
  const char* w2 = reinterpret_cast<const char*>(p.w2) + (long long)(MT * wm) * S * 1024 + lane * 16;
  // conv1's bias first (the accumulators start at it; in-order vmcnt), then its first weight steps
  f32x4 bias1[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) bias1[mt] = *reinterpret_cast<const f32x4*>(p.b1 + ch0 + 16 * mt);
  Frag ring[D][MT];
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < S)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) ring[i][mt] = *reinterpret_cast<const Frag*>(w1 + ((long long)mt * S + i) * 1024);

  // ---- stage g = lrelu(h) (zero outside the utterance) ----
  {
    const int cc = tid % VPR, r0 = tid / VPR;
    constexpr int rstep = NTHR / VPR;
    const int gs = n0 - PO - a1 - A2;
    const T* xc = X + cc * 8;
    if (gs >= 0 && gs + RG <= len) {  // interior tile: no clamps, no masks
      for (int rb = r0; rb < RG; rb += PAIR_SU * rstep) {
        uint4 v[PAIR_SU];
#pragma unroll
        for (int i = 0; i < PAIR_SU; ++i)
          v[i] = *reinterpret_cast<const uint4*>(xc + (long long)(gs + min(rb + i * rstep, RG - 1)) * C);
#pragma unroll
        for (int i = 0; i < PAIR_SU; ++i) {
          const int r = rb + i * rstep;
          const uint4 g = lrelu_unit<T>(v[i], slope);  // consumed unconditionally (waitcnt)
          if (r < RG) *reinterpret_cast<uint4*>(Gs + r * RS + (cc ^ swz(r)) * 16) = g;
        }
      }
    } else
    for (int rb = r0; rb < RG; rb += PAIR_SU * rstep) {
      uint4 v[PAIR_SU];
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int gr = min(max(gs + min(rb + i * rstep, RG - 1), 0), len - 1);
        v[i] = *reinterpret_cast<const uint4*>(xc + (long long)gr * C);
      }
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int r = rb + i * rstep;
        const int gr = gs + r;
        const uint4 g = lrelu_unit<T>(v[i], slope);
        if (r < RG)
          *reinterpret_cast<uint4*>(Gs + r * RS + (cc ^ swz(r)) * 16) = (gr >= 0 && gr < len) ? g : uint4{0u, 0u, 0u, 0u};
      }
    }
  }
  __syncthreads();
  TTS_PSTAMP(1);

  constexpr int NIT = (BO * VPR + NTHR - 1) / NTHR;  // 16-byte row pieces per thread in the row pass
  uint4 xin[NIT];  // the row pass's residual pieces (load_rows)
  if constexpr (G::RESREG) {  // L2-hot: the block just staged these rows
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NTHR;
      xin[it] = *reinterpret_cast<const uint4*>(X + min(max(n0 - PO + idx / VPR, 0), len - 1) * C + (idx % VPR) * 8);
    }
  }

  // ---- conv1 over T rows [0, 16*NT1): T row t <-> global row n0 - PO - a2 + t ----
  // Tiles are dealt round-robin to the WN waves of an M slice; a wave whose share is one
  // short repeats the block's last tile (straight-line loop, result not stored).
  f32x4 acc1[NU1][MT];
#pragma unroll
  for (int u = 0; u < NU1; ++u)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc1[u][mt] = acc_init(bias1[mt]);
  // (a wave whose share is one short repeats the block's last tile: its offset from tile 0)
  auto last_off = [&](int nt, int nu) { return 16 * (min(wn + WN * (nu - 1), nt - 1) - wn) * RS; };
  pair_conv<T, C, S, NU1, D, MT, (C >= TTS_PAIR_MTO_MIN), 16 * WN * RS>(acc1, ring, w1, Gs + (16 * wn + l15) * RS, d * RS,
                                                                        d, l15, lq, last_off(NT1, NU1));
  __builtin_amdgcn_sched_barrier(0);
  TTS_PSTAMP(2);
  // conv2's bias first, then its first weight steps (in flight during the conv1 epilogue): vmcnt
  // retires in order, so waiting for the bias does not wait for the weights
  f32x4 bias2[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) bias2[mt] = *reinterpret_cast<const f32x4*>(p.b2 + ch0 + 16 * mt);
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < S)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) ring[i][mt] = *reinterpret_cast<const Frag*>(w2 + ((long long)mt * S + i) * 1024);
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();  // T overwrites G: every wave is done reading it
  {
    const f32x4 (&bias)[MT] = bias1;
    int eo[MT];  // this lane's T bytes in the wave's tile 0 (tile u: + u * 16 WN rows)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) eo[mt] = pair_lds4<C>(16 * wn + l15, ch0 + 16 * mt);
    const int gr0 = n0 - PO - A2 + 16 * wn + l15;  // utterance row of the lane's row in tile 0
#pragma unroll
    for (int u = 0; u < NU1; ++u)
      if (NT1 % WN == 0 || wn + WN * u < NT1) {
        const bool valid = (unsigned)(gr0 + 16 * WN * u) < (unsigned)len;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          uint2 pk = epi_conv1<T>(acc1[u][mt], bias[mt], slope);
          if (!valid) pk = uint2{0u, 0u};
          *reinterpret_cast<uint2*>(Ts + eo[mt] + u * 16 * WN * RS) = pk;
        }
      }
  }
  __syncthreads();
  TTS_PSTAMP(3);

  // ---- conv2 over the BN output rows: output row o reads T rows o .. o + 2*a2 ----
  f32x4 acc2[NU2][MT];
#pragma unroll
  for (int u = 0; u < NU2; ++u)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc2[u][mt] = acc_init(bias2[mt]);
  pair_conv<T, C, S, NU2, D, MT, (C >= TTS_PAIR_MTO_MIN), 16 * WN * RS>(acc2, ring, w2, Ts + (16 * wn + l15) * RS, RS, 1,
                                                                        l15, lq, last_off(NT2, NU2));
  __builtin_amdgcn_sched_barrier(0);  // keep the epilogue's loads out of the MFMA tail
  TTS_PSTAMP(4);
  // residual h (input rows) and, for accumulating launches, the MRF-sum rows in flight while
  // the tile is staged.  The sum is read through a buffer descriptor with no records when the
  // launch does not accumulate: the load is issued unconditionally (no branch for the waitcnt
  // pass) and fetches nothing.
  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.T * C;
  const auto yrsrc = __builtin_amdgcn_make_buffer_rsrc(Y, 0, p.accum ? len * C * (int)sizeof(T) : 0, 0x00020000);
  uint4 sin[NIT];
  auto load_rows = [&](bool lx, bool ls) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NTHR;
      const int e = min(max(n0 - PO + idx / VPR, 0), len - 1) * C + (idx % VPR) * 8;
      if (lx) xin[it] = *reinterpret_cast<const uint4*>(X + e);
      if (ls) sin[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yrsrc, e * (int)sizeof(T), 0, 0));
    }
  };
  // with conv_post fused the residual rows wait until the accumulators are staged (registers)
  const f32x4 (&bias)[MT] = bias2;
  load_rows(!POST && !G::RESREG, true);
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();  // T no longer read
  {
    char* ob = smem + (16 * wn + l15) * YS16 + ch0 * 2;  // the lane's output bytes in the wave's tile 0
#pragma unroll
    for (int u = 0; u < NU2; ++u)
      if (NT2 % WN == 0 || wn + WN * u < NT2) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          *reinterpret_cast<uint2*>(ob + u * 16 * WN * YS16 + 32 * mt) = epi_conv2<T>(acc2[u][mt], bias[mt]);
      }
  }
  __syncthreads();
  TTS_PSTAMP(5);
  if constexpr (POST) {
    // final MRF-sum rows (rounded to T as the unfused path stores them) -> lrelu -> LDS tile
    // [BO][32] (chunk c of row r at c ^ ((r >> 2) & 3), conv_post16's layout), then conv_post
    // for the BN rows in conv_post16's arithmetic order
    load_rows(true, false);
    uint4 gv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NTHR;
      const int o = min(idx / VPR, BO - 1), c8 = idx % VPR;
      const int gr = n0 - PO + o;
      const uint4 y = *reinterpret_cast<const uint4*>(smem + o * YS16 + c8 * 16);
      const uint4 v = lrelu_unit<T>(epi_row<T>(y, xin[it], p.accum, sin[it], p.scale), p.post_slope);
      gv[it] = (gr >= 0 && gr < len) ? v : uint4{0u, 0u, 0u, 0u};
    }
    __syncthreads();  // output staging no longer read
    auto slot = [](int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); };
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NTHR;
      if (idx < BO * VPR) *reinterpret_cast<uint4*>(smem + slot(idx / VPR, idx % VPR)) = gv[it];
    }
    __syncthreads();
    const unsigned* wpk = reinterpret_cast<const unsigned*>(p.post_wpk);
    const int r0 = PO - (p.post_k - 1) / 2 + tid;
    float acc0 = p.post_b, acc1 = p.post_b;
    for (int j = 0; j < p.post_k; ++j) {
      const unsigned* wj = wpk + j * (C / 2);
#pragma unroll
      for (int c = 0; c < VPR; ++c) {
        const uint4 a = *reinterpret_cast<const uint4*>(smem + slot(r0 + j, c));
        const uint4 e = *reinterpret_cast<const uint4*>(smem + slot(r0 + 256 + j, c));
        acc0 = Dot2<T>::dot(a.x, wj[4 * c + 0], acc0);
        acc0 = Dot2<T>::dot(a.y, wj[4 * c + 1], acc0);
        acc0 = Dot2<T>::dot(a.z, wj[4 * c + 2], acc0);
        acc0 = Dot2<T>::dot(a.w, wj[4 * c + 3], acc0);
        acc1 = Dot2<T>::dot(e.x, wj[4 * c + 0], acc1);
        acc1 = Dot2<T>::dot(e.y, wj[4 * c + 1], acc1);
        acc1 = Dot2<T>::dot(e.z, wj[4 * c + 2], acc1);
        acc1 = Dot2<T>::dot(e.w, wj[4 * c + 3], acc1);
      }
    }
    const int ta = n0 + tid, tb = ta + 256;
    float* wv = p.wav + b * p.swb;
    if (ta < p.T) wv[ta] = ta < len ? tanhf(acc0) : 0.f;
    if (tb < p.T) wv[tb] = tb < len ? tanhf(acc1) : 0.f;
    return;
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = tid + it * NTHR;
    const int o = idx / VPR, c8 = idx % VPR;
    const int gr = n0 + o;
    if ((BO * VPR % NTHR != 0 && idx >= BO * VPR) || gr >= len) continue;
    T* dst = Y + (long long)gr * C + c8 * 8;
    const uint4 y = *reinterpret_cast<const uint4*>(smem + o * YS16 + c8 * 16);
    uint4 v = epi_row<T>(y, xin[it], p.accum, sin[it], p.scale);
    if constexpr (OUTACT) v = lrelu_unit<T>(v, p.out_slope);
    store16<TTS_ROW_STORE>(Y, (int)((dst - Y) * (long long)sizeof(T)), v);
  }
#if TTS_PAIR_STAMP
  TTS_PSTAMP(6);
  if (stamp_on && tid == 0 && blockIdx.x < (1u << 17)) {
    unsigned long long* r = g_pair_stamp + blockIdx.x * 16;
    for (int i = 0; i < 7; ++i) r[i] = stp[i];
    r[7] = rtp0;
    r[8] = __builtin_amdgcn_s_memrealtime();
    r[9] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)) << 32) |
           (unsigned)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
  }
#endif
}
#undef TTS_PSTAMP

#ifndef TTS_PAIR_SHORT
#define TTS_PAIR_SHORT 128             // short tiles below this many full-height blocks (0: never)
#endif
#ifndef TTS_PAIR_SHORT_DIV
#define TTS_PAIR_SHORT_DIV 4           // tile height divisor of the short tiles
#endif
// Short tiles multiply the L2 weight stream (every block reads the pair's 2*k*C*C weights), so
// they pay only where the full-height grid leaves most CUs idle.  Measured on the C5 windows
// (batch 8, 48 frames, tools/c5_probe.py under rocprofv3): C = 256 at 48 blocks 380 -> 329 us
// for the stage's 9 launches; C = 128 at 192 blocks 167 -> 193 us (slower), C = 32 / 64 neutral.
// TTS_PAIR_DIV=1 / any other value forces full-height / short tiles (tests).
static int pair_div(int C, const MrfPairParams& p, bool post) {
  if (post) return 1;
  const int force = sw(SW_PAIR_DIV);
  if (force >= 0) return force == 1 ? 1 : TTS_PAIR_SHORT_DIV;
  const int bn = C == 32 ? PairGeom<32>::BN : C == 64 ? PairGeom<64>::BN : C == 128 ? PairGeom<128>::BN : PairGeom<256>::BN;
  return (long long)((p.T + bn - 1) / bn) * p.B < TTS_PAIR_SHORT ? TTS_PAIR_SHORT_DIV : 1;
}


// ---------------------------------------------------------------- channel-split form (small grids)
// A pair launch whose full-height grid leaves most CUs idle (the streamed vocoder's first chunk:
// batch 8 x 48 frames, stage 0 at 36 blocks, stage 1 at 192) is bound by the weight stream: every
// block of mrf_pair_kernel reads the pair's 2 k C^2 weights from L2 (2.9 MB for k = 11 at C = 256,
// ~41 us at the per-CU L2 rate of ~70 GB/s: the C5 trace's 42 us per launch,
// profiles/r05j_c5_trace.txt).  Here the two convs are two launches over (row tile, channel slice)
// blocks: each block stages the tile's input rows for every input channel and computes one 64-channel
// slice, reading a quarter (C = 256) or half (C = 128) of a conv's weights; conv1's t rows go
// through an HBM scratch (the engine's free T1 buffer).  Every output element is the same
// k-step sequence (pair_conv: bias-initialised accumulators, taps x 32-channel k-steps in order),
// the same roundings (epi_conv1 -> T, epi_conv2 -> T, epi_row) and the same zeros outside the
// utterance as mrf_pair_kernel, so the result is bit-identical (tests/test_vocoder_gpu.py).
#ifndef TTS_PSPLIT_WM
#define TTS_PSPLIT_WM 4  // waves per block, one 16-channel M tile each (4: a 64-channel slice)
#endif
#ifndef TTS_PSPLIT_NU
#define TTS_PSPLIT_NU 2  // 16-row tiles per wave: 32 rows per block (C5 chunk A/B: 4 -> 2 rows tiles 0.745 -> 0.719 ms, profiles/r05l_ab_pair_split.txt)
#endif
constexpr int PSPLIT_WM = TTS_PSPLIT_WM;
constexpr int PSPLIT_NU = TTS_PSPLIT_NU;
constexpr int PSPLIT_D = 4;   // weight ring depth (k-steps)

template <typename T, int C, int K, bool CONV2, bool OUTACT>
__global__ __launch_bounds__(64 * PSPLIT_WM) void mrf_pair_split_kernel(MrfPairParams p) {
  using G = PairGeom<C>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int WM = PSPLIT_WM, NU = PSPLIT_NU, D = PSPLIT_D, BN = 16 * NU, NTHR = 64 * WM;
  constexpr int RS = G::RS, KS = C / 32, S = K * KS, A2 = (K - 1) / 2, VPR = C / 8;
  constexpr int NSL = C / (16 * WM);   // channel slices
  constexpr int SL = 16 * WM;          // channels per slice
  constexpr int OS = SL * 2 + 16;      // conv2 output staging row stride (bytes)
  static_assert(C % SL == 0 && NTHR % VPR == 0, "geometry");
  auto swz = [](int r) { return ((r * G::SW_MUL) >> G::SW_S) & G::SW_M; };
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int ntile = (p.T + BN - 1) / BN;
  int v = blockIdx.x;
  const int slice = v % NSL;
  v /= NSL;
  const int tile = v % ntile, b = v / ntile;
  if (b >= p.B) return;
  const int n0 = tile * BN;
  const int len = min(p.len[b], p.T);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  const int mtile = slice * WM + wave;  // this wave's 16-channel M tile
  const int ch0 = 16 * mtile + 4 * lq;  // the lane's 4 output channels
  T* Tb = reinterpret_cast<T*>(p.tbuf) + (long long)b * p.T * C;
  if (!CONV2 && n0 >= len) {
    // t rows past the utterance are zero (conv2 reads them as padding)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int row = n0 + 16 * u + l15;
      if (row < p.T) *reinterpret_cast<uint2*>(Tb + (long long)row * C + ch0) = uint2{0u, 0u};
    }
    return;
  }
  if (CONV2 && n0 >= len) return;
  const int d = CONV2 ? 1 : p.d;
  const int a = A2 * d;               // input rows needed past each side of the tile
  const int RG = BN + 2 * a;
  const int gs = n0 - a;              // utterance row of LDS row 0
  const char* wsrc = reinterpret_cast<const char*>(CONV2 ? p.w2 : p.w1) + (long long)mtile * S * 1024 + lane * 16;
  const f32x4 bias = *reinterpret_cast<const f32x4*>((CONV2 ? p.b2 : p.b1) + ch0);
  Frag ring[D][1];
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < S) ring[i][0] = *reinterpret_cast<const Frag*>(wsrc + (long long)i * 1024);

  // ---- stage the input rows: conv1 g = lrelu(h), conv2 t (zero outside the utterance) ----
  {
    const T* src = CONV2 ? Tb : reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;
    const int cc = tid % VPR, r0 = tid / VPR;
    constexpr int rstep = NTHR / VPR;
    for (int rb = r0; rb < RG; rb += PAIR_SU * rstep) {
      uint4 vv[PAIR_SU];
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int gr = min(max(gs + min(rb + i * rstep, RG - 1), 0), len - 1);
        vv[i] = *reinterpret_cast<const uint4*>(src + (long long)gr * C + cc * 8);
      }
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int r = rb + i * rstep;
        const int gr = gs + r;
        const uint4 g = CONV2 ? vv[i] : lrelu_unit<T>(vv[i], p.slope);
        if (r < RG)
          *reinterpret_cast<uint4*>(smem + r * RS + (cc ^ swz(r)) * 16) = (gr >= 0 && gr < len) ? g : uint4{0u, 0u, 0u, 0u};
      }
    }
  }
  __syncthreads();

  f32x4 acc[NU][1];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc[u][0] = acc_init(bias);
  pair_conv<T, C, S, NU, D, 1, false, 16 * RS>(acc, ring, wsrc, smem + l15 * RS, d * RS, d, l15, lq, (NU - 1) * 16 * RS);
  __builtin_amdgcn_sched_barrier(0);

  if constexpr (!CONV2) {
    // t = epi_conv1 -> the scratch (zero past the utterance), as mrf_pair_kernel writes T
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int row = n0 + 16 * u + l15;
      uint2 pk = epi_conv1<T>(acc[u][0], bias, p.slope);
      if (row >= len) pk = uint2{0u, 0u};
      if (row < p.T) *reinterpret_cast<uint2*>(Tb + (long long)row * C + ch0) = pk;
    }
    return;
  } else {
    // conv2 -> T in LDS [BN rows][SL channels], then the row pass of mrf_pair_kernel
    __syncthreads();  // staged rows no longer read
#pragma unroll
    for (int u = 0; u < NU; ++u)
      *reinterpret_cast<uint2*>(smem + (16 * u + l15) * OS + (16 * wave + 4 * lq) * 2) = epi_conv2<T>(acc[u][0], bias);
    __syncthreads();
    constexpr int PPR = SL / 8;                         // 16-byte pieces per row of the slice
    constexpr int NIT = (BN * PPR + NTHR - 1) / NTHR;
    const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;
    T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.T * C;
    const auto yrsrc = __builtin_amdgcn_make_buffer_rsrc(Y, 0, p.accum ? len * C * (int)sizeof(T) : 0, 0x00020000);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NTHR;
      const int o = idx / PPR, c8 = idx % PPR;
      const int gr = n0 + o;
      if ((BN * PPR % NTHR != 0 && idx >= BN * PPR) || gr >= len) continue;
      const int e = gr * C + SL * slice + c8 * 8;
      const uint4 xin = *reinterpret_cast<const uint4*>(X + e);
      const uint4 sin = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yrsrc, e * (int)sizeof(T), 0, 0));
      const uint4 y = *reinterpret_cast<const uint4*>(smem + o * OS + c8 * 16);
      uint4 vo = epi_row<T>(y, xin, p.accum, sin, p.scale);
      if constexpr (OUTACT) vo = lrelu_unit<T>(vo, p.out_slope);
      store16<TTS_ROW_STORE>(Y, e * (int)sizeof(T), vo);
    }
  }
}

template <typename T, int C, int K>
static hipError_t launch_pair_split(const MrfPairParams& p, hipStream_t s) {
  constexpr int BN = 16 * PSPLIT_NU, NSL = C / (16 * PSPLIT_WM);
  const int blocks = (p.T + BN - 1) / BN * p.B * NSL;
  const int a1 = (K - 1) / 2 * p.d;
  const size_t lds1 = (size_t)(BN + 2 * a1) * PairGeom<C>::RS;
  const size_t lds2 = std::max((size_t)(BN + K - 1) * PairGeom<C>::RS, (size_t)BN * (16 * PSPLIT_WM * 2 + 16));
  if (lds1 > 160 * 1024 || blocks <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL((mrf_pair_split_kernel<T, C, K, false, false>), dim3(blocks), dim3(64 * PSPLIT_WM), lds1, s, p);
  HIP_RETURN_IF_ERR(hipGetLastError());
  if (p.out_act)
    hipLaunchKernelGGL((mrf_pair_split_kernel<T, C, K, true, true>), dim3(blocks), dim3(64 * PSPLIT_WM), lds2, s, p);
  else
    hipLaunchKernelGGL((mrf_pair_split_kernel<T, C, K, true, false>), dim3(blocks), dim3(64 * PSPLIT_WM), lds2, s, p);
  return hipGetLastError();
}

#ifndef TTS_PAIR_SPLIT_MAXBLK
#define TTS_PAIR_SPLIT_MAXBLK 256  // full-height blocks below which C >= 128 pairs run channel-split (0: never)
#endif
// whether a launch runs the channel-split form: C = 128 / 256 (the weight-heavy stages), a scratch
// given, and a full-height grid under TTS_PAIR_SPLIT_MAXBLK blocks (TTS_PAIR_SPLIT=0/1 forces it
// off / on wherever possible: tests)
#ifndef TTS_PAIR_SPLIT_CMIN
#define TTS_PAIR_SPLIT_CMIN 256  // C = 128 measured slower split (C5 trace: k = 3 / 7 / 11 pairs 12 / 18 / 24 -> 17 / 22 / 27 us)
#endif
static bool pair_split(int C, const MrfPairParams& p) {
  if (C < 128 || C < TTS_PAIR_SPLIT_CMIN || !p.tbuf || p.post_wpk) return false;
  const int force = sw(SW_PAIR_SPLIT);
  if (force >= 0) return force != 0;
  const int bn = C == 128 ? PairGeom<128>::BN : PairGeom<256>::BN;
  return (long long)((p.T + bn - 1) / bn) * p.B < TTS_PAIR_SPLIT_MAXBLK;
}

// output activation compiled for the stage-final pairs of HiFi-GAN V1 (k = 11 at C = 64 .. 256)
template <int C, int K>
constexpr bool pair_outact_compiled() { return K == 11 && (C == 64 || C == 128 || C == 256); }

template <typename T, int C, int K, bool POST, int DIV>
static hipError_t launch_pair_g(const MrfPairParams& p, hipStream_t s) {
  using G = PairGeomS<C, DIV, K, POST>;
  const size_t lds = pair_lds_bytes<C, DIV, K, POST>(K, p.d, POST);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  dim3 grid(xcd_grid((p.T + G::BN - 1) / G::BN, p.B));
  if constexpr (!POST && pair_outact_compiled<C, K>()) {
    if (p.out_act) {
      hipLaunchKernelGGL((mrf_pair_kernel<T, C, K, POST, DIV, true>), grid, dim3(64 * G::WM * G::WN), lds, s, p);
      return hipGetLastError();
    }
  }
  if (p.out_act) return hipErrorInvalidValue;
  hipLaunchKernelGGL((mrf_pair_kernel<T, C, K, POST, DIV>), grid, dim3(64 * G::WM * G::WN), lds, s, p);
  return hipGetLastError();
}

template <typename T, int C, int K, bool POST = false>
static hipError_t launch_pair_t(const MrfPairParams& p, hipStream_t s) {
  if constexpr (!POST && C >= 128)
    if (pair_split(C, p)) return launch_pair_split<T, C, K>(p, s);
  if constexpr (!POST)
    if (pair_div(C, p, POST) != 1) return launch_pair_g<T, C, K, POST, TTS_PAIR_SHORT_DIV>(p, s);
  return launch_pair_g<T, C, K, POST, 1>(p, s);
}

template <typename T, int C, bool POST = false>
static hipError_t launch_pair_k(const MrfPairParams& p, hipStream_t s) {
  switch (p.k) {
    case 3: return launch_pair_t<T, C, 3, POST>(p, s);
    case 5: return launch_pair_t<T, C, 5, POST>(p, s);
    case 7: return launch_pair_t<T, C, 7, POST>(p, s);
    case 11: return launch_pair_t<T, C, 11, POST>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// kernel sizes with a compiled pair kernel: HiFi-GAN V1/V2 (3, 7, 11) and V3 (3, 5, 7);
// other sizes run the per-conv path
#ifndef TTS_PAIR_C256_KMAX
#define TTS_PAIR_C256_KMAX 11  // C = 256 resblocks with a larger k run as single convs (A/B knob)
#endif
bool mrf_pair_supported(int dtype, int C, int k) {
  return (dtype == DT_F16 || dtype == DT_BF16) &&
         (C == 32 || C == 64 || C == 128 || (TTS_PAIR_C256 && C == 256 && k <= TTS_PAIR_C256_KMAX)) &&
         (k == 3 || k == 5 || k == 7 || k == 11);
}

bool mrf_pair_outact_supported(int dtype, int C, int k) {
  return mrf_pair_supported(dtype, C, k) && k == 11 && (C == 64 || C == 128 || C == 256);
}

bool mrf_pair_post_supported(int dtype, int C, int post_k) {
  return (dtype == DT_F16 || dtype == DT_BF16) && C == 32 && post_k >= 1 && post_k % 2 == 1 &&
         post_k <= 2 * PAIR_PO + 1;
}

hipError_t mrf_pair_launch(int dtype, int C, const MrfPairParams& p, hipStream_t s) {
  if (!mrf_pair_supported(dtype, C, p.k) || p.d < 1) return hipErrorInvalidValue;
  if (!(p.slope >= 0.f && p.slope <= 1.f)) return hipErrorInvalidValue;  // lrelu_unit / epi_conv1
  if (p.out_act && (!(p.out_slope >= 0.f && p.out_slope <= 1.f) || p.post_wpk)) return hipErrorInvalidValue;
  if (p.post_wpk && !(p.post_slope >= 0.f && p.post_slope <= 1.f)) return hipErrorInvalidValue;
  if (p.post_wpk) {
    if (!mrf_pair_post_supported(dtype, C, p.post_k) || !p.wav) return hipErrorInvalidValue;
    return dtype == DT_F16 ? launch_pair_k<half_t, 32, true>(p, s) : launch_pair_k<bf16_t, 32, true>(p, s);
  }
  if (dtype == DT_F16) {
    if (C == 32) return launch_pair_k<half_t, 32>(p, s);
    if (C == 64) return launch_pair_k<half_t, 64>(p, s);
    if (C == 256) return launch_pair_k<half_t, 256>(p, s);
    return launch_pair_k<half_t, 128>(p, s);
  }
  if (C == 32) return launch_pair_k<bf16_t, 32>(p, s);
  if (C == 64) return launch_pair_k<bf16_t, 64>(p, s);
  if (C == 256) return launch_pair_k<bf16_t, 256>(p, s);
  return launch_pair_k<bf16_t, 128>(p, s);
}

#if TTS_PAIR_STAMP
extern "C" int tts_debug_pair_target(int C, int k, int d) {  // also clears the records
  const int t[3] = {C, k, d};
  void* buf = nullptr;
  if (hipDeviceSynchronize() != hipSuccess || hipGetSymbolAddress(&buf, HIP_SYMBOL(g_pair_stamp)) != hipSuccess ||
      hipMemset(buf, 0, sizeof(unsigned long long) << 21) != hipSuccess)
    return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pair_stamp_target), t, sizeof(t)) == hipSuccess ? 0 : -1;
}
extern "C" int tts_debug_pair_stamps(unsigned long long* host, long long words) {
  const long long n = words < (1LL << 21) ? words : (1LL << 21);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace tts
