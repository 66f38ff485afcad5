// Warp-specialised, persistent ResBlock pair for the k = 3 pairs at C = 128 / 256 (HiFi-GAN V1
// stages 0-1, resblock 0): the same arithmetic as mrf_pair_kernel (mrf_pair.hip) -- the same
// pair_conv k-step order, conv1 / conv2 epilogues and row pass, so the output is bit-identical --
// with the memory traffic moved off the MFMA waves.
//
// Why (tools/pair_stamps.py, profiles/r04b_pair_stamps.txt): a k = 3 pair block at C = 128 spent
// 24 % of its time staging its input tile from HBM (7.8 k cycles of load latency under load),
// 10 % in the row pass and ~17 % in the epilogue barriers, against 49 % in its two convs; three
// blocks per CU did not cover each other's memory phases (MFMA pipe 55 % busy).  A prefetch of
// the next tile inside the same waves cannot hide that latency: vmcnt retires in issue order, so
// the weight ring's waits would wait for any older staging load.
//
// Block = 4 x TTS_PAIR_WS_WN compute waves (16 * MT channels x a share of the rows each) + NL
// loader waves, two LDS buffers, persistent over a contiguous range of (utterance, row tile) items
// per XCD:
//   loader:  DMA (buffer_load ... lds) of tile k+1's input rows h into the other buffer, with the
//            G tile's chunk swizzle on the source address (rows outside the utterance read 0
//            through the descriptor's range), then LeakyReLU in place -> G;
//            row pass of tile k-1 from its output tile in LDS: + h (+ S) (x scale), stores
//            through a descriptor whose range ends at the utterance (rows past it are dropped);
//   compute: conv1 on G -> T (same buffer) -> conv2 -> output tile (same buffer).
// Four block barriers per tile order the two roles:
//   A(k)  G_k ready (loader) and OUT_{k-1} written (compute)
//   B(k)  compute done reading G_k (it writes T over it); loader done reading OUT_{k-1}
//   C(k)  T written;                loader's DMA of G_{k+1} issued into the other buffer
//   D(k)  conv2 done reading T;     G_{k+1} landed and activated
// The loader waves have their own vmcnt, so the MFMA waves' weight-ring waits never wait on a
// staging load or a store.  Default: 8 compute + 4 loader waves, one block per CU (3 waves per
// SIMD; a block's waves must spread evenly over the 4 SIMDs, which 6-wave blocks do not).
// Measured slower than mrf_pair_kernel (profiles/r04i_ab_pair_ws.txt: with one block per CU
// nothing overlaps the MFMA waves' own epilogues), so TTS_PAIR_WS is off by default.
#include "common.h"
#include "kernels.h"
#include "mrf_tile.h"
#include "switches.h"

#include <algorithm>

#ifndef TTS_PAIR_MTO_MIN
#define TTS_PAIR_MTO_MIN 64  // (mrf_pair.hip's: M-tile-outer MFMA order from this channel count up)
#endif
#ifndef TTS_PAIR_WS_NL
#define TTS_PAIR_WS_NL 4  // loader waves per block
#endif
#ifndef TTS_PAIR_WS_WN
#define TTS_PAIR_WS_WN 2  // compute waves along the rows (x 4 along the channels)
#endif
#ifndef TTS_PAIR_WS_DEFAULT
#define TTS_PAIR_WS_DEFAULT 0  // off: slower than mrf_pair_kernel so far (profiles/r04e_ab_pair_ws.txt)
#endif
#ifndef TTS_PWS_BN_128
#define TTS_PWS_BN_128 (144 * TTS_PAIR_WS_WN - 2)  // output rows per tile at C = 128: conv1's rows in whole 16-row tiles
#endif
#ifndef TTS_PWS_BN_256
#define TTS_PWS_BN_256 (64 * TTS_PAIR_WS_WN - 2)   // at C = 256
#endif

#ifndef TTS_PWS_STAMP
#define TTS_PWS_STAMP 0  // diagnostic builds only: barrier arrival times per role (tools/pws_stamps.py)
#endif

namespace tts {

#if TTS_PWS_STAMP
// The launches whose (C, d) match g_pws_target (the last one of the workload wins): per block 256
// words -- [0] tiles, [1] entry time, then per tile k < 31 eight s_memtime values: the compute
// wave 0's arrival at barriers A(k), B(k), C(k), D(k) and the first loader wave's.  Never in the product.
__device__ int g_pws_target[2];
__device__ unsigned long long g_pws_stamp[1 << 20];
#define TTS_WSTAMP(role_, j_)                                                                       \
  if (stamp_on && lane == 0 && k < 31) stamp_rec[2 + 8 * k + 4 * (role_) + (j_)] = __builtin_amdgcn_s_memtime()
#else
#define TTS_WSTAMP(role_, j_) (void)0
#endif

// the pair kernel's per-wave tiles (channels x 16-row tiles, weight ring), TTS_PAIR_WS_WN wave rows
template <int C>
struct PwsGeom : PairGeom<C> {
  // 4 waves along the channels (16 * MT channels each), whatever wave grid mrf_pair_kernel uses
  static constexpr int WM = 4, WN = TTS_PAIR_WS_WN, MT = C / 64;
};

template <int C>
constexpr int pws_bn() { return C == 128 ? TTS_PWS_BN_128 : TTS_PWS_BN_256; }

// bytes of one LDS buffer: the G tile at dilation d (incl. conv1's overrun rows), the T tile and
// the output staging tile, rounded up to whole 1 KiB DMA pieces
template <int C, int K>
static int pws_buf_bytes(int d) {
  using G = PwsGeom<C>;
  constexpr int BN = pws_bn<C>(), A2 = (K - 1) / 2;
  constexpr int NT1 = (BN + 2 * A2 + 15) / 16, NT2 = (BN + 15) / 16;
  const int g = (16 * NT1 + 2 * A2 * d) * G::RS;
  const int o = 16 * NT2 * (C * 2 + 16);
  const int m = g > o ? g : o;
  return (m + 1023) / 1024 * 1024;
}

// one 16-byte-per-lane buffer load straight into LDS (a __device__ function: inside the kernel's
// lambdas, which are host-device, the host pass rejects the LDS address space and the kernel's
// host stub silently vanishes)
__device__ inline void pws_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

template <typename T, int C, int K, int NL, bool OUTACT>
__global__ __launch_bounds__(64 * (4 * TTS_PAIR_WS_WN + NL), 3) void mrf_pair_ws_kernel(MrfPairParams p, int buf_bytes) {
  using G = PwsGeom<C>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int BN = pws_bn<C>(), WM = G::WM, WN = G::WN, RS = G::RS, D = G::D, MT = G::MT;
  constexpr int NCW = WM * WN;  // compute waves
  static_assert((NCW + NL) % 4 == 0, "whole waves per SIMD: a block's waves spread evenly over the 4 SIMDs");
  constexpr int KS = C / 32, S = K * KS;
  constexpr int A2 = (K - 1) / 2;
  constexpr int BO = BN, RT = BO + 2 * A2;
  constexpr int NT1 = (RT + 15) / 16, NU1 = (NT1 + WN - 1) / WN;
  constexpr int NT2 = (BO + 15) / 16, NU2 = (NT2 + WN - 1) / WN;
  static_assert(NT2 <= NT1, "conv2's overrun rows read inside the G / T region");
  constexpr int VPR = C / 8;                  // 16-byte pieces per row
  constexpr int YS16 = C * 2 + 16;            // output staging row stride
  constexpr int RPI = 1024 / RS;              // G rows per 1 KiB DMA piece
  constexpr int NLT = 64 * NL;                // loader threads
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto swz = [](int r) { return ((r * G::SW_MUL) >> G::SW_S) & G::SW_M; };

  // ---- the block's items: XCD x = blockIdx % 8 owns items [x * per, (x + 1) * per) of the
  // (utterance, row tile) sequence; its blocks take them round robin.  Both roles walk the same
  // sequence and skip the same empty tiles (rows past the utterance), so their barriers match.
  const int nx = (p.T + BN - 1) / BN;
  const int items = nx * p.B;
  const int per = (items + 7) / 8;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int nbx = (gridDim.x - xcd + 7) >> 3;  // this XCD's blocks
  const int it0 = xcd * per + jb, it_end = min(items, (xcd + 1) * per);
  auto item_ok = [&](int it) {  // a tile with rows inside its utterance (block-uniform)
    const int b = it / nx;
    return (it - b * nx) * BN < min(p.len[b], p.T);
  };
  auto next_item = [&](int it) {
    for (it += nbx; it < it_end && !item_ok(it); it += nbx) {}
    return it;
  };
  int first = it0;
  if (first < it_end && !item_ok(first)) first = next_item(first);
  if (first >= it_end) return;  // no work (both roles alike)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int d = p.d;
#if TTS_PWS_STAMP
  const bool stamp_on = g_pws_target[0] == C && g_pws_target[1] == p.d && (wave == 0 || wave == NCW) &&
                        blockIdx.x < (1u << 12);
  unsigned long long* stamp_rec = g_pws_stamp + blockIdx.x * 256;
  if (stamp_on && wave == 0 && lane == 0) stamp_rec[1] = __builtin_amdgcn_s_memtime();
#endif
  const int a1 = A2 * d;
  const int RG = 16 * NT1 + 2 * a1;  // G rows (conv1 overrun included)
  const size_t utt = (size_t)p.T * C;  // elements per utterance
  const float slope = p.slope;

  if (wave >= NCW) {
    // =============================== loader waves ===============================
    const int lt = tid - 64 * NCW;  // 0 .. NLT-1
    const int lw = wave - NCW;
    const int NQ = (RG * RS + 1023) / 1024;  // DMA pieces of the G tile
    // DMA of item `it`'s input rows into buffer `buf`: G row r <-> utterance row n0 - a1 - A2 + r
    // (item, utterance and length made wave-uniform: a descriptor built from a value the compiler
    // cannot prove uniform becomes a waterfall loop around every buffer instruction)
    auto dma = [&](int it, char* buf) __attribute__((always_inline)) {
      it = __builtin_amdgcn_readfirstlane(it);
      const int b = it / nx, n0 = (it - b * nx) * BN, len = __builtin_amdgcn_readfirstlane(min(p.len[b], p.T));
      const T* Xb = reinterpret_cast<const T*>(p.x) + (size_t)b * utt;
      const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Xb), 0, len * C * (int)sizeof(T), 0x00020000);
      const int gs = n0 - a1 - A2;
      const int lr = lane / (RS / 16), pos = lane % (RS / 16);
      for (int q = lw; q < NQ; q += NL) {
        const int r = RPI * q + lr;
        const int c = pos ^ swz(r);
        // rows before 0 give a negative offset: outside the descriptor (unsigned), read as 0
        const int voff = ((gs + r) * C + 8 * c) * (int)sizeof(T);
        pws_dma16(xr, buf + q * 1024, voff);
      }
    };
    // LeakyReLU in place over the landed G tile (element-wise: the swizzle does not matter)
    // (four pieces per lane in flight: one LDS round trip per four, not per piece)
    auto activate = [&](char* buf) __attribute__((always_inline)) {
      const int n16 = NQ * 64;
      for (int i0 = lt; i0 < n16; i0 += 4 * NLT) {
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const uint4*>(buf + 16 * min(i0 + j * NLT, n16 - 1));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (i0 + j * NLT < n16) *reinterpret_cast<uint4*>(buf + 16 * (i0 + j * NLT)) = lrelu_unit<T>(v[j], slope);
      }
    };
    // row pass of item `it` from its output tile in `buf` (mrf_pair_kernel's, piece for piece;
    // never accumulating: the launcher takes only pairs that write the MRF sum fresh): every
    // input-row load of the lane's P pieces goes out at once (one round trip; the rows are
    // L2-hot, staged as this tile's G two tiles ago), then LDS read + epilogue + store
    constexpr int NP = BO * VPR, P = (NP + NLT - 1) / NLT;
    auto row_pass = [&](int it, const char* buf) __attribute__((always_inline)) {
      it = __builtin_amdgcn_readfirstlane(it);
      const int b = it / nx, n0 = (it - b * nx) * BN, len = __builtin_amdgcn_readfirstlane(min(p.len[b], p.T));
      const T* Xb = reinterpret_cast<const T*>(p.x) + (size_t)b * utt;
      T* Yb = reinterpret_cast<T*>(p.y) + (size_t)b * utt;
      const int nb = len * C * (int)sizeof(T);
      const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Xb), 0, nb, 0x00020000);
      const auto yr = __builtin_amdgcn_make_buffer_rsrc(Yb, 0, nb, 0x00020000);  // rows >= len: dropped
      const int base = n0 * C * (int)sizeof(T);
      uint4 h[P];
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int idx = min(lt + j * NLT, NP - 1);
        h[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, base + idx * 16, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int idx = lt + j * NLT;
        if (idx < NP) {
          const int o = idx / VPR, c8 = idx % VPR;
          const uint4 y = *reinterpret_cast<const uint4*>(buf + o * YS16 + c8 * 16);
          uint4 v = epi_row<T>(y, h[j], false, uint4{0u, 0u, 0u, 0u}, p.scale);
          if constexpr (OUTACT) v = lrelu_unit<T>(v, p.out_slope);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yr, base + idx * 16, 0, TTS_ROW_STORE);
        }
      }
    };
    dma(first, smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    activate(smem);
    int k = 0;
    TTS_WSTAMP(1, 0);
    __syncthreads();  // A(0)
    int prev = -1;
    for (int it = first; it < it_end; it = next_item(it), ++k) {
      char* cur_other = smem + ((k + 1) & 1) * buf_bytes;  // the buffer of tiles k - 1 and k + 1
      if (prev >= 0) row_pass(prev, cur_other);
      TTS_WSTAMP(1, 1);
      __syncthreads();  // B(k)
      const int nxt = next_item(it);
      if (nxt < it_end) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the row pass's LDS reads are done)
        dma(nxt, cur_other);
      }
      TTS_WSTAMP(1, 2);
      __syncthreads();  // C(k)
      if (nxt < it_end) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        activate(cur_other);
      }
      TTS_WSTAMP(1, 3);
      __syncthreads();  // D(k)
      {
        ++k;
        TTS_WSTAMP(1, 0);
        --k;
      }
      __syncthreads();  // A(k + 1)
      prev = it;
    }
    row_pass(prev, smem + ((k + 1) & 1) * buf_bytes);  // the last tile's output (buffer of tile k - 1)
    return;
  }

  // =============================== compute waves ===============================
  const int wm = WM == 1 ? 0 : wave % WM, wn = WN == 1 ? 0 : wave / WM;
  const int l15 = lane & 15, lq = lane >> 4;
  const int ch0 = 16 * MT * wm + 4 * lq;  // + 16*mt: this lane's 4 output channels
  const char* w1 = reinterpret_cast<const char*>(p.w1) + (long long)(MT * wm) * S * 1024 + lane * 16;
  const char* w2 = reinterpret_cast<const char*>(p.w2) + (long long)(MT * wm) * S * 1024 + lane * 16;
  // Every tile re-derives the weight-step addresses from w1 / w2 made opaque here: hoisted out of
  // the tile loop, the 64-bit address of every ring load stayed live across it and spilled.
  auto opaque = [](const char* q) {
    asm volatile("" : "+v"(q));
    return q;
  };
  Frag ring[D][MT];
  auto prologue = [&](const char* w) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (i < S)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) ring[i][mt] = *reinterpret_cast<const Frag*>(w + ((long long)mt * S + i) * 1024);
  };
  auto last_off = [&](int nt, int nu) { return 16 * (min(wn + WN * (nu - 1), nt - 1) - wn) * RS; };
  int eo[MT];  // this lane's T bytes in the wave's tile 0 (tile u: + u * 16 WN rows)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) eo[mt] = pair_lds4<C>(16 * wn + l15, ch0 + 16 * mt);
  prologue(w1);
  int k = 0;
  TTS_WSTAMP(0, 0);
  __syncthreads();  // A(0)
  for (int it = first; it < it_end; it = next_item(it), ++k) {
    char* buf = smem + (k & 1) * buf_bytes;
    const int b = it / nx, n0 = (it - b * nx) * BN, len = min(p.len[b], p.T);
    const char* w1t = opaque(w1);
    const char* w2t = opaque(w2);
    // ---- conv1 over T rows [0, 16*NT1): T row t <-> utterance row n0 - A2 + t ----
    // (biases reloaded per tile, L1-hot: registers are the compute waves' limit)
    f32x4 bias1[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) bias1[mt] = *reinterpret_cast<const f32x4*>(p.b1 + ch0 + 16 * mt);
    f32x4 acc1[NU1][MT];
#pragma unroll
    for (int u = 0; u < NU1; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc1[u][mt] = acc_init(bias1[mt]);
    pair_conv<T, C, S, NU1, D, MT, (C >= TTS_PAIR_MTO_MIN), 16 * WN * RS>(acc1, ring, w1t, buf + (16 * wn + l15) * RS,
                                                                          d * RS, d, l15, lq, last_off(NT1, NU1));
    __builtin_amdgcn_sched_barrier(0);
    // conv2's bias first, then its first weight steps (in flight during the conv1 epilogue)
    f32x4 bias2[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) bias2[mt] = *reinterpret_cast<const f32x4*>(p.b2 + ch0 + 16 * mt);
    prologue(w2t);
    __builtin_amdgcn_sched_barrier(0);
    TTS_WSTAMP(0, 1);
    __syncthreads();  // B(k): T overwrites G
    {
      const int gr0 = n0 - A2 + 16 * wn + l15;  // utterance row of the lane's row in tile 0
#pragma unroll
      for (int u = 0; u < NU1; ++u)
        if (NT1 % WN == 0 || wn + WN * u < NT1) {
          const bool valid = (unsigned)(gr0 + 16 * WN * u) < (unsigned)len;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            uint2 pk = epi_conv1<T>(acc1[u][mt], bias1[mt], slope);
            if (!valid) pk = uint2{0u, 0u};
            *reinterpret_cast<uint2*>(buf + eo[mt] + u * 16 * WN * RS) = pk;
          }
        }
    }
    TTS_WSTAMP(0, 2);
    __syncthreads();  // C(k)
    // ---- conv2 over the BN output rows: output row o reads T rows o .. o + 2*a2 ----
    f32x4 acc2[NU2][MT];
#pragma unroll
    for (int u = 0; u < NU2; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc2[u][mt] = acc_init(bias2[mt]);
    pair_conv<T, C, S, NU2, D, MT, (C >= TTS_PAIR_MTO_MIN), 16 * WN * RS>(acc2, ring, w2t, buf + (16 * wn + l15) * RS, RS, 1,
                                                                          l15, lq, last_off(NT2, NU2));
    __builtin_amdgcn_sched_barrier(0);
    TTS_WSTAMP(0, 3);
    __syncthreads();  // D(k): T no longer read
    {
      char* ob = buf + (16 * wn + l15) * YS16 + ch0 * 2;
#pragma unroll
      for (int u = 0; u < NU2; ++u)
        if (NT2 % WN == 0 || wn + WN * u < NT2) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            *reinterpret_cast<uint2*>(ob + u * 16 * WN * YS16 + 32 * mt) = epi_conv2<T>(acc2[u][mt], bias2[mt]);
        }
    }
    prologue(opaque(w1));  // the next tile's conv1 weights, in flight across the barrier
    {
      ++k;
      TTS_WSTAMP(0, 0);
      --k;
    }
    __syncthreads();  // A(k + 1): the output tile is written; the loader's next G is ready
  }
#if TTS_PWS_STAMP
  if (stamp_on && wave == 0 && lane == 0) stamp_rec[0] = (unsigned long long)k;
#endif
}
#undef TTS_WSTAMP

template <int C>
static bool pws_shape(int dtype, const MrfPairParams& p) {
  return (dtype == DT_F16 || dtype == DT_BF16) && p.k == 3 && p.d >= 1 && p.d <= 5 && !p.post_wpk && !p.accum &&
         2 * pws_buf_bytes<C, 3>(p.d) <= 160 * 1024 && p.slope >= 0.f && p.slope <= 1.f;
}

bool mrf_pair_ws_supported(int dtype, int C, const MrfPairParams& p) {
  if (sw(SW_PAIR_WS) == 0 || (sw(SW_PAIR_WS) < 0 && !TTS_PAIR_WS_DEFAULT)) return false;
  if (C == 128) return pws_shape<128>(dtype, p);
  if (C == 256) return pws_shape<256>(dtype, p);
  return false;
}

template <typename T, int C>
static hipError_t launch_ws(const MrfPairParams& p, hipStream_t s) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  const int nx = (p.T + pws_bn<C>() - 1) / pws_bn<C>();
  const long long items = (long long)nx * p.B;
  const int bb = pws_buf_bytes<C, 3>(p.d);
  const size_t lds = 2 * (size_t)bb;
  constexpr int NL = TTS_PAIR_WS_NL, NW = 4 * TTS_PAIR_WS_WN + NL;
  // blocks per CU: by LDS and by wave slots (3 waves per SIMD at the kernel's register budget);
  // a multiple of 8 (every XCD the same number), at most one block per item
  const int bpc = std::max(1, std::min((int)(163840 / lds), 12 / NW));
  long long nb = std::min<long long>((long long)bpc * ncu, items);
  nb = std::max<long long>(8, nb / 8 * 8);

  if (p.out_act) {
    if (!(p.out_slope >= 0.f && p.out_slope <= 1.f)) return hipErrorInvalidValue;
    hipLaunchKernelGGL((mrf_pair_ws_kernel<T, C, 3, NL, true>), dim3((unsigned)nb), dim3(64 * (4 * TTS_PAIR_WS_WN + NL)), lds, s, p, bb);
  } else {
    hipLaunchKernelGGL((mrf_pair_ws_kernel<T, C, 3, NL, false>), dim3((unsigned)nb), dim3(64 * (4 * TTS_PAIR_WS_WN + NL)), lds, s, p, bb);
  }
  return hipGetLastError();
}

hipError_t mrf_pair_ws_launch(int dtype, int C, const MrfPairParams& p, hipStream_t s) {
  if (!mrf_pair_ws_supported(dtype, C, p)) return hipErrorInvalidValue;
  if (dtype == DT_F16) return C == 128 ? launch_ws<half_t, 128>(p, s) : launch_ws<half_t, 256>(p, s);
  return C == 128 ? launch_ws<bf16_t, 128>(p, s) : launch_ws<bf16_t, 256>(p, s);
}

#if TTS_PWS_STAMP
extern "C" int tts_debug_pws_target(int C, int d) {  // also clears the records
  const int t[2] = {C, d};
  void* buf = nullptr;
  if (hipDeviceSynchronize() != hipSuccess || hipGetSymbolAddress(&buf, HIP_SYMBOL(g_pws_stamp)) != hipSuccess ||
      hipMemset(buf, 0, sizeof(unsigned long long) << 20) != hipSuccess)
    return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pws_target), t, sizeof(t)) == hipSuccess ? 0 : -1;
}
extern "C" int tts_debug_pws_stamps(unsigned long long* host, long long words) {
  const long long n = words < (1LL << 20) ? words : (1LL << 20);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pws_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace tts
