// Software-pipelined ResBlock pair for C = 32 (HiFi-GAN stage 3), the same arithmetic as
// mrf_pair_kernel (mrf_pair.hip), bit for bit:
//
//   t  = lrelu( conv_{k,d}( lrelu(h) ) + b1 )
//   h' = conv_{k,1}( t ) + b2 + h            out = h'  or  S = (S + h') * scale
//
// Why a second kernel.  At C = 32 a 16-row output tile of one conv is k x 2 MFMAs (K = 32 per
// tap) against a per-tile epilogue of ~12-16 VALU instructions and two LDS writes, so the pair
// kernel's phase structure -- every conv's MFMAs for all of a wave's tiles (k-step outer, the
// weights streamed from L2 and reused across the tiles), then a barrier, then every tile's
// epilogue -- leaves the matrix pipe idle through each epilogue unless another block's MFMAs
// happen to fill it: the C = 32 pairs ran at 44-50 % MFMA busy at their clock, the chains at
// 31-47 % (profiles/r02e_clock_mfma_c2.txt).  Here a conv's weights (k x 2 fragments, <= 88
// VGPRs at k = 11) are held in registers for the whole conv, so a wave runs its tiles one
// after another (tile outer) and the epilogue of tile u sits in the same basic block as the
// MFMAs of tile u + 1: the wave's own VALU issues while its MFMAs execute.
//
// LDS: G = lrelu(h) (staged once, rows n0 - a1 - a2 ...) and T = conv1 output in separate
// tiles (the pair kernel writes T over G after a barrier; here conv1 tiles finish one by one
// while other waves still read G).  conv2's epilogue goes straight to HBM: each lane holds 4
// channels of one row, a 16-row tile of C = 32 is one contiguous KiB, written by the wave's two
// 8-byte stores per lane (buffer stores: rows past the utterance fall outside the descriptor
// and are dropped); the residual h and the MRF sum S come the same way (L2-hot: the block just
// staged the rows).
#include "common.h"
#include "kernels.h"
#include "mrf_tile.h"

#include <type_traits>

namespace tts {

// Output rows per block.  conv1 covers BN + 2 a2 rows = BN / 16 + 1 tiles: with BN = 16 (4q + 3)
// those are 4 (q + 1) tiles, an even share for each of the 4 waves, and conv2's BN / 16 tiles
// leave one wave a repeated tile (a multiple of 64 would leave three repeats in conv1).
#ifndef TTS_SP_BN3
#define TTS_SP_BN3 240
#endif
#ifndef TTS_SP_BN7
#define TTS_SP_BN7 240
#endif
#ifndef TTS_SP_BN11
#define TTS_SP_BN11 240
#endif
#ifndef TTS_SP_SCHED
#define TTS_SP_SCHED 1  // 0: leave the MFMA / epilogue interleave to the compiler's scheduler
#endif
#ifndef TTS_SP_OCC
#define TTS_SP_OCC 3
#endif

template <int K>
struct SpGeom {
  static constexpr int BN = K <= 3 ? TTS_SP_BN3 : K <= 7 ? TTS_SP_BN7 : TTS_SP_BN11;
};

// LDS rows of one launch: T = 16 * NT1 rows, then G = 16 * NT1 + 2 * a1 rows rounded up to
// the staging step (64 rows at C = 32: every staging store lands inside the allocation)
template <int K, int BN>
struct SpPlan {
  static constexpr int C = 32, RS = 64, A2 = (K - 1) / 2;
  static constexpr int RT = BN + 2 * A2, NT1 = (RT + 15) / 16, NT2 = BN / 16;
  static constexpr int RSTEP = 64;  // staging rows per round (256 threads x 16 B / 64 B rows)
  __host__ __device__ static int grows(int d) { return (16 * NT1 + 2 * A2 * d + RSTEP - 1) / RSTEP * RSTEP; }
  __host__ __device__ static size_t lds_bytes(int d) { return (size_t)(16 * NT1 + grows(d)) * RS; }
};

template <typename T, int K, int BN>
__global__ __launch_bounds__(256, TTS_SP_OCC) void mrf_pair_sp_kernel(MrfPairParams p) {
  using P = SpPlan<K, BN>;
  using G = PairGeom<32>;
  using MF = Mfma16<T>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int C = 32, RS = 64, MT = 2, WN = 4, S = K, A2 = P::A2;
  constexpr int NT1 = P::NT1, NT2 = P::NT2;
  constexpr int NU1 = (NT1 + WN - 1) / WN, NU2 = (NT2 + WN - 1) / WN;
  static_assert(BN % 16 == 0 && 2 * A2 <= 16, "16-row tiles; conv1 overrun within one tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto swz = [](int r) { return ((r * G::SW_MUL) >> G::SW_S) & G::SW_M; };

  int b, tile0;
  if (!xcd_tile((p.T + BN - 1) / BN, p.B, b, tile0)) return;
  const int n0 = tile0 * BN;
  const int len = min(p.len[b], p.T);
  if (n0 >= len) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wn = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  const int d = p.d, a1 = A2 * d;
  const float slope = p.slope;
  const int ch0 = 4 * lq;  // + 16 * mt: this lane's 4 output channels
  char* Ts = smem;
  char* Gs = smem + 16 * NT1 * RS;
  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;
  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.T * C;
  const int rbytes = len * C * (int)sizeof(T);
  // rows outside [0, len) are outside these descriptors: loads return 0, stores are dropped
  const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(X), 0, rbytes, 0x00020000);
  const auto sr = __builtin_amdgcn_make_buffer_rsrc(Y, 0, p.accum ? rbytes : 0, 0x00020000);

  // conv1 weights: all k steps x 2 M tiles in registers ([C/16][k][1][64][8]: m tile mt, step s
  // at (mt * S + s) KiB), in flight during the staging
  Frag W[S][MT];
  auto load_w = [&](const void* w) __attribute__((always_inline)) {
    const char* wp = reinterpret_cast<const char*>(w) + lane * 16;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) W[s][mt] = *reinterpret_cast<const Frag*>(wp + (mt * S + s) * 1024);
  };
  load_w(p.w1);
  f32x4 bias1[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) bias1[mt] = *reinterpret_cast<const f32x4*>(p.b1 + ch0 + 16 * mt);

  // ---- stage G = lrelu(h): G row g <-> utterance row n0 - a1 - A2 + g (zero outside) ----
  {
    const int cc = tid & 3, r0 = tid >> 2;  // 4 pieces of 16 B per row, 64 rows per round
    const int gs = n0 - a1 - A2;
    const int nround = P::grows(d) / P::RSTEP;
    for (int rb = 0; rb < nround; rb += PAIR_SU) {
      u32x4 v[PAIR_SU];
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        // a round past the tile gets an offset outside the descriptor: issued, fetches nothing
        const int off = rb + i < nround ? ((gs + r0 + (rb + i) * 64) * C + cc * 8) * (int)sizeof(T) : 0x7ffffff0;
        v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      }
      __builtin_amdgcn_sched_barrier(0);  // every load of the round in flight before the first use
#pragma unroll
      for (int i = 0; i < PAIR_SU; ++i) {
        const int r = r0 + (rb + i) * 64;
        const uint4 g = lrelu_unit<T>(__builtin_bit_cast(uint4, v[i]), slope);
        if (rb + i < nround) *reinterpret_cast<uint4*>(Gs + r * RS + ((cc ^ swz(r)) << 4)) = g;
      }
    }
  }
  __syncthreads();

  // B-fragment addresses: tile j = wn + 4u of a conv reads rows 16 j + l15 + s * trow; the
  // swizzle depends on the row mod 8 only, so lane address ad[s] covers u = 0 and tile u is the
  // immediate offset u * 64 rows (no per-tile address arithmetic)
  static_assert(NT1 % WN == 0, "BN = 16 (4q + 3): conv1 tiles dealt evenly (no clamped repeats)");
  const char* ad[S];
  auto set_ad = [&](const char* base, int trow) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int r = l15 + s * trow;
      ad[s] = base + (16 * wn + r) * RS + ((lq ^ swz(r)) << 4);
    }
  };
  // One conv over the wave's NU tiles, software-pipelined: the B fragments run PF steps ahead
  // through a register ring over the flattened (tile, step) sequence, and the epilogue of tile
  // u - 1 (epi(acc, u - 1)) is scheduled between the MFMAs of tile u -- V VALU instructions
  // after each MFMA (sched_group_barrier), so the wave's own vector work issues while its
  // matrix instructions execute.  pre(u) issues tile u's global loads (conv2: residual rows)
  // one tile ahead of its epilogue.
  constexpr int PF = S < 4 ? S : S >= 11 ? 3 : 4;  // k = 11: 88 weight VGPRs leave room for 3
  auto conv_pipe = [&](auto NUC, auto VC, const f32x4 (&binit)[MT], auto&& epi, auto&& pre, auto&& before_last)
                       __attribute__((always_inline)) {
    constexpr int NU = decltype(NUC)::value, V = decltype(VC)::value;
    Frag ring[PF];
#pragma unroll
    for (int g = 0; g < PF; ++g) ring[g] = *reinterpret_cast<const Frag*>(ad[g % S] + (g / S) * 64 * RS);
    f32x4 acc[2][MT];
    pre(0);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      if (u + 1 < NU) pre(u + 1);
      f32x4 (&a)[MT] = acc[u & 1];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = acc_init(binit[mt]);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int g = u * S + s;
        const Frag bf = ring[g % PF];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[mt] = MF::mma(W[s][mt], bf, a[mt]);
        const int gn = g + PF;
        if (gn < NU * S) ring[g % PF] = *reinterpret_cast<const Frag*>(ad[gn % S] + (gn / S) * 64 * RS);
      }
      if (u > 0) epi(acc[(u - 1) & 1], u - 1);
      if (TTS_SP_SCHED && u > 0) {  // interleave: MFMA, V x VALU, ... ; a DS read after every MT MFMAs
#pragma unroll
        for (int s = 0; s < S; ++s) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    before_last();
    epi(acc[(NU - 1) & 1], NU - 1);
  };
  // VALU instructions of an epilogue (two M tiles) spread over a tile's 2 S MFMAs
  constexpr int VEPI = 22, VPM = (VEPI + 2 * S - 1) / (2 * S);

  // ---- conv1 over T rows [0, 16 NT1): T row t <-> utterance row n0 - A2 + t ----
  {
    set_ad(Gs, d);
    // this lane's T-row bytes for its 4 channels of M tile mt, tile u = 0 (+ u * 64 rows)
    int eo[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int cb = (ch0 + 16 * mt) * 2, tr = 16 * wn + l15;
      eo[mt] = tr * RS + (((cb >> 4) ^ swz(tr)) << 4) + (cb & 15);
    }
    const int gr0 = n0 - A2 + 16 * wn + l15;  // utterance row of this lane's row in tile u = 0
    auto epi1 = [&](const f32x4 (&acc)[MT], int u) __attribute__((always_inline)) {
      const bool valid = (unsigned)(gr0 + 64 * u) < (unsigned)len;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        uint2 pk = epi_conv1<T>(acc[mt], bias1[mt], slope);
        if (!valid) pk = uint2{0u, 0u};
        *reinterpret_cast<uint2*>(Ts + eo[mt] + u * 64 * RS) = pk;
      }
    };
    // conv2's weights in flight during the last epilogue and the barrier
    conv_pipe(std::integral_constant<int, NT1 / WN>{}, std::integral_constant<int, VPM>{}, bias1, epi1, [](int) {},
              [&] { load_w(p.w2); });
  }
  f32x4 bias2[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) bias2[mt] = *reinterpret_cast<const f32x4*>(p.b2 + ch0 + 16 * mt);
  __syncthreads();

  // ---- conv2 over output rows [0, 64 NU2): row o <-> utterance row n0 + o, reads T rows
  // o .. o + 2 A2.  Tiles past BN (a wave's last tile when BN / 16 is not a multiple of 4) read
  // T rows up to 64 NU2 + 2 A2 <= the allocation and are dropped by the store descriptor, which
  // ends at row min(len, n0 + BN). ----
  {
    set_ad(Ts, 1);
    const auto yr = __builtin_amdgcn_make_buffer_rsrc(Y, 0, min(len, n0 + BN) * C * (int)sizeof(T), 0x00020000);
    int ro[MT];  // byte offset of this lane's 4 channels in its row of tile u = 0
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ro[mt] = ((n0 + 16 * wn + l15) * C + ch0 + 16 * mt) * (int)sizeof(T);
    // residual rows of tile u in slot u % 3: tile u + 1's loads are issued while tile u - 1's
    // epilogue still reads its slot
    uint2 hv[3][MT], sv[3][MT];
    auto load_res = [&](int u) __attribute__((always_inline)) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        // the tile offset goes into the VGPR offset: the descriptor's range check does not
        // include soffset
        const int off = ro[mt] + u * 64 * RS;
        hv[u % 3][mt] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0));
        sv[u % 3][mt] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(sr, off, 0, 0));
      }
    };
    const float scale = p.scale;
    auto epi2 = [&](const f32x4 (&acc)[MT], int u) __attribute__((always_inline)) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint2 y = epi_conv2<T>(acc[mt], bias2[mt]);
        const uint2 o = epi_row4_nb<T>(y, hv[u % 3][mt], sv[u % 3][mt], scale);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), yr, ro[mt] + u * 64 * RS, 0, TTS_ROW_STORE);
      }
    };
    constexpr int NU = (NT2 + WN - 1) / WN;
    conv_pipe(std::integral_constant<int, NU>{}, std::integral_constant<int, VPM>{}, bias2, epi2, load_res, [] {});
  }
}

template <typename T, int K>
static hipError_t launch_sp_t(const MrfPairParams& p, hipStream_t s) {
  constexpr int BN = SpGeom<K>::BN;
  const size_t lds = SpPlan<K, BN>::lds_bytes(p.d);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  dim3 grid(xcd_grid((p.T + BN - 1) / BN, p.B));
  hipLaunchKernelGGL((mrf_pair_sp_kernel<T, K, BN>), grid, dim3(256), lds, s, p);
  return hipGetLastError();
}

bool mrf_pair_sp_supported(int dtype, int C, int k) {
  return (dtype == DT_F16 || dtype == DT_BF16) && C == 32 && (k == 3 || k == 5 || k == 7 || k == 11);
}

hipError_t mrf_pair_sp_launch(int dtype, int C, const MrfPairParams& p, hipStream_t s) {
  if (p.out_act) return hipErrorInvalidValue;  // (no output activation in the pipelined form)
  if (!mrf_pair_sp_supported(dtype, C, p.k) || p.d < 1 || p.post_wpk) return hipErrorInvalidValue;
  if (!(p.slope >= 0.f && p.slope <= 1.f)) return hipErrorInvalidValue;  // lrelu_unit / epi_conv1
  const bool f16 = dtype == DT_F16;
  switch (p.k) {
    case 3: return f16 ? launch_sp_t<half_t, 3>(p, s) : launch_sp_t<bf16_t, 3>(p, s);
    case 5: return f16 ? launch_sp_t<half_t, 5>(p, s) : launch_sp_t<bf16_t, 5>(p, s);
    case 7: return f16 ? launch_sp_t<half_t, 7>(p, s) : launch_sp_t<bf16_t, 7>(p, s);
    default: return f16 ? launch_sp_t<half_t, 11>(p, s) : launch_sp_t<bf16_t, 11>(p, s);
  }
}

}  // namespace tts
