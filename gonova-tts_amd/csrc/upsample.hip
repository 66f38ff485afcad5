// Streaming ConvTranspose1d for the small upsamplers (HiFi-GAN V1 stages 2 and 3: 128 -> 64
// and 64 -> 32 channels, k = 4, stride 2), whose weights fit in LDS.
//
//   y[s*u + r - p][co] = b[co] + sum_{t<2} sum_ci lrelu(x[u + t - 1][ci]) * W[ci][co][r + (1-t)*s]
//
// (k = 2s, two taps per output phase; oracle: vocoder.conv_transpose1d).  As a GEMM per input
// row u: [lrelu x[u-1], lrelu x[u]] (K = 2*Cin) x W' (K x M, M = s*Co) -> the M outputs of rows
// s*u - p .. s*u - p + s - 1, which are contiguous in [rows][Co] memory.
//
// conv_xres ran these at 12-22 % MFMA and 3.6-4.2 TB/s: a block stages an X tile with few
// loads in flight, computes briefly, and stores through two LDS halves.  Here the packed
// weights (<= 64 KB) are loaded into LDS once per persistent block, and each wave streams
// 16*NU-row items on its own with no block barriers:
//   * B fragments come straight from HBM: for v_mfma_f32_16x16x32, lane l of a fragment needs
//     16 contiguous bytes (row u0 + (l & 15), channels 8*(l >> 4) ..), one buffer load per
//     fragment; rows outside [0, len) fall outside the descriptor's range and read as 0;
//   * the next item's fragments are in flight while the current one computes and stores;
//   * A fragments (weights) are read from LDS, each feeding NU row tiles;
//   * the output tile goes through a per-wave LDS slice into 16-byte row pieces: the item's
//     outputs are one contiguous span (rows s*u0 - p ...), written with non-temporal stores.
#include <algorithm>
#include <atomic>

#include "common.h"
#include "kernels.h"
#include "mrf_tile.h"

#define HIP_RETURN_IF(expr)               \
  do {                                    \
    const hipError_t e_ = (expr);         \
    if (e_ != hipSuccess) return e_;      \
  } while (0)

namespace tts {

template <typename T, int CIN, int M>
struct UpGeom;
// NU: 16-row tiles per item; NW: waves per block (LDS: weights + NW staging slices)
#ifndef TTS_UP2_NU
#define TTS_UP2_NU 1
#endif
#ifndef TTS_UP2_NW
#define TTS_UP2_NW 12
#endif
#ifndef TTS_UP2_NW_BF16
#define TTS_UP2_NW_BF16 8  // bf16: its LeakyReLU goes through f32, and at 12 waves (168 VGPRs) it spilled
#endif
#ifndef TTS_UP3_NU
#define TTS_UP3_NU 2
#endif
#ifndef TTS_UP3_NW
#define TTS_UP3_NW 8
#endif
template <typename T>
struct UpGeom<T, 128, 128> {  // stage 2: 64 KB weights
  static constexpr int NU = TTS_UP2_NU, NW = __is_same(T, bf16_t) ? TTS_UP2_NW_BF16 : TTS_UP2_NW;
};
template <typename T>
struct UpGeom<T, 64, 64> { static constexpr int NU = TTS_UP3_NU, NW = TTS_UP3_NW; };  // stage 3: 16 KB weights

template <typename T, int CIN, int M>
constexpr size_t up_lds_bytes() {
  using G = UpGeom<T, CIN, M>;
  return (size_t)M * 2 * CIN * 2 + (size_t)M * 4 + (size_t)G::NW * 16 * G::NU * (M * 2 + 16);
}

// LeakyReLU of 8 x 16-bit, branch-free (0 <= slope <= 1, checked at launch): f16 packed
// max(x, slope*x); bf16 through f32
template <typename T>
__device__ inline uint4 up_lrelu(uint4 u, float slope) {
  if constexpr (__is_same(T, half_t)) {
    half8 v = *reinterpret_cast<half8*>(&u);
    v = __builtin_elementwise_max(v, v * (_Float16)slope);
    return *reinterpret_cast<uint4*>(&v);
  } else {
    return lrelu_unit<T>(u, slope);
  }
}

template <typename T, int CIN, int M>
__global__ __launch_bounds__((64 * UpGeom<T, CIN, M>::NW)) void upsample_stream_kernel(UpsampleParams p) {
  using G = UpGeom<T, CIN, M>;
  using MF = Mfma16<T>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int NU = G::NU, NW = G::NW, K = 2 * CIN, KS = K / 32, MT = M / 16;
  constexpr int ROWS = 16 * NU;        // input rows per item
  constexpr int YS = M * 2 + 16;       // staging row stride (bytes): one input row's M outputs
  constexpr int PPR = M / 8;           // 16-byte output pieces per input row
  constexpr int NP = ROWS * PPR / 64;  // pieces per lane
  static_assert(ROWS * PPR % 64 == 0, "row pass");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  char* Ws = smem;                                              // [MT][KS][64][16 B]
  float* Bs = reinterpret_cast<float*>(smem + M * K * 2);       // bias [M]
  char* Ys = smem + M * K * 2 + M * 4 + wave * ROWS * YS;       // this wave's output slice

  {
    const uint4* src = reinterpret_cast<const uint4*>(p.wpk);
    for (int i = tid; i < M * K / 8; i += 64 * NW) reinterpret_cast<uint4*>(Ws)[i] = src[i];
    for (int i = tid; i < M; i += 64 * NW) Bs[i] = p.bias[i];
  }
  __syncthreads();
  // per-utterance lengths through the scalar cache (s_load): a vector load here would be
  // counted by vmcnt behind the prefetched fragments, and waiting for it would drain them
  const __attribute__((address_space(4))) int* lens =
      (const __attribute__((address_space(4))) int*)(p.len);
  const __attribute__((address_space(4))) int* up_lens =
      (const __attribute__((address_space(4))) int*)(p.up_len);

  const int ipu = (p.T + 1 + ROWS - 1) / ROWS;  // items per utterance: input rows u = 0 .. T
  const int items = ipu * p.B;
  const int step = gridDim.x * NW;
  const float slope = p.slope;

  // fragments of item `it` (rows outside [0, len) read as zero through the descriptor)
  auto load = [&](int it, Frag (&bf)[NU][KS]) __attribute__((always_inline)) {
    // wave-uniform by construction; readfirstlane lets the compiler see it (a descriptor
    // it cannot prove uniform becomes a waterfall loop with a vmcnt(0) drain per load)
    const int b = __builtin_amdgcn_readfirstlane(it / ipu);
    const int u0 = __builtin_amdgcn_readfirstlane((it - b * ipu) * ROWS);
    const int len = min(lens[b], p.T);
    const T* xb = reinterpret_cast<const T*>(p.x) + (long long)b * p.sxb;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(xb), 0, len * CIN * (int)sizeof(T), 0x00020000);
#pragma unroll
    for (int j = 0; j < NU; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k0 = ks * 32 + 8 * lq;       // tap k0 / CIN: row u - 1 (tap 0) or u (tap 1)
        const int u = u0 + 16 * j + l15 + k0 / CIN - 1;
        const int off = (u * CIN + k0 % CIN) * (int)sizeof(T);  // u = -1: wraps past the range -> 0
        bf[j][ks] = __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    __builtin_amdgcn_sched_barrier(0);  // issue here: the scheduler would sink them into compute()
  };
  auto compute = [&](int it, Frag (&bf)[NU][KS]) __attribute__((always_inline)) {
    const int b = __builtin_amdgcn_readfirstlane(it / ipu);
    const int u0 = __builtin_amdgcn_readfirstlane((it - b * ipu) * ROWS);
    const int len = min(lens[b], p.T);
    f32x4 acc[NU][MT];
#pragma unroll
    for (int j = 0; j < NU; ++j)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[j][mt] = f32x4{};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      Frag g[NU];
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        const uint4 v = up_lrelu<T>(__builtin_bit_cast(uint4, bf[j][ks]), slope);
        g[j] = __builtin_bit_cast(Frag, v);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const Frag a = *reinterpret_cast<const Frag*>(Ws + ((mt * KS + ks) * 64 + lane) * 16);
#pragma unroll
        for (int j = 0; j < NU; ++j) acc[j][mt] = MF::mma(a, g[j], acc[j][mt]);
      }
    }
    // D fragment: output m = mt*16 + 4*lq + e of input row u0 + 16j + l15
#pragma unroll
    for (int j = 0; j < NU; ++j)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
      {  // fp32 bias add, one rounding (as conv_xres)
        const f32x4 v = acc[j][mt] + *reinterpret_cast<const f32x4*>(Bs + mt * 16 + 4 * lq);
        *reinterpret_cast<uint2*>(Ys + (16 * j + l15) * YS + (mt * 16 + 4 * lq) * 2) = pack4<T>(v);
      }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slice is written before it is read back
    __builtin_amdgcn_wave_barrier();
    const int tlen = min(up_lens[b], p.T * p.s);
    T* yb = reinterpret_cast<T*>(p.y) + (long long)b * p.syb;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int q = lane + 64 * i;
      const int ul = q / PPR, c = q % PPR;
      const int u = u0 + ul, m0 = c * 8;
      const int orow = p.s * u + m0 / p.co - p.pad;
      const uint4 v = *reinterpret_cast<const uint4*>(Ys + ul * YS + c * 16);
      if (u <= len && orow >= 0 && orow < tlen)
        store16<2>(yb, (int)(((long long)orow * p.co + m0 % p.co) * (long long)sizeof(T)), v);
    }
    __builtin_amdgcn_wave_barrier();
  };

  int it = blockIdx.x * NW + wave;
  if (it >= items) return;
  Frag b0[NU][KS], b1[NU][KS];
  load(it, b0);
  // two items per trip: each computes while the next one's fragments load.  The loads are
  // unconditional (past the end: the last item again, discarded) so the waitcnt pass keeps
  // them in flight instead of draining at a branch.
  for (;;) {
    const int n1 = it + step;
    load(min(n1, items - 1), b1);
    compute(it, b0);
    if (n1 >= items) break;
    const int n2 = n1 + step;
    load(min(n2, items - 1), b0);
    compute(n1, b1);
    if (n2 >= items) break;
    it = n2;
  }
}

bool upsample_stream_supported(int dtype, int Cin, int M, int taps) {
  return (dtype == DT_F16 || dtype == DT_BF16) && taps == 2 &&
         ((Cin == 128 && M == 128) || (Cin == 64 && M == 64));
}

template <typename T, int CIN, int M>
static hipError_t launch_up_t(const UpsampleParams& p, hipStream_t s) {
  using G = UpGeom<T, CIN, M>;
  constexpr size_t lds = up_lds_bytes<T, CIN, M>();
  static_assert(lds <= 160 * 1024, "LDS");
  // blocks that fit at once, per device (engines on several GPUs launch from their own threads)
  static std::atomic<int> grid_of[64];
  int dev = 0;
  HIP_RETURN_IF(hipGetDevice(&dev));
  int grid = dev >= 0 && dev < 64 ? grid_of[dev].load(std::memory_order_relaxed) : 0;
  if (!grid) {
    int per_cu = 0, cus = 0;
    HIP_RETURN_IF(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, upsample_stream_kernel<T, CIN, M>,
                                                               64 * G::NW, lds));
    HIP_RETURN_IF(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    grid = std::max(1, per_cu) * cus;
    if (dev >= 0 && dev < 64) grid_of[dev].store(grid, std::memory_order_relaxed);
  }
  const int ipu = (p.T + 1 + 16 * G::NU - 1) / (16 * G::NU);
  const int blocks = std::min(grid, (ipu * p.B + G::NW - 1) / G::NW);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL((upsample_stream_kernel<T, CIN, M>), dim3(blocks), dim3(64 * G::NW), lds, s, p);
  return hipGetLastError();
}

hipError_t upsample_stream_launch(int dtype, int Cin, int M, const UpsampleParams& p, hipStream_t s) {
  if (!upsample_stream_supported(dtype, Cin, M, 2) || p.s < 1 || M % p.s || p.co != M / p.s || p.co % 8 ||
      !(p.slope >= 0.f && p.slope <= 1.f))
    return hipErrorInvalidValue;
  const bool f16 = dtype == DT_F16;
  if (Cin == 128) return f16 ? launch_up_t<half_t, 128, 128>(p, s) : launch_up_t<bf16_t, 128, 128>(p, s);
  return f16 ? launch_up_t<half_t, 64, 64>(p, s) : launch_up_t<bf16_t, 64, 64>(p, s);
}

}  // namespace tts
