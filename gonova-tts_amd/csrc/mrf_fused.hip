// Fused multi-receptive-field (MRF) stack of a HiFi-GAN stage, one launch per stage.
//
//   for each resblock j (k_j in {3,7,11}):                        (oracle: vocoder.resblock)
//     h = x
//     for each pair p (dilation d in {1,3,5}):
//       t = lrelu( conv_{k,d}( lrelu(h) ) + b1 )     -> LDS T
//       h = conv_{k,1}( t ) + b2 + h                  -> LDS H (in place) / S registers
//   S = (h_0 + h_1 + h_2) / 3                          -> HBM, once
//
// The unfused path moves every intermediate through HBM: 18 convs each read and write
// [rows][C] (+ residual), ~2.9 KB/row at C=32.  Here a block owns BN output rows, loads
// the x tile (with the resblock's receptive-field halo) once per resblock from HBM/L2, keeps
// h and t in LDS, accumulates the three resblock outputs in fp32 registers and writes S
// once: ~0.26 KB/row.  Every conv is an implicit GEMM on v_mfma_f32_32x32x16_{f16,bf16}:
// M = C output channels, N = 32-row time tiles, K = taps x C.
//
// Each conv phase computes only the rows its successor needs (the halo shrinks by the
// conv's half-width every phase), rounded up to 32-row tiles; rows outside the utterance
// are forced to 0 after every conv, which reproduces the per-utterance zero padding of
// the unfused convs exactly.
//
// LDS (one block per CU): H, T = [RP rows][C] in the compute dtype, 16-byte chunks
// XOR-swizzled by row (chunk ^ (row / (256/rowbytes)) & (chunks-1)) so ds_read_b128 of any
// 16 consecutive rows at one chunk hits 16 distinct 4-bank slots; weights stream per tap
// group through a double-buffered LDS slab, prefetched through registers one group ahead.
// 8 waves; 32-row tiles are dealt to waves round robin; the final phase's tiles are fixed
// per wave so the S accumulators stay in registers across the three resblocks.
#include "common.h"
#include "kernels.h"

namespace tts {

template <int C>
struct MrfGeom {
  static constexpr int RB = C * 2;              // LDS row bytes (16-bit dtype)
  static constexpr int CPR = RB / 16;           // 16-byte chunks per row
  static constexpr int SWZ_DIV = 256 / RB;      // rows sharing one 256-byte bank row
  static constexpr int G = C == 32 ? 11 : 2;    // taps per weight group
  static constexpr int WG_BYTES = G * C * RB;   // weight slab bytes per group
};

template <int C>
__device__ inline int lds_off(int row, int chunk) {
  using Gm = MrfGeom<C>;
  return row * Gm::RB + 16 * (chunk ^ ((row / Gm::SWZ_DIV) & (Gm::CPR - 1)));
}

template <typename T>
__device__ inline typename Mfma<T>::frag lrelu_frag(typename Mfma<T>::frag v, float slope) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float f = (float)v[i];
    v[i] = (T)(f >= 0.f ? f : f * slope);
  }
  return v;
}

template <typename T, int C, int BN>
__global__ __launch_bounds__(512, 2) void mrf_fused_kernel(MrfParams p) {
  using MF = Mfma<T>;
  typedef typename MF::frag Frag;
  using Gm = MrfGeom<C>;
  constexpr int NW = 8;
  constexpr int NTHR = 512;
  constexpr int MT = C / 32;                      // 32-row M tiles per unit
  constexpr int KS = C / 16;                      // MFMA k-steps per tap
  constexpr int MAXU = (BN + 2 * 60 + 31) / 32 / NW + 1;  // tiles per wave per phase (upper bound)
  constexpr int SU = BN / 32 / NW;                // final-phase tiles per wave
  constexpr int WPF = (Gm::WG_BYTES + 16 * NTHR - 1) / (16 * NTHR);  // weight prefetch vectors
  static_assert(BN % (32 * NW) == 0, "BN must be a multiple of 256");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MrfTable* __restrict__ tb = p.tab;
  char* Hs = smem;
  char* Ts = smem + p.rp * Gm::RB;
  char* Ws = smem + 2 * p.rp * Gm::RB;

  const int b = blockIdx.y;
  const int n0 = blockIdx.x * BN;
  const int len = min(p.len[b], p.T);
  if (n0 >= len) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int l31 = lane & 31;
  const int hh = lane >> 5;
  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;

  auto load_x = [&](int halo) {
    const int rows = BN + 2 * halo;
    for (int v = tid; v < rows * Gm::CPR; v += NTHR) {
      const int r = v / Gm::CPR, c = v - r * Gm::CPR;
      const int g = n0 - halo + r;
      uint4 u = *reinterpret_cast<const uint4*>(X + (long long)min(max(g, 0), len - 1) * C + c * 8);
      if (g < 0 || g >= len) u = uint4{0u, 0u, 0u, 0u};
      *reinterpret_cast<uint4*>(Hs + lds_off<C>(r, c)) = u;
    }
  };
  // weight group s: [ntaps][C][C] contiguous in HBM -> registers (WPF <= 3 named vectors)
  static_assert(WPF <= 3, "weight prefetch sized for <= 3 vectors per thread");
  uint4 wp0 = {}, wp1 = {}, wp2 = {};
#define TTS_LOAD_W(S_)                                                                    \
  do {                                                                                    \
    const char* src_ = reinterpret_cast<const char*>(tb->step_w[S_]);                     \
    const int nb_ = tb->step[S_].z * C * Gm::RB;                                          \
    wp0 = *reinterpret_cast<const uint4*>(src_ + min(tid * 16, nb_ - 16));               \
    if (WPF > 1) wp1 = *reinterpret_cast<const uint4*>(src_ + min((tid + NTHR) * 16, nb_ - 16));     \
    if (WPF > 2) wp2 = *reinterpret_cast<const uint4*>(src_ + min((tid + 2 * NTHR) * 16, nb_ - 16)); \
  } while (0)
#define TTS_STORE_W1(V_, W_, NB_, BUF_)                                                  \
  if ((V_) * 16 < (NB_)) {                                                                \
    const int row_ = (V_) / Gm::CPR, c_ = (V_) - row_ * Gm::CPR;                          \
    *reinterpret_cast<uint4*>((BUF_) + lds_off<C>(row_, c_)) = (W_);                      \
  }
#define TTS_STORE_W(S_, BUF_)                                                             \
  do {                                                                                    \
    const int nb_ = tb->step[S_].z * C * Gm::RB;                                          \
    TTS_STORE_W1(tid, wp0, nb_, BUF_);                                                    \
    if (WPF > 1) { TTS_STORE_W1(tid + NTHR, wp1, nb_, BUF_); }                            \
    if (WPF > 2) { TTS_STORE_W1(tid + 2 * NTHR, wp2, nb_, BUF_); }                        \
  } while (0)

  f32x16 acc[MAXU][MT];
  f32x16 sacc[SU][MT];
#pragma unroll
  for (int u = 0; u < MAXU; ++u)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[u][m] = f32x16{};
#pragma unroll
  for (int u = 0; u < SU; ++u)
#pragma unroll
    for (int m = 0; m < MT; ++m) sacc[u][m] = f32x16{};

  load_x(tb->halo[0]);
  TTS_LOAD_W(0);
  TTS_STORE_W(0, Ws);
  __syncthreads();

  for (int s = 0; s < tb->nsteps; ++s) {
    const int4 st = tb->step[s];
    const int j = st.x & 15, pr = (st.x >> 4) & 15, cv = (st.x >> 8) & 1, last = (st.x >> 12) & 1;
    const int tap0 = st.y, ntap = st.z;
    const int k = tb->k[j];
    const int hk = (k - 1) / 2;
    const int halo = tb->halo[j];
    const int R0 = BN + 2 * halo;
    // input range of this pair and the conv's output range
    int lo = 0;
    for (int q = 0; q < pr; ++q) lo += hk * tb->dil[j][q] + hk;
    const int a = cv == 0 ? hk * tb->dil[j][pr] : hk;     // this conv's half-width
    const int d = cv == 0 ? tb->dil[j][pr] : 1;
    const int olo = lo + (cv == 0 ? a : hk * tb->dil[j][pr] + hk);
    const int ohi = R0 - olo;
    const int nt = (ohi - olo + 31) / 32;
    const bool final_phase = cv == 1 && pr == tb->npair - 1;
    const char* in = cv == 0 ? Hs : Ts;
    const char* wbuf = Ws + (s & 1) * Gm::WG_BYTES;
    if (s + 1 < tb->nsteps) TTS_LOAD_W(s + 1);

    // ---- MFMA: my tiles x this tap group ----
    // Per tap: all B fragments of this wave's tiles are read first (rows clamped in-bounds,
    // no branch around any LDS read), the next tap's A fragments are prefetched, then the
    // MFMA batch runs; tiles past nt are skipped with a wave-uniform branch.
    const int nu = nt > wave ? (nt - wave + NW - 1) / NW : 0;
    const int rbase = olo + wave * 32 + l31 - a;
    Frag af[MT][KS];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        af[m][ks] = *reinterpret_cast<const Frag*>(wbuf + lds_off<C>(m * 32 + l31, 2 * ks + hh));
    for (int tl = 0; tl < ntap; ++tl) {
      const int tap = tap0 + tl;
      Frag bf[MAXU][KS];
#pragma unroll
      for (int u = 0; u < MAXU; ++u) {
        const int row = min(rbase + u * NW * 32 + tap * d, p.rp - 1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bf[u][ks] = *reinterpret_cast<const Frag*>(in + lds_off<C>(row, 2 * ks + hh));
      }
      Frag an[MT][KS];
      const int tn = tl + 1 < ntap ? tl + 1 : tl;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          an[m][ks] = *reinterpret_cast<const Frag*>(wbuf + lds_off<C>(tn * C + m * 32 + l31, 2 * ks + hh));
      if (cv == 0) {
#pragma unroll
        for (int u = 0; u < MAXU; ++u)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) bf[u][ks] = lrelu_frag<T>(bf[u][ks], p.slope);
      }
#pragma unroll
      for (int u = 0; u < MAXU; ++u) {
        if (u < nu) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[u][m] = MF::mma(af[m][ks], bf[u][ks], acc[u][m]);
        }
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) af[m][ks] = an[m][ks];
    }

    // ---- epilogue of the conv (after its last tap group) ----
    if (last) {
      const float* bias = tb->step_b[s];
#pragma unroll
      for (int u = 0; u < MAXU; ++u) {
        const int t = wave + u * NW;
        if (t < nt) {
          const int row = olo + t * 32 + l31;
          const int grow = n0 - halo + row;
          const bool valid = grow >= 0 && grow < len;
#pragma unroll
          for (int m = 0; m < MT; ++m) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int ch = m * 32 + 8 * g + 4 * hh;
              const int off = lds_off<C>(row, ch >> 3) + (ch & 7) * 2;
              const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + ch);
              f32x4 v = {acc[u][m][4 * g + 0], acc[u][m][4 * g + 1], acc[u][m][4 * g + 2], acc[u][m][4 * g + 3]};
              v += bb;
              if (cv == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = leaky(v[i], p.slope);
                if (!valid) v = f32x4{};
                Vec4<T>::store(reinterpret_cast<T*>(Ts + off), v);
              } else {
                v += Vec4<T>::load(reinterpret_cast<const T*>(Hs + off));
                if (final_phase) {
                  // t < BN/32 here: tile t belongs to this wave as slot u (t = wave + u*NW)
#pragma unroll
                  for (int su = 0; su < SU; ++su)
                    if (su == u) {
#pragma unroll
                      for (int i = 0; i < 4; ++i) sacc[su][m][4 * g + i] += v[i];
                    }
                } else {
                  if (!valid) v = f32x4{};
                  Vec4<T>::store(reinterpret_cast<T*>(Hs + off), v);
                }
              }
            }
            acc[u][m] = f32x16{};
          }
        }
      }
    }
    if (s + 1 < tb->nsteps) TTS_STORE_W(s + 1, Ws + ((s + 1) & 1) * Gm::WG_BYTES);
    if (final_phase && last && j + 1 < tb->nblk) {
      __syncthreads();   // every wave is done with H / T of resblock j
      load_x(tb->halo[j + 1]);
    }
    __syncthreads();
  }

  // ---- S = mean over resblocks -> HBM ----
  T* S = reinterpret_cast<T*>(p.s) + (long long)b * p.T * C;
#pragma unroll
  for (int su = 0; su < SU; ++su) {
    const int t = wave + su * NW;
    const int grow = n0 + t * 32 + l31;
    if (grow >= len) continue;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch = m * 32 + 8 * g + 4 * hh;
        f32x4 v = {sacc[su][m][4 * g + 0], sacc[su][m][4 * g + 1], sacc[su][m][4 * g + 2], sacc[su][m][4 * g + 3]};
        v *= p.out_scale;
        Vec4<T>::store(S + (long long)grow * C + ch, v);
      }
  }
}

template <typename T, int C, int BN>
static hipError_t launch_mrf_t(const MrfParams& p, hipStream_t s) {
  using Gm = MrfGeom<C>;
  const size_t lds = (size_t)2 * p.rp * Gm::RB + 2 * Gm::WG_BYTES;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  dim3 grid((p.T + BN - 1) / BN, p.B);
  hipLaunchKernelGGL((mrf_fused_kernel<T, C, BN>), grid, dim3(512), lds, s, p);
  return hipGetLastError();
}

int mrf_fused_taps_per_group(int C) { return C == 32 ? MrfGeom<32>::G : MrfGeom<64>::G; }

int mrf_fused_bn(int C) { return C == 32 ? 512 : 256; }

hipError_t mrf_fused_launch(int dtype, int C, const MrfParams& p, hipStream_t s) {
  if (dtype == DT_F16) {
    if (C == 32) return launch_mrf_t<half_t, 32, 512>(p, s);
    if (C == 64) return launch_mrf_t<half_t, 64, 256>(p, s);
  } else if (dtype == DT_BF16) {
    if (C == 32) return launch_mrf_t<bf16_t, 32, 512>(p, s);
    if (C == 64) return launch_mrf_t<bf16_t, 64, 256>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace tts
