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
// VALU budget (measured: the first version issued 38 VALU per MFMA and was VALU-bound):
//  * H holds g = lrelu(h), the conv1 operand, so conv1 B fragments go LDS -> MFMA with no
//    arithmetic; the residual h is recovered in the conv2 epilogue as g >= 0 ? g : g/slope
//    (LeakyReLU is invertible), once per output element instead of once per tap.
//  * H/T rows are padded by 16 bytes (80 B at C=32, 144 B at C=64: ds_read_b128 of 16
//    consecutive rows hits 16 distinct bank slots), so a tap is one address add.
//  * weight slabs are XOR-swizzled with a tap-invariant pattern (one add per tap as well).
//  * tiles are dealt round robin; reads and MFMAs of a wave's absent tiles are skipped by
//    wave-uniform branches.
//
// Each conv phase computes only the rows its successor needs (the halo shrinks by the
// conv's half-width every phase), rounded up to 32-row tiles; rows outside the utterance
// are forced to 0 after every conv, which reproduces the per-utterance zero padding of
// the unfused convs.
#include "common.h"
#include "kernels.h"

namespace tts {

template <int C>
struct MrfGeom {
  static constexpr int RB = C * 2;              // payload bytes per row (16-bit dtype)
  static constexpr int RBP = RB + 16;           // padded activation row stride in LDS
  static constexpr int CPR = RB / 16;           // 16-byte chunks per row
  static constexpr int SWZ_DIV = 256 / RB;      // weight rows sharing one 256-byte bank row
  static constexpr int G = C == 32 ? 11 : 2;    // taps per weight group
  static constexpr int WG_BYTES = G * C * RB;   // weight slab bytes per group
};

// weight slab layout: row = tap*C + m, 16-byte chunk XOR-swizzled by (row / SWZ_DIV) & (CPR-1);
// the swizzle term is unchanged by a +C row step (C / SWZ_DIV is a multiple of CPR).
template <int C>
__device__ inline int w_off(int row, int chunk) {
  using Gm = MrfGeom<C>;
  return row * Gm::RB + 16 * (chunk ^ ((row / Gm::SWZ_DIV) & (Gm::CPR - 1)));
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
// 16-byte load through the global address space: a pointer read from the step table is
// generic, and flat loads are counted on lgkmcnt too, which would make every LDS wait of
// the MFMA loop also wait for the in-flight weight prefetch.
__device__ inline uint4 gload16(const char* p) {
  const u32x4 v = *(gu32x4*)(p);
  uint4 r;
  r.x = v[0]; r.y = v[1]; r.z = v[2]; r.w = v[3];
  return r;
}

template <typename T>
__device__ inline uint4 lrelu16(uint4 u, float slope) { return lrelu_chunk<T>(u, slope); }

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
  static_assert(WPF <= 3, "weight prefetch sized for <= 3 vectors per thread");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const MrfTable* __restrict__ tb = p.tab;
  char* Hs = smem;
  char* Ts = smem + p.rp * Gm::RBP;
  char* Ws = smem + 2 * p.rp * Gm::RBP;

  const int b = blockIdx.y;
  const int n0 = blockIdx.x * BN;
  const int len = min(p.len[b], p.T);
  if (n0 >= len) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar tile branches
  const int l31 = lane & 31;
  const int hh = lane >> 5;
  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.T * C;
  const float inv_slope = 1.0f / p.slope;

  // x tile of resblock j -> H as g0 = lrelu(x); rows outside the utterance are 0.
  // Loaded into registers first (xload) so the next resblock's tile is in flight during
  // the current resblock's last conv, then written to LDS (xstore).
  constexpr int XPF = ((BN + 2 * 60) * Gm::CPR + NTHR - 1) / NTHR;
  uint4 xr[XPF];
#define TTS_XLOAD(HALO_)                                                                  \
  do {                                                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < XPF; ++i_) {                                  \
      const int v_ = tid + i_ * NTHR;                                                     \
      const int r_ = v_ / Gm::CPR, c_ = v_ - r_ * Gm::CPR;                                \
      const int g_ = min(max(n0 - (HALO_) + r_, 0), len - 1);                             \
      xr[i_] = *reinterpret_cast<const uint4*>(X + (long long)g_ * C + c_ * 8);          \
    }                                                                                     \
  } while (0)
#define TTS_XSTORE(HALO_)                                                                 \
  do {                                                                                    \
    const int rows_ = BN + 2 * (HALO_);                                                   \
    _Pragma("unroll") for (int i_ = 0; i_ < XPF; ++i_) {                                  \
      const int v_ = tid + i_ * NTHR;                                                     \
      if (v_ < rows_ * Gm::CPR) {                                                         \
        const int r_ = v_ / Gm::CPR, c_ = v_ - r_ * Gm::CPR;                              \
        const int g_ = n0 - (HALO_) + r_;                                                 \
        const uint4 u_ = (g_ < 0 || g_ >= len) ? uint4{0u, 0u, 0u, 0u} : lrelu16<T>(xr[i_], p.slope); \
        *reinterpret_cast<uint4*>(Hs + r_ * Gm::RBP + c_ * 16) = u_;                       \
      }                                                                                   \
    }                                                                                     \
  } while (0)
  // all biases of the stage -> LDS once per block
  float* Bs = reinterpret_cast<float*>(smem + 2 * p.rp * Gm::RBP + 2 * Gm::WG_BYTES);
  for (int i = tid; i < tb->nconv * C; i += NTHR) Bs[i] = tb->bias[i];

  uint4 wp0 = {}, wp1 = {}, wp2 = {};
#define TTS_LOAD_W(S_)                                                                    \
  do {                                                                                    \
    const char* src_ = reinterpret_cast<const char*>(tb->step_w[S_]);                     \
    const int nb_ = tb->step[S_].z * C * Gm::RB;                                          \
    wp0 = gload16(src_ + min(tid * 16, nb_ - 16));                                       \
    if (WPF > 1) wp1 = gload16(src_ + min((tid + NTHR) * 16, nb_ - 16));                   \
    if (WPF > 2) wp2 = gload16(src_ + min((tid + 2 * NTHR) * 16, nb_ - 16));               \
  } while (0)
#define TTS_STORE_W1(V_, W_, NB_, BUF_)                                                  \
  if ((V_) * 16 < (NB_)) {                                                                \
    const int row_ = (V_) / Gm::CPR, c_ = (V_) - row_ * Gm::CPR;                          \
    *reinterpret_cast<uint4*>((BUF_) + w_off<C>(row_, c_)) = (W_);                        \
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

  // per-lane A-fragment byte offsets in a weight slab (tap 0); + tap * C * RB per tap
  int aoff[MT][KS];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) aoff[m][ks] = w_off<C>(m * 32 + l31, 2 * ks + hh);

  TTS_XLOAD(tb->halo[0]);
  TTS_XSTORE(tb->halo[0]);
  TTS_LOAD_W(0);
  TTS_STORE_W(0, Ws);
  __syncthreads();

  for (int s = 0; s < tb->nsteps; ++s) {
    const int4 st = tb->step[s];
    const int4 geo = tb->geo[s];
    const int j = st.x & 15, cv = (st.x >> 8) & 1, last = (st.x >> 12) & 1;
    const bool final_phase = (st.x >> 13) & 1;
    const int tap0 = st.y, ntap = st.z;
    const int olo = geo.x, a = geo.y, d = geo.z, nt = geo.w;
    const int halo = tb->halo[j];
    const int nu = nt > wave ? (nt - wave + NW - 1) / NW : 0;
    const char* in = cv == 0 ? Hs : Ts;
    const char* wbuf = Ws + (s & 1) * Gm::WG_BYTES;
    if (s + 1 < tb->nsteps) TTS_LOAD_W(s + 1);
    const bool next_blk = final_phase && last && j + 1 < tb->nblk;

    // ---- MFMA: my tiles x this tap group ----
    const int bbase = (olo + wave * 32 + l31 - a + tap0 * d) * Gm::RBP + 16 * hh;
    const int dstep = d * Gm::RBP;
    Frag af[MT][KS];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[m][ks] = *reinterpret_cast<const Frag*>(wbuf + aoff[m][ks]);
    for (int tl = 0; tl < ntap; ++tl) {
      // all LDS reads of this tap first (B of every present tile, A of the next tap) ...
      const char* bt = in + bbase + tl * dstep;
      Frag bf[MAXU][KS];
#pragma unroll
      for (int u = 0; u < MAXU; ++u)
        if (u < nu) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            bf[u][ks] = *reinterpret_cast<const Frag*>(bt + u * (NW * 32 * Gm::RBP) + 32 * ks);
        }
      Frag an[MT][KS];
      const char* wn = wbuf + (tl + 1 < ntap ? tl + 1 : tl) * C * Gm::RB;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) an[m][ks] = *reinterpret_cast<const Frag*>(wn + aoff[m][ks]);
      // ... then the MFMA batch
#pragma unroll
      for (int u = 0; u < MAXU; ++u)
        if (u < nu) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[u][m] = MF::mma(af[m][ks], bf[u][ks], acc[u][m]);
        }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) af[m][ks] = an[m][ks];
    }

    // next resblock's x tile in flight during this epilogue (fragment registers are dead here)

    // ---- epilogue of the conv (after its last tap group) ----
    if (last) {
      const float* bias = Bs + st.w * C;
#pragma unroll
      for (int u = 0; u < MAXU; ++u) {
        if (u < nu) {
          const int row = olo + (wave + u * NW) * 32 + l31;
          const int grow = n0 - halo + row;
          const bool valid = grow >= 0 && grow < len;
#pragma unroll
          for (int m = 0; m < MT; ++m) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int ch = m * 32 + 8 * g + 4 * hh;
              const int off = row * Gm::RBP + ch * 2;
              const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + ch);
              f32x4 v = {acc[u][m][4 * g + 0], acc[u][m][4 * g + 1], acc[u][m][4 * g + 2], acc[u][m][4 * g + 3]};
              v += bb;
              if (cv == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = leaky(v[i], p.slope);
                if (!valid) v = f32x4{};
                Vec4<T>::store(reinterpret_cast<T*>(Ts + off), v);
              } else {
                f32x4 gr = Vec4<T>::load(reinterpret_cast<const T*>(Hs + off));
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] += gr[i] >= 0.f ? gr[i] : gr[i] * inv_slope;  // + h (residual)
                if (final_phase) {
#pragma unroll
                  for (int su = 0; su < SU; ++su)
                    if (su == u) {
#pragma unroll
                      for (int i = 0; i < 4; ++i) sacc[su][m][4 * g + i] += v[i];
                    }
                } else {
#pragma unroll
                  for (int i = 0; i < 4; ++i) v[i] = leaky(v[i], p.slope);  // store g = lrelu(h)
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
    if (next_blk) {
      __syncthreads();   // every wave is done with H / T of resblock j
      TTS_XLOAD(tb->halo[j + 1]);
      TTS_XSTORE(tb->halo[j + 1]);
    }
    __syncthreads();
  }
#undef TTS_LOAD_W
#undef TTS_STORE_W1
#undef TTS_STORE_W

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
  const size_t lds = (size_t)2 * p.rp * Gm::RBP + 2 * Gm::WG_BYTES + (size_t)4 * 4 * 2 * 4 * C;  // + biases
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
