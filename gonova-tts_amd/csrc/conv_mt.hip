// Macro-tiled implicit-GEMM convolution for the acoustic model's dense layers (16-bit, gfx950).
//
//   Y[b][n][m] = epi( sum_{t, c} W[m][t][c] * X[b][n + t*dil - pad][c] )
//
// The decoder's FFN convs (k = 3, 384 -> 1536 -> 384), Q|K|V, attention-output and pointwise
// projections (k = 1) and the postnet convs (k = 5) -- the mel half of the reference's
// `model.generate` (services/tts/core/synthesizer.py:344-350; HF FastSpeech2ConformerModel,
// oracle/acoustic.py).  conv_xres_kernel (conv_gemm.hip) ran these as 128 x 128 tiles of four
// waves, each wave streaming its own A fragments from L2 through a register ring: ~30 % MFMA busy
// at batch 32.  Here a block is one workgroup per CU of 8 waves (two per SIMD) owning a BM x BN
// output tile (channels x time rows), and BOTH operands go through LDS:
//
//   * one k-tile = (tap t, 64-channel group c): the A tile W[m0 .. m0+BM)[t][64c .. +64) and the
//     B tile X[n0 + t*dil - pad .. + BN)[64c .. +64), 128-byte rows, copied global -> LDS by
//     buffer_load ... lds (16 bytes per lane, 1 KiB per wave instruction, no staging registers)
//     into a two-stage ring: tile i + 1 lands while tile i's MFMAs run;
//   * chunk j of LDS row r sits at slot j ^ ((r >> 1) & 7): the DMA's LDS image is lane-linear,
//     so the swizzle is applied to the source address, and the fragment reads (16 rows x 4
//     chunks per ds_read_b128) hit 16 distinct 16-byte slots per lane group -- conflict-free
//     (the bank model of MI355X_MICROARCH.md §LDS, same image as conv_xres's DMA form);
//   * the implicit-GEMM halo is only a row shift of the B tile's source (t*dil - pad rows): rows
//     outside [0, len[b]) fall outside the utterance's buffer descriptor and read 0;
//   * MFMA v_mfma_f32_16x16x32_{f16,bf16}; each wave owns MT x NT 16 x 16 accumulator tiles
//     (16*MT channels x 16*NT rows), every A fragment feeds NT MFMAs and every B fragment MT;
//   * epilogue: (acc + bias) * alpha -> activation -> T, staged in LDS, then a row pass of
//     16-byte pieces adds the residual, scales and stores; when the block owns every channel of
//     its rows (BM == M) the post-LayerNorm (HF:551-645, ln_rows.h) runs on the staged rows in the
//     same launch and only its output is written.
//
// One K order (k-tiles in (t, c) order, 32-deep MFMA steps) for every tile shape and batch
// size, so a row's result does not depend on the batch it runs in (tests/test_acoustic_gpu.py).
#include "common.h"
#include "kernels.h"
#include "ln_rows.h"
#include "switches.h"

#include <algorithm>
#include <atomic>

namespace tts {

// CUs of the calling thread's current device (cached per device; engines on several GPUs launch
// from their own threads at once)
static int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

template <typename T>
struct Mma16;
template <>
struct Mma16<half_t> {
  typedef half8 frag;
  __device__ static inline f32x4 mma(half8 a, half8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
};
template <>
struct Mma16<bf16_t> {
  typedef bf16x8 frag;
  __device__ static inline f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
};

__device__ inline void mt_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

#ifndef TTS_MT_LN_RB
#define TTS_MT_LN_RB 2  // rows per wave normalised together in the fused post-LN
#endif
#ifndef TTS_MT_PROBE
#define TTS_MT_PROBE 0  // timing-only diagnostic builds: 1 = no DMA after the prologue, 2 = no MFMA, 3 = no fragment reads
#endif
#ifndef TTS_MT_STORE
#define TTS_MT_STORE 2  // output store cache policy (store16, common.h)
#endif

// geometry of one configuration
template <int WM_, int WN_, int MT_, int NT_>
struct MtGeom {
  static constexpr int WM = WM_, WN = WN_, MT = MT_, NT = NT_;
  static constexpr int NW = WM * WN, NTHR = 64 * NW;
  static constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  static constexpr int PA = BM / 8, PB = BN / 8;          // 1 KiB pieces of the A / B tile
  static constexpr int JA = PA / NW;                      // A pieces per wave
  static constexpr int JB = (PB + NW - 1) / NW;           // B pieces per wave (the last may be padding)
  static constexpr bool PAD = JB * NW > PB;               // padding pieces land in a junk slot
  static constexpr int STAGE = (PA + PB + (PAD ? 1 : 0)) * 1024;
  static constexpr int OS = BM * 2 + 16;                  // epilogue staging row stride (bytes)
  static constexpr int LDS = STAGE * 2 > BN * OS ? STAGE * 2 : BN * OS;
  static_assert(PA % NW == 0, "A pieces split evenly over the waves");
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <typename T, typename G>
__global__ __launch_bounds__(G::NTHR, G::NW / 4) void conv_mt_kernel(ConvParams p, int lnf) {
  using MM = Mma16<T>;
  typedef typename MM::frag Frag;
  constexpr int WM = G::WM, MT = G::MT, NT = G::NT, NW = G::NW, NTHR = G::NTHR;
  constexpr int BM = G::BM, BN = G::BN, PA = G::PA, PB = G::PB, JA = G::JA, JB = G::JB;
  constexpr int STAGE = G::STAGE, OS = G::OS;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // XCD-ordered 1-D grid: block i takes item (i mod 8) * per + i / 8 of the (utterance, row tile,
  // M block) sequence, M block fastest -- an XCD walks the M blocks of the same X rows (its L2)
  const int nmb = p.M / BM;
  const int nrt = (p.y_rows + BN - 1) / BN;
  const int total = nmb * nrt * p.B;
  const int per = (total + 7) / 8;
  const int v = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (v >= total) return;
  const int mb = v % nmb;
  const int rt = (v / nmb) % nrt;
  const int b = v / (nmb * nrt);
  const int n0 = rt * BN;
  const int ylen = p.y_len ? min(p.y_len[b], p.y_rows) : p.y_rows;
  if (n0 >= ylen) return;
  const int xlen = p.x_len ? min(p.x_len[b], p.x_rows) : p.x_rows;
  const int m0 = mb * BM;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;

  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.sxb;
  const int KW = p.w_ld;  // = taps * Cin
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.w), 0, p.M * KW * (int)sizeof(T), 0x00020000);
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(X), 0, xlen * p.sxr * (int)sizeof(T), 0x00020000);

  // this lane's source byte offsets of its pieces at k-tile 0 (k-tile (t, c) adds a uniform amount)
  const int lr = lane >> 3;                       // row within a piece
  int va[JA], vb[JB];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int r = 8 * (j * NW + wave) + lr;       // A tile row
    va[j] = ((m0 + r) * KW + 8 * ((lane & 7) ^ ((r >> 1) & 7))) * (int)sizeof(T);
  }
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int q = j * NW + wave;                  // B piece
    const int r = 8 * q + lr;                     // B tile row
    vb[j] = q < PB ? ((n0 + r - p.pad) * p.sxr + 8 * ((lane & 7) ^ ((r >> 1) & 7))) * (int)sizeof(T)
                   : (int)0x80000000;             // padding piece: out of range, lands in the junk slot
  }
  const int CPT = p.Cin / 64;
  const int KT = p.taps * CPT;
  // k-tile kt's pieces into `stage`; past the last k-tile every piece is out of range (it reads
  // nothing and writes zeros): the loop issues the same count every iteration, with no branch
  auto issue = [&](int kt, int stage) __attribute__((always_inline)) {
    const bool live = kt < KT;
    const int t = kt / CPT, c = kt - t * CPT;
    char* sb = smem + stage * STAGE;
    const int ao = (t * p.Cin + 64 * c) * (int)sizeof(T);
    const int bo = (t * p.dil * p.sxr + 64 * c) * (int)sizeof(T);
#pragma unroll
    for (int j = 0; j < JA; ++j) mt_dma16(wrs, sb + (j * NW + wave) * 1024, live ? va[j] + ao : (int)0x80000000);
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int q = j * NW + wave;
      mt_dma16(xrs, sb + (PA + (q < PB ? q : PB)) * 1024, live ? vb[j] + bo : (int)0x80000000);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: lane l reads row (l & 15) of a 16-row tile, chunk 4 ks + (l >> 4)
  int fo[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) fo[ks] = (lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4);
  const int arow = wm * MT * 16 * 128;
  const int brow = PA * 1024 + wn * NT * 16 * 128;

  // Software pipeline over k-tiles, two LDS stages, one barrier per k-tile placed between a
  // tile's two 32-deep k-steps: the k-step-0 fragments of tile kt are in registers when iteration
  // kt starts; its k-step-1 fragments are read while the k-step-0 MFMAs run; then every wave waits
  // for its reads (lgkmcnt) and for tile kt + 1's DMA (vmcnt), the barrier makes both block-wide,
  // tile kt + 2's DMA goes into the stage tile kt just vacated, tile kt + 1's k-step-0 fragments
  // are read, and the k-step-1 MFMAs cover that DMA issue and those reads.
  Frag fa0[MT], fb0[NT], fa1[MT], fb1[NT];
  auto readf = [&](Frag (&a)[MT], Frag (&bq)[NT], const char* sb, int ks) __attribute__((always_inline)) {
#if TTS_MT_PROBE == 3
    if (ks == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = *reinterpret_cast<const Frag*>(smem + 16 * mt + fo[0]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bq[nt] = *reinterpret_cast<const Frag*>(smem + 1024 + 16 * nt + fo[0]);
    }
    return;
#endif
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = *reinterpret_cast<const Frag*>(sb + arow + mt * 2048 + fo[ks]);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bq[nt] = *reinterpret_cast<const Frag*>(sb + brow + nt * 2048 + fo[ks]);
  };
  auto mmas = [&](const Frag (&a)[MT], const Frag (&bq)[NT]) __attribute__((always_inline)) {
#if TTS_MT_PROBE == 2
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) asm volatile("" ::"v"(a[mt]));
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) asm volatile("" ::"v"(bq[nt]));
    return;
#endif
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = MM::mma(a[mt], bq[nt], acc[mt][nt]);
  };
  issue(0, 0);
  issue(1, 1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(JA + JB) : "memory");  // tile 0's pieces (tile 1's stay in flight)
  __builtin_amdgcn_s_barrier();  // (not __syncthreads: its fence may drain tile 1's pieces too)
  asm volatile("" ::: "memory");
  readf(fa0, fb0, smem, 0);
  // instruction interleave (sched_group_barrier masks: 0x008 MFMA, 0x020 VMEM read -- the LDS-DMA
  // pieces --, 0x100 DS read): reads and DMA issues spread between the MFMAs instead of bunched
  // ahead of them (the scheduler otherwise also sinks the next tile's reads to their first use,
  // exposing their latency at the top of the next k-step)
  constexpr int NF = MT + NT, NMF = MT * NT, ND = JA + JB;
  constexpr int MPR = NMF / NF > 0 ? NMF / NF : 1;  // MFMAs per fragment read
  constexpr int MPD = 2;                            // MFMAs per DMA piece
  for (int kt = 0; kt < KT; ++kt) {
    const char* sb = smem + (kt & 1) * STAGE;
    readf(fa1, fb1, sb, 1);
    mmas(fa0, fb0);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MPR, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NF * MPR > 0 ? NMF - NF * MPR : 0, 0);
    // (the MFMAs are register-only: without the pins the scheduler moves them across the barrier)
    __builtin_amdgcn_sched_barrier(0);
    // tile kt + 1's pieces: the compiler does not count an LDS-DMA as an LDS write at the barrier
    // (it emits only lgkmcnt(0) there), so the wait is explicit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // + lgkmcnt(0): tile kt read by every wave, tile kt + 1 landed everywhere
    __builtin_amdgcn_sched_barrier(0);
#if TTS_MT_PROBE != 1
    issue(kt + 2, kt & 1);
#endif
    readf(fa0, fb0, smem + ((kt + 1) & 1) * STAGE, 0);  // (after the last tile: unused)
    mmas(fa1, fb1);
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - ND - NF > 0 ? NMF - ND - NF : 0, 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing out-of-range pieces land before LDS is reused

  // ---- epilogue: (acc + bias) * alpha -> act -> T, staged as [BN rows][BM channels] ----
  f32x4 bl[MT];
  {
    const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias ? p.bias : reinterpret_cast<const float*>(p.y)),
                                                       0, p.bias ? p.M * 4 : 0, 0x00020000);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      bl[mt] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              brs, (m0 + (wm * MT + mt) * 16 + 4 * (lane >> 4)) * 4, 0, 0));
  }
  __syncthreads();  // every wave's MFMAs are past the last stage
  auto stage_acc = [&](auto act_c) __attribute__((always_inline)) {
    constexpr int ACT = decltype(act_c)::value;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        f32x4 x = (acc[mt][nt] + bl[mt]) * p.alpha;
        if constexpr (ACT != ACT_NONE) {
#pragma unroll
          for (int i = 0; i < 4; ++i) x[i] = apply_act(x[i], ACT, p.out_slope);
        }
        *reinterpret_cast<uint2*>(smem + ((wn * NT + nt) * 16 + (lane & 15)) * OS + ((wm * MT + mt) * 16 + 4 * (lane >> 4)) * 2) =
            pack4<T>(x);
      }
  };
  switch (p.act_out) {
    case ACT_RELU: stage_acc(ActC<ACT_RELU>{}); break;
    case ACT_TANH: stage_acc(ActC<ACT_TANH>{}); break;
    case ACT_LRELU: stage_acc(ActC<ACT_LRELU>{}); break;
    case ACT_SILU: stage_acc(ActC<ACT_SILU>{}); break;
    default: stage_acc(ActC<ACT_NONE>{}); break;
  }
  __syncthreads();

  // ---- row pass: 16-byte pieces (8 channels) + residual, * out_scale -> Y (or back to LDS) ----
  constexpr int PPR = BM / 8;
  constexpr int NIT = (BN * PPR + NTHR - 1) / NTHR;
  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.syb;
  const T* R1 = p.r1 ? reinterpret_cast<const T*>(p.r1) + (long long)b * p.srb : nullptr;
  const bool plain = !R1 && p.out_scale == 1.0f;
  const int nrow = min(BN, ylen - n0);
  // residual pieces all in flight at once, through a descriptor with no records when there is no
  // residual (unconditional loads: a load under `if (R1)` is waited on right after it issues)
  uint4 res[NIT];
  {
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(R1 ? R1 : Y), 0, R1 ? 0x7fffffff : 0, 0x00020000);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int pc = tid + it * NTHR;
      const int r = min(pc / PPR, nrow - 1), cp = pc % PPR;
      res[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rrs, ((n0 + r) * p.srr + m0 + cp * 8) * (int)sizeof(T), 0, 0));
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int pc = tid + it * NTHR;
    if (pc >= nrow * PPR) break;
    const int r = pc / PPR, cp = pc % PPR;
    char* sp = smem + r * OS + cp * 16;
    uint4 y = *reinterpret_cast<const uint4*>(sp);
    if (!plain) {
      const T* e = reinterpret_cast<const T*>(&y);
      const T* f = reinterpret_cast<const T*>(&res[it]);
      f32x4 v0 = {(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
      f32x4 v1 = {(float)e[4], (float)e[5], (float)e[6], (float)e[7]};
      if (R1) {
        v0 += f32x4{(float)f[0], (float)f[1], (float)f[2], (float)f[3]};
        v1 += f32x4{(float)f[4], (float)f[5], (float)f[6], (float)f[7]};
      }
      v0 *= p.out_scale;
      v1 *= p.out_scale;
      y = pack8<T>(v0, v1);
    }
    if (lnf) *reinterpret_cast<uint4*>(sp) = y;
    else store16<TTS_MT_STORE>(Y, (int)(((long long)(n0 + r) * p.syr + m0 + cp * 8) * (long long)sizeof(T)), y);
  }
  if (!lnf) return;

  // ---- the post-LayerNorm of the staged rows (BM == M: the block owns whole rows) ----
  __syncthreads();
  constexpr int RB = TTS_MT_LN_RB;
  const int C = p.M;
  int ch[8];
  bool on[8];
  ln_lanes8(ch, on, C, lane);
  float g[2][8], bb[2][8];
  ln_params8v(g, bb, on[0], ch[0], p.ln_g1, p.ln_b1, p.ln_g2, p.ln_b2);
  T* L = reinterpret_cast<T*>(p.ln_out) + (long long)b * p.syb;
  const int c0 = on[0] ? ch[0] : 0;
  for (int r0 = wave; r0 < nrow; r0 += NW * RB) {
    float vv[RB][8];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = min(r0 + NW * k, nrow - 1);
      const uint4 u = on[0] ? *reinterpret_cast<const uint4*>(smem + r * OS + c0 * 2) : uint4{0u, 0u, 0u, 0u};
      ln_unpack8<T>(u, vv[k]);
    }
    if (p.ln_g2) ln_batch<T, RB, 8, true>(vv, on, C, g, bb, p.ln_eps);
    else ln_batch<T, RB, 8, false>(vv, on, C, g, bb, p.ln_eps);
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = r0 + NW * k;
      if (on[0] && r < nrow)
        store16<TTS_MT_STORE>(L, (int)(((long long)(n0 + r) * p.syr + c0) * (long long)sizeof(T)), ln_pack8<T>(vv[k]));
    }
  }
}

// ------------------------------------------------------------------------------- host side
#ifndef TTS_CONV_MT
#define TTS_CONV_MT 1
#endif

typedef MtGeom<4, 2, 4, 7> MtA;  // 256 channels x 224 rows (FFN up-projection, wide projections)
typedef MtGeom<4, 2, 3, 7> MtB;  // 192 x 224
typedef MtGeom<8, 1, 3, 7> MtC;  // 384 x 112 (whole 384-channel rows: the fused post-LN)
typedef MtGeom<4, 2, 2, 4> MtD;  // 128 x 128 (small grids)

namespace {
struct MtCfg {
  int id, BM, BN;
};
constexpr MtCfg kCfgs[] = {{0, MtA::BM, MtA::BN}, {1, MtB::BM, MtB::BN}, {2, MtC::BM, MtC::BN}, {3, MtD::BM, MtD::BN}};

// whether the post-LN can run in the launch (ln_out form; the block owns whole rows of <= 512 channels)
bool mt_ln_ok(const ConvParams& p, int BM) {
  return p.ln_out && !p.ln_lin_out && BM == p.M && p.M <= 512 && p.M % 8 == 0 && sw(SW_LN_FUSE) != 0 &&
         p.syr % 8 == 0 && p.syb % 8 == 0;
}
}  // namespace

bool conv_mt_eligible(int dtype, const ConvParams& p) {
  if (!TTS_CONV_MT || sw(SW_CONV_MT) == 0 || dtype == DT_F32) return false;
  if (p.nh != 1 || p.up_s || p.in_slope != 1.0f || p.Cin % 64 || p.M % 128 && p.M % 192 && p.M % 384) return false;
  if (p.r2 || p.ln_lin_out) return false;
  if (p.sxr % 8 || p.sxb % 8 || p.syr % 8 || p.syb % 8 || (p.r1 && (p.srr % 8 || p.srb % 8))) return false;
  if (p.w_ld != p.taps * p.Cin) return false;
  if ((long long)p.x_rows * p.sxr * 2 >= (1LL << 31) || (long long)p.M * p.w_ld * 2 >= (1LL << 31)) return false;
  if ((long long)p.y_rows * p.syr * 2 >= (1LL << 31) || (p.r1 && (long long)p.y_rows * p.srr * 2 >= (1LL << 31)))
    return false;
  return true;
}

// Tile choice: the configuration whose grid, in rounds of one block per CU, covers the launch in
// the least tile area (rounds x BM x BN), preferring larger tiles on ties.  A row's arithmetic
// is the same in every configuration.
static int mt_pick(const ConvParams& p, int ncu) {
  const int force = sw(SW_MT_TILE);
  if (force >= 0 && force < 4 && p.M % kCfgs[force].BM == 0) return force;
  int best = -1;
  double best_cost = 0;
  for (const MtCfg& c : kCfgs) {
    if (p.M % c.BM) continue;
    const long long tiles = (long long)(p.M / c.BM) * ((p.y_rows + c.BN - 1) / c.BN) * p.B;
    const long long rounds = (tiles + ncu - 1) / ncu;
    const double cost = (double)rounds * c.BM * c.BN;
    if (best < 0 || cost < best_cost * 0.999 || (cost <= best_cost * 1.001 && c.BM * c.BN > kCfgs[best].BM * kCfgs[best].BN)) {
      best = c.id;
      best_cost = cost;
    }
  }
  return best;
}

template <typename T, typename G>
static hipError_t mt_launch_g(const ConvParams& p, hipStream_t s, bool* ln_done) {
  const int lnf = mt_ln_ok(p, G::BM) ? 1 : 0;
  if (ln_done) *ln_done = lnf != 0;
  const int total = (p.M / G::BM) * ((p.y_rows + G::BN - 1) / G::BN) * p.B;
  const dim3 grid(8 * ((total + 7) / 8));
  hipLaunchKernelGGL((conv_mt_kernel<T, G>), grid, dim3(G::NTHR), G::LDS, s, p, lnf);
  return hipGetLastError();
}

template <typename T>
static hipError_t mt_launch_t(const ConvParams& p, hipStream_t s, bool* ln_done) {
  switch (mt_pick(p, device_cu_count())) {
    case 0: return mt_launch_g<T, MtA>(p, s, ln_done);
    case 1: return mt_launch_g<T, MtB>(p, s, ln_done);
    case 2: return mt_launch_g<T, MtC>(p, s, ln_done);
    case 3: return mt_launch_g<T, MtD>(p, s, ln_done);
  }
  return hipErrorInvalidValue;
}

hipError_t conv_mt_launch(int dtype, const ConvParams& p, hipStream_t s, bool* ln_done) {
  if (dtype == DT_F16) return mt_launch_t<half_t>(p, s, ln_done);
  if (dtype == DT_BF16) return mt_launch_t<bf16_t>(p, s, ln_done);
  return hipErrorInvalidValue;
}

}  // namespace tts
