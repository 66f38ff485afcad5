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
#define TTS_MT_PROBE 0  // timing-only diagnostic builds: 1 = no DMA after the prologue, 2 = no MFMA, 3 = no fragment reads,
                        // 4 = no epilogue stores, 5 = (conv_tap) no DMA after the prologue and one LDS stage read throughout,
                        // 6 = (conv_tap) no DMA after the prologue, fragments read once, 7 = (conv_tap) no epilogue
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

// Shared epilogue of the macro-tiled kernels: (acc + bias) * alpha -> activation -> T, staged as
// [BN rows][BM channels] in LDS, then a row pass of 16-byte pieces adds the residual, scales and
// stores; with lnf (BM == M: the block owns whole rows) the post-LayerNorm runs on the staged rows
// and only its output is written.
template <typename T, int BM, int BN, int WM, int MT, int NT, int NTHR, int OS>
__device__ __forceinline__ void mt_epilogue(const ConvParams& p, f32x4 (&acc)[MT][NT], char* smem, int b, int n0, int m0,
                                            int ylen, int wave, int lane, int lnf) {
  constexpr int NW = NTHR / 64;
  const int tid = threadIdx.x;
  const int wm = wave % WM, wn = wave / WM;
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
#if TTS_MT_PROBE == 4
    else if (y.x == 0x7fc07fc0u && y.y == 0x12345678u) store16<TTS_MT_STORE>(Y, 0, y);  // (never: keeps the row pass)
#else
    else store16<TTS_MT_STORE>(Y, (int)(((long long)(n0 + r) * p.syr + m0 + cp * 8) * (long long)sizeof(T)), y);
#endif
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

  mt_epilogue<T, BM, BN, WM, MT, NT, NTHR, OS>(p, acc, smem, b, n0, m0, ylen, wave, lane, lnf);
}

// ------------------------------------------------------------------- multi-tap form (conv_tap)
// The k = 3 FFN convs (and the postnet's k = 5) as one implicit GEMM whose X tile is shared by
// the taps.  conv_mt_kernel above stages a separate B tile per (tap, 64 channels), so the X rows
// of a block cross L2 -> LDS once per tap; its no-MFMA probe build (TTS_MT_PROBE=2) measured the
// FFN up-projection's data movement alone at 73 of its 113 us (profiles/r05c_mt_probe.txt):
// the launch is bound by L2 -> LDS bytes (~70 GB/s per CU, MI355X_MICROARCH.md §Indexed rows),
// not by the MFMA.  Here a stage is one 32-channel group: the A tiles of every tap (taps x BM
// channels x 64 B) and ONE B tile of BN + (taps - 1) * dil rows, from which tap t's fragments
// are read t * dil rows down.  Per stage the block moves (taps * BM + BN + halo) * 64 bytes for
// taps * BM * BN * 64 FLOP: at BM = 128, BN = 448, k = 3, 206 FLOP/B against conv_mt's 119.
//   * 64-byte LDS rows, chunk c of row r at slot c ^ (((r >> 2) & 1) << 1): the 16 x 16 x 32
//     fragment reads (16 rows x 4 chunks per ds_read_b128) take 16 distinct 16-byte slots per
//     bank group at EVERY row shift (checked exhaustively: the taps' shifted reads of the one B
//     image stay conflict-free); the DMA's LDS image is lane-linear, so the swizzle is applied to
//     the source chunk;
//   * an NS-stage ring (NS - 1 channel groups in flight, one barrier per group);
//   * K order: channel group (32) outer, tap inner, one v_mfma_f32_16x16x32 per (group, tap) --
//     the same for every tile shape and batch size (a row's bits do not depend on the batch);
//   * the epilogue is conv_mt's.
template <int WM_, int WN_, int MT_, int NT_, int TAPS_, int NS_>
struct TapGeom {
  static constexpr int WM = WM_, WN = WN_, MT = MT_, NT = NT_, TAPS = TAPS_, NS = NS_;
  static constexpr int NW = WM * WN, NTHR = 64 * NW;
  static constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  static constexpr int HALO = 16;                          // rows past BN staged (>= (taps - 1) * dil)
  static constexpr int BH = BN + HALO;                     // B tile rows
  static constexpr int PA = TAPS * BM / 16, PB = BH / 16;  // 1 KiB pieces (16 rows of 64 B)
  static constexpr int P = PA + PB;
  static constexpr int JP = (P + NW - 1) / NW;             // pieces per wave (the last may be padding)
  static constexpr bool PAD = JP * NW > P;
  static constexpr int STAGE = (P + (PAD ? 1 : 0)) * 1024;
  static constexpr int OS = BM * 2 + 16;                   // epilogue staging row stride (bytes)
  static constexpr int LDS = STAGE * NS > BN * OS ? STAGE * NS : BN * OS;
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(NS >= 2 && (NS - 2) * JP <= 63, "vmcnt wait count");
  // blocks per CU the LDS allows, and the waves per SIMD the register budget is sized for
  static constexpr int OCC = 160 * 1024 / LDS;
  static constexpr int WPE = OCC * NW / 4 > 1 ? OCC * NW / 4 : 1;
};

// row r's chunk slot swizzle of the 64-byte-row images
__device__ inline int tap_swz(int r) { return ((r >> 2) & 1) << 1; }

template <typename T, typename G>
__global__ __launch_bounds__(G::NTHR, G::WPE) void conv_tap_kernel(ConvParams p, int lnf) {
  using MM = Mma16<T>;
  typedef typename MM::frag Frag;
  constexpr int WM = G::WM, MT = G::MT, NT = G::NT, NW = G::NW, NTHR = G::NTHR, TAPS = G::TAPS, NS = G::NS;
  constexpr int BM = G::BM, BN = G::BN, PA = G::PA, P = G::P, JP = G::JP, STAGE = G::STAGE, OS = G::OS;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // XCD-ordered 1-D grid (as conv_mt_kernel): M block fastest within an XCD's run of items
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

  // this lane's source byte offsets of its pieces for channel group 0 (group g adds 64 g bytes);
  // lane l of a piece lands at LDS row l >> 2, slot l & 3, and loads the source chunk that slot holds
  const int rip = lane >> 2;
  const int csrc = (lane & 3) ^ tap_swz(rip);
  int off[JP];
#pragma unroll
  for (int j = 0; j < JP; ++j) {
    const int q = j * NW + wave;
    if (q < PA) {
      const int t = q / (BM / 16), i = q - t * (BM / 16);
      off[j] = ((m0 + 16 * i + rip) * KW + t * p.Cin + 8 * csrc) * (int)sizeof(T);
    } else if (q < P) {
      off[j] = ((n0 - p.pad + 16 * (q - PA) + rip) * p.sxr + 8 * csrc) * (int)sizeof(T);  // rows < 0: out of range
    } else {
      off[j] = (int)0x80000000;  // padding piece: reads nothing, lands in the junk slot
    }
  }
  const int NG = p.Cin / 32;  // stages: one per 32-channel group
  // stage g's pieces into ring slot `slot`; past the last group every piece is out of range (the
  // per-wave count of memory operations is the same every stage)
  auto issue = [&](int g, int slot) __attribute__((always_inline)) {
    char* sb = smem + slot * STAGE;
    const bool live = g < NG;
#pragma unroll
    for (int j = 0; j < JP; ++j) {
      const int q = j * NW + wave;
      const bool isa = q < PA;
      const auto rs = isa ? wrs : xrs;
      mt_dma16(rs, sb + (q < P ? q : P) * 1024, live ? off[j] + 64 * g : (int)0x80000000);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment byte offsets in a stage: A of tap t at t * BM * 64 (+ the wave's rows), B of tap t
  // t * dil rows down the one B image
  const int l15 = lane & 15, lq = lane >> 4;
  const int aoff = (wm * MT * 16 + l15) * 64 + ((lq ^ tap_swz(l15)) << 4);
  int boff[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t) {
    const int r = l15 + t * p.dil;
    boff[t] = PA * 1024 + (wn * NT * 16 + r) * 64 + ((lq ^ tap_swz(r)) << 4);
  }

  // Software pipeline over steps (group g, tap t): step j's fragments are in registers while
  // step j + 1's are read (two register sets, alternating; two groups per loop trip keep the
  // alternation static for an odd tap count, so NG must be even).  At a group's last tap the
  // block syncs on the next group first: its pieces have landed (the younger NS - 2 groups' stay
  // in flight) and every wave has read the group before it, whose slot takes group g + NS.
  Frag f0a[MT], f0b[NT], f1a[MT], f1b[NT];
  auto readf = [&](Frag (&a)[MT], Frag (&bq)[NT], const char* sb, int t) __attribute__((always_inline)) {
#if TTS_MT_PROBE == 5
    sb = smem;
#endif
#if TTS_MT_PROBE == 6
    if (t != 0 || sb != smem) return;
#endif
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = *reinterpret_cast<const Frag*>(sb + t * BM * 64 + aoff + mt * 1024);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bq[nt] = *reinterpret_cast<const Frag*>(sb + boff[t] + nt * 1024);
  };
  auto mmas = [&](const Frag (&a)[MT], const Frag (&bq)[NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = MM::mma(a[mt], bq[nt], acc[mt][nt]);
  };
  auto sync_group = [&](int g) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NS - 2) * JP) : "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#if TTS_MT_PROBE != 1 && TTS_MT_PROBE != 5 && TTS_MT_PROBE != 6
    issue(g + NS - 1, (g + NS - 1) % NS);
#endif
  };
  // reads of the next step spread between this step's MFMAs (masks: 0x008 MFMA, 0x100 DS read)
  constexpr int NF = MT + NT, NMF = MT * NT;
  constexpr int MPR = NMF / NF > 0 ? NMF / NF : 1;
  auto interleave = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MPR, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NF * MPR > 0 ? NMF - NF * MPR : 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // one step: the next step's fragments into (na, nb) while (ca, cb)'s MFMAs run
  auto step = [&](Frag (&ca)[MT], Frag (&cb)[NT], Frag (&na)[MT], Frag (&nb)[NT], int g, int t) __attribute__((always_inline)) {
    if (t + 1 < TAPS) {
      readf(na, nb, smem + (g % NS) * STAGE, t + 1);
    } else if (g + 1 < NG) {
      sync_group(g + 1);
      readf(na, nb, smem + ((g + 1) % NS) * STAGE, 0);
    }
    mmas(ca, cb);
    interleave();
  };
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(i, i);
  sync_group(0);
  readf(f0a, f0b, smem, 0);
  for (int g = 0; g < NG; g += 2) {
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      if ((t & 1) == 0) step(f0a, f0b, f1a, f1b, g, t);
      else step(f1a, f1b, f0a, f0b, g, t);
    }
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      if (((TAPS + t) & 1) == 0) step(f0a, f0b, f1a, f1b, g + 1, t);
      else step(f1a, f1b, f0a, f0b, g + 1, t);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing out-of-range pieces land before LDS is reused
#if TTS_MT_PROBE == 7
  if (acc[0][0][0] != 12345.f) return;  // (timing probe: no epilogue)
#endif

  mt_epilogue<T, BM, BN, WM, MT, NT, NTHR, OS>(p, acc, smem, b, n0, m0, ylen, wave, lane, lnf);
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

static bool conv_tap_eligible(const ConvParams& p);

// Default off (TTS_CONV_MT=1 opts in): measured per layer against conv_xres in the acoustic
// forward (profiles/r05d_ac_trace_tap_vs_xres.txt), the macro-tiled kernels tie at batch 32 and
// lose ~5 % at batch 8 (the C5 first-chunk path); a layer's kernel may not depend on the batch size
// (its K order fixes the row's bits), so one choice serves both.
#ifndef TTS_CONV_MT_DEFAULT
#define TTS_CONV_MT_DEFAULT 0
#endif
bool conv_mt_eligible(int dtype, const ConvParams& p) {
  const int on = sw(SW_CONV_MT) < 0 ? TTS_CONV_MT_DEFAULT : sw(SW_CONV_MT);
  if (!TTS_CONV_MT || on == 0 || dtype == DT_F32) return false;
  if (p.nh != 1 || p.up_s || p.in_slope != 1.0f) return false;
  if (!conv_tap_eligible(p) && (p.Cin % 64 || p.M % 128 && p.M % 192 && p.M % 384)) return false;
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

// ---- the multi-tap form: k = 3 layers (the FFN convs).  Configurations (TTS_MT_TILE = 4 + index
// forces one; a row's arithmetic is the same in every one):
#ifndef TTS_CONV_TAP
#define TTS_CONV_TAP 1
#endif
#ifndef TTS_TAP_AUTO_N
#define TTS_TAP_AUTO_N 5  // configurations the automatic choice considers (the rest: forced only)
#endif
typedef TapGeom<2, 4, 3, 7, 3, 3> TapA;  // 96 channels x 448 rows, 3 stages (144 KB)
typedef TapGeom<4, 2, 3, 7, 3, 3> TapB;  // 192 x 224, 3 stages (156 KB)
typedef TapGeom<4, 2, 3, 7, 3, 2> TapC;  // 192 x 224, 2 stages (104 KB)
typedef TapGeom<4, 2, 2, 7, 3, 3> TapD;  // 128 x 224, 3 stages (120 KB)
typedef TapGeom<4, 2, 2, 4, 3, 3> TapE;  // 128 x 128, 3 stages (small grids)
typedef TapGeom<2, 2, 2, 7, 3, 2> TapF;  // 4 waves, 64 x 224, 2 stages (56 KB: two blocks per CU)
typedef TapGeom<2, 2, 3, 7, 3, 2> TapG;  // 4 waves, 96 x 224, 2 stages (68 KB: two blocks per CU)
// (wave tiles of 4 x 7 accumulator tiles spill with the software-pipelined fragment sets)
namespace {
constexpr MtCfg kTapCfgs[] = {{0, TapA::BM, TapA::BN}, {1, TapB::BM, TapB::BN}, {2, TapC::BM, TapC::BN},
                              {3, TapD::BM, TapD::BN}, {4, TapE::BM, TapE::BN}, {5, TapF::BM, TapF::BN},
                              {6, TapG::BM, TapG::BN}};
constexpr int kNTap = sizeof(kTapCfgs) / sizeof(kTapCfgs[0]);
}  // namespace

static bool conv_tap_eligible(const ConvParams& p) {
  if (!TTS_CONV_TAP || sw(SW_CONV_MT) == 2) return false;  // (TTS_CONV_MT=2: k = 3 layers on conv_mt_kernel)
  if (p.taps != 3 || p.Cin % 64 || (p.taps - 1) * p.dil > 16 || p.dil < 1) return false;  // (an even group count)
  for (const MtCfg& c : kTapCfgs)
    if (p.M % c.BM == 0) return true;
  return false;
}

static int tap_pick(const ConvParams& p, int ncu) {
  const int force = sw(SW_MT_TILE) - 4;
  if (force >= 0 && force < kNTap && p.M % kTapCfgs[force].BM == 0) return force;
  int best = -1;
  double best_cost = 0;
  for (const MtCfg& c : kTapCfgs) {
    if (p.M % c.BM || c.id >= TTS_TAP_AUTO_N) continue;
    const long long tiles = (long long)(p.M / c.BM) * ((p.y_rows + c.BN - 1) / c.BN) * p.B;
    const long long rounds = (tiles + ncu - 1) / ncu;
    const double cost = (double)rounds * c.BM * c.BN;
    if (best < 0 || cost < best_cost * 0.999 || (cost <= best_cost * 1.001 && c.BM * c.BN > kTapCfgs[best].BM * kTapCfgs[best].BN)) {
      best = c.id;
      best_cost = cost;
    }
  }
  return best;
}

template <typename T, typename G>
static hipError_t tap_launch_g(const ConvParams& p, hipStream_t s, bool* ln_done) {
  const int lnf = mt_ln_ok(p, G::BM) ? 1 : 0;
  if (ln_done) *ln_done = lnf != 0;
  const int total = (p.M / G::BM) * ((p.y_rows + G::BN - 1) / G::BN) * p.B;
  const dim3 grid(8 * ((total + 7) / 8));
  hipLaunchKernelGGL((conv_tap_kernel<T, G>), grid, dim3(G::NTHR), G::LDS, s, p, lnf);
  return hipGetLastError();
}

template <typename T>
static hipError_t tap_launch_t(const ConvParams& p, hipStream_t s, bool* ln_done) {
  switch (tap_pick(p, device_cu_count())) {
    case 0: return tap_launch_g<T, TapA>(p, s, ln_done);
    case 1: return tap_launch_g<T, TapB>(p, s, ln_done);
    case 2: return tap_launch_g<T, TapC>(p, s, ln_done);
    case 3: return tap_launch_g<T, TapD>(p, s, ln_done);
    case 4: return tap_launch_g<T, TapE>(p, s, ln_done);
    case 5: return tap_launch_g<T, TapF>(p, s, ln_done);
    case 6: return tap_launch_g<T, TapG>(p, s, ln_done);
  }
  return hipErrorInvalidValue;
}

hipError_t conv_mt_launch(int dtype, const ConvParams& p, hipStream_t s, bool* ln_done) {
  const bool tap = conv_tap_eligible(p);
  if (dtype == DT_F16) return tap ? tap_launch_t<half_t>(p, s, ln_done) : mt_launch_t<half_t>(p, s, ln_done);
  if (dtype == DT_BF16) return tap ? tap_launch_t<bf16_t>(p, s, ln_done) : mt_launch_t<bf16_t>(p, s, ln_done);
  return hipErrorInvalidValue;
}

}  // namespace tts
