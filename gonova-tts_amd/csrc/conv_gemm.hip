// Implicit-GEMM 1-D convolution on gfx950 MFMA, channels-last.
//
//   Y[b][n][m] = epi( sum_{tap, c} W[m][tap][c] * act_in( X[b][n + tap*dil - pad][c] ) )
//
// This one kernel family carries every dense contraction of the hot path:
//   * HiFi-GAN conv_pre / MRF dilated convs (k=3,7,11; d=1,3,5) with the
//     LeakyReLU(0.1) pre-activation fused into the LDS staging and the
//     residual add + MRF sum/3 fused into the epilogue
//     (oracle: oracle/vocoder.py resblock / vocoder_forward);
//   * ConvTranspose1d upsamplers as polyphase convs (taps = k/s, M = s*Cout,
//     output row n*s + m/Cout - p), see engine.cpp pack_transposed();
//   * the acoustic model's FFN convs (k=3), linears (k=1), attention GEMMs.
//
// Layout in HBM: activations [B][rows][C] with C contiguous (one mel frame /
// sample per row).  A dilated conv then reads k shifted copies of one LDS
// tile of X rows, so each input row is fetched from HBM once per block.
//
// Tiling: a block = WM x WN waves; each wave owns MT x NT 32x32 MFMA tiles
// (M = output channels, N = time).  Weights stream from L2 straight into the
// A fragments, prefetched one tap ahead (every wave reads distinct rows of W,
// so there is no intra-block sharing to stage through LDS).  The X tile is
// staged through LDS in CK-channel chunks, double-buffered: the global loads of
// chunk c+1 are issued into registers before chunk c's MFMAs and written to the
// other LDS buffer after them (one barrier per chunk).  LDS rows carry a 16-byte
// pad (row stride 80 B or 144 B) so ds_read_b128 of 16 consecutive rows hits 16
// distinct 4-bank slots: conflict-free.  Loads are clamped in-bounds and masked
// after the fact (no per-element branches around loads).
#include "common.h"
#include "conv_epilogue.h"
#include "acoustic_kernels.h"
#include "kernels.h"
#include "ln_rows.h"
#include "switches.h"

#include <algorithm>
#include <cstdlib>

namespace tts {

constexpr int HALO_MAX = 64;  // max (taps-1)*dil supported (HiFi-GAN V1: 50)

template <typename T>
__device__ inline uint4 act16(uint4 u, bool valid, float slope) {
  if (!valid) return uint4{0u, 0u, 0u, 0u};
  if (slope != 1.0f) u = lrelu_chunk<T>(u, slope);
  return u;
}

template <typename T>
__device__ inline typename Mfma<T>::frag load_afrag(const T* ptr, bool valid) {
  typedef typename Mfma<T>::frag F;
  if constexpr (sizeof(T) == 4) {
    const float v = *ptr;
    return valid ? v : 0.0f;
  } else {
    uint4 u = *reinterpret_cast<const uint4*>(ptr);
    if (!valid) u = uint4{0u, 0u, 0u, 0u};
    return *reinterpret_cast<F*>(&u);
  }
}

template <typename T, int MT, int NT, int WM, int WN, int CK>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_gemm_kernel(ConvParams p) {
  using MF = Mfma<T>;
  typedef typename MF::frag Frag;
  constexpr int BM = 32 * MT * WM;
  constexpr int BN = 32 * NT * WN;
  constexpr int NTHR = 64 * WM * WN;
  constexpr int EPV = 16 / (int)sizeof(T);      // elements per 16-byte vector
  constexpr int VPR = CK / EPV;                 // vectors per row chunk
  constexpr int LDSR = CK + EPV;                // LDS row stride (elements): +16 B pad
  constexpr int KS = CK / MF::KSTEP;            // MFMA k-steps per chunk and tap
  constexpr int PF = ((BN + HALO_MAX) * VPR + NTHR - 1) / NTHR;  // prefetch vectors per thread

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nh = p.nh;
  // (bx, by, bz): row tile, M block, utterance x head -- the grid's own, or decoded from the 1-D
  // XCD-ordered grid (ConvParams::xres_order)
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  int gx = gridDim.x, gy = gridDim.y;
  if (p.xres_order) {
    gx = (p.y_rows + BN - 1) / BN;
    gy = (p.M + BM - 1) / BM;
    const int total = gx * gy * p.B * nh;
    const int per = (total + 7) / 8;
    const int v = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (v >= total) return;  // padding blocks of the last XCD range (no tile, no counter)
    by = v % gy;
    const int r = v / gy;
    bx = r % gx;
    bz = r / gx;
  }
  // split-K (ConvParams::kslices, fp32): grid z = utterance x slice; slice sl covers Cin chunks
  // [c_lo, c_hi) of every tap and leaves its raw sums to the reduce
  const int S = p.kslices > 1 ? p.kslices : 1;
  const int sl = bz % S;
  bz /= S;
  const int b = bz / nh;
  const int hd = bz - b * nh;
  const int n0 = bx * BN;
  const int ylen = p.y_len ? min(p.y_len[b], p.y_rows) : p.y_rows;
  if (n0 >= ylen) return;
  const int xlen = p.x_len ? min(p.x_len[b], p.x_rows) : p.x_rows;
  const int m_blk = by * BM;  // (the decoded M block on the XCD-ordered grid)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int m_w0 = m_blk + wm * 32 * MT;
  const int n_w0 = wn * 32 * NT;
  const int l31 = lane & 31;
  const int hh = lane >> 5;

  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.sxb + (long long)hd * p.sxh;
  const T* W = reinterpret_cast<const T*>(p.w) + (long long)b * p.swb + (long long)hd * p.swh;
  const int R = BN + (p.taps - 1) * p.dil;
  const int RV = R * VPR;
  const int x_start = n0 - p.pad;
  const int tile = R * LDSR;
  T* xs0 = reinterpret_cast<T*>(smem);
  T* xs1 = xs0 + tile;
  const int nchunks = (p.Cin + CK - 1) / CK;
  const int cps = (nchunks + S - 1) / S;
  const int c_lo = sl * cps, c_hi = min(nchunks, c_lo + cps);
  const int k_end = min(p.Cin, c_hi * CK);  // this slice's channel end
  const int xlast = xlen > 0 ? xlen - 1 : 0;

  // ---- X chunk staging: global -> registers (raw) -> act/mask -> LDS ----
  uint4 pf[PF];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int v = tid + i * NTHR;
      const int r = v / VPR;
      const int cv = v - r * VPR;
      const int xr = min(max(x_start + r, 0), xlast);
      const int c = min(c0 + cv * EPV, p.Cin - EPV);
      pf[i] = *reinterpret_cast<const uint4*>(X + (long long)xr * p.sxr + c);
    }
  };
  auto store_chunk = [&](T* buf, int c0) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int v = tid + i * NTHR;
      if (v < RV) {
        const int r = v / VPR;
        const int cv = v - r * VPR;
        const int xr = x_start + r;
        const bool ok = (xr >= 0) && (xr < xlen) && (c0 + cv * EPV < p.Cin);
        *reinterpret_cast<uint4*>(buf + r * LDSR + cv * EPV) = act16<T>(pf[i], ok, p.in_slope);
      }
    }
  };

  // ---- A (weight) fragments, one tap of one chunk ----
  const T* wrow[MT];
  bool mok[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = m_w0 + mt * 32 + l31;
    mok[mt] = m < p.M;
    wrow[mt] = W + (long long)(mok[mt] ? m : 0) * p.w_ld;
  }
  auto load_a = [&](Frag (&a)[MT][KS], int c0, int tap) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int k = c0 + ks * MF::KSTEP + hh * MF::KPL;
        const bool ok = mok[mt] && (k < p.Cin);
        a[mt][ks] = load_afrag<T>(wrow[mt] + tap * p.Cin + (ok ? k : 0), ok);
      }
  };

  f32x16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x16{};

  Frag a_cur[MT][KS], a_nxt[MT][KS];
  load_chunk(c_lo * CK);
  load_a(a_cur, c_lo * CK, 0);
  store_chunk(xs0, c_lo * CK);
  __syncthreads();

  for (int ci = c_lo; ci < c_hi; ++ci) {
    const T* cur = ((ci - c_lo) & 1) ? xs1 : xs0;
    T* nxt = ((ci - c_lo) & 1) ? xs0 : xs1;
    const int c0 = ci * CK;
    const bool has_next = ci + 1 < c_hi;
    if (has_next) load_chunk(c0 + CK);
    for (int tap = 0; tap < p.taps; ++tap) {
      int ntap = tap + 1, nc0 = c0;
      if (ntap == p.taps) { ntap = 0; nc0 = c0 + CK; }
      if (nc0 < k_end) load_a(a_nxt, nc0, ntap);
      const T* xrow = cur + (n_w0 + l31 + tap * p.dil) * LDSR + hh * MF::KPL;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag bf[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          bf[nt] = *reinterpret_cast<const Frag*>(xrow + nt * 32 * LDSR + ks * MF::KSTEP);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = MF::mma(a_cur[mt][ks], bf[nt], acc[mt][nt]);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a_cur[mt][ks] = a_nxt[mt][ks];
    }
    if (has_next) store_chunk(nxt, c0 + CK);
    __syncthreads();
  }

  if (S > 1) {  // this slice's raw sums: ws[sl][b][n][m] (split_reduce_launch applies the epilogue)
    float* P = p.ws + ((long long)sl * p.B + b) * p.y_rows * p.M;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = n0 + n_w0 + nt * 32 + l31;
        if (n >= ylen) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m = m_w0 + mt * 32 + 8 * g + 4 * hh;
          if (m < p.M)
            *reinterpret_cast<f32x4*>(P + (long long)n * p.M + m) =
                f32x4{acc[mt][nt][4 * g], acc[mt][nt][4 * g + 1], acc[mt][nt][4 * g + 2], acc[mt][nt][4 * g + 3]};
        }
      }
    return;
  }
  conv_epilogue<T, MT, NT>(p, acc, b, hd, n0 + n_w0, m_w0, ylen, l31, hh);
}

// ---------------------------------------------------------------------------------------
// X-resident variant for M >= 64, 16-bit dtypes, Cin % 64 == 0, fragment-packed weights
// (ConvParams::wpk): HiFi-GAN stages 0-1 and upsamplers, acoustic linears/FFN.
//
// Why (measured on conv_gemm_kernel at C=128/256: 70-83 % of wave cycles in s_waitcnt,
// MFMA busy 13-32 %):
//  * its weight fragments are loaded straight from L2 in fragment shape, 32 rows x 32 B per
//    wave instruction (32 cache lines touched per 1 KiB), which loads the address path;
//    here weights come pre-packed in fragment order, so every weight load is one
//    contiguous 1 KiB wave read;
//  * the next chunk's X rows (an HBM read) were issued before the next tap's weights, and
//    vmcnt retires loads in order; here a block stages one channel group of its X tile
//    (every tap's rows, LeakyReLU applied) in LDS once, and the MFMA loop then has only
//    weight loads in flight: no barriers, weights two quads (4 k-steps = 4*NT MFMAs each)
//    ahead in a 3-deep register ring;
//  * the epilogue's residual reads and output writes were fragment-shaped too (32 rows x
//    8 B); here the fp32 tile goes through LDS (two 64-row halves) and the bias / act /
//    residual / scale pass reads and writes whole 16-byte row pieces.
// The group's X load latency is covered by the other blocks on the CU (LDS <= 53 KB: 3).
//
// Block: 4 waves, WM along M (32 output channels each) x WN = 4/WM along N (32*NT rows
// each): 128 x 128 tiles for M >= 128, 64 x 256 for M = 64.  X tile row
// stride CG*2+16 bytes (an odd number of 16-byte slots: conflict-free ds_read_b128 of 32
// consecutive rows).
constexpr int XRES_HR = 64;            // output rows per N-wave staged per half
#ifndef TTS_XRES_STORE
#define TTS_XRES_STORE 2               // output store cache policy (store16 in common.h)
#endif
#ifndef TTS_XRES_EPI16
#define TTS_XRES_EPI16 1               // epilogue staged in the compute dtype (0: fp32 staging in two halves)
#endif
#ifndef TTS_XRES_OCC
#define TTS_XRES_OCC 3                 // blocks per CU (register budget; LDS tile cap below)
#endif
#ifndef TTS_XRES_SU
#define TTS_XRES_SU 4                  // more spills at 3 blocks/CU: acc + ring are live
#endif
constexpr int XRES_SU = TTS_XRES_SU;   // X staging loads in flight per thread
#ifndef TTS_XRES_UPFIRST
#define TTS_XRES_UPFIRST 1             // transposed-conv (upsampler) launches: X-first staging (XF below)
#endif
constexpr int XRES_SU_XF = 9;          // XF staging: a group's X loads in flight at once (R <= 9 * rstep)

template <typename T>
__device__ inline void ld8(const T* p, f32x4& a, f32x4& b) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const T* e = reinterpret_cast<const T*>(&u);
  a = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
  b = f32x4{(float)e[4], (float)e[5], (float)e[6], (float)e[7]};
}

#ifndef TTS_XRES_STAMP
#define TTS_XRES_STAMP 0               // diagnostic builds only: per-block phase timestamps
#endif
#if TTS_XRES_STAMP
// Phase timestamps of the launches whose (M, Cin, taps) match g_xres_stamp_target, one record of
// 8 words per block (tools/xres_stamps.py): s_memtime at entry / first group staged / MFMA loop
// done / epilogue done, the summed staging cycles of every group, s_memrealtime at entry and end,
// and the hardware ids.  Never built into the product library.
__device__ int g_xres_stamp_target[3];
__device__ unsigned long long g_xres_stamp[1 << 20];
#endif

#ifndef TTS_LN_TAIL
#define TTS_LN_TAIL 1  // 0: timing-only probe builds -- fused post-LN tails load their rows but compute nothing
#endif
#ifndef TTS_LN_LOADPOL
#define TTS_LN_LOADPOL -1  // diagnostic builds: cache-policy bits of the tail's row loads (buffer loads)
#endif
#ifndef TTS_LN_FUSE_MINBLK
#define TTS_LN_FUSE_MINBLK 512  // GEMM blocks from which a launch applies its post-LN itself (same-box A/B: 0 slower at batch 8)
#endif
#ifndef TTS_LN_RB
#define TTS_LN_RB 4    // rows per wave in flight in the fused post-LN tail (8 spills at three blocks per CU)
#endif
// The fused post-LN of a conv_xres launch (ConvParams::ln_cnt): rows [n0, min(n0 + BN, ylen)) of
// utterance b's output Y (all M channels, written by the tile's M blocks), one wave per row, eight
// rows in flight per wave; arithmetic of layernorm8_kernel / ln_linear1_kernel (ln_rows.h).
template <typename T, int BN>
__device__ inline void xres_tile_ln(const ConvParams& p, const T* Y, int b, int n0, int ylen, int wave, int lane) {
  if constexpr (BN > 128) {
    // 128-row pieces: at 256 rows the tail's loop below is not fully unrolled, and its
    // double buffer u[it & 1] went to scratch (144 B/lane)
    for (int h = 0; h < BN && n0 + h < ylen; h += 128) xres_tile_ln<T, 128>(p, Y, b, n0 + h, ylen, wave, lane);
    return;
  }
  const int nrow = min(BN, ylen - n0);
  const int C = p.M;
  constexpr int RB = TTS_LN_RB;  // rows per wave in flight and normalised together
  if (p.ln_lin_out) {    // LayerNorm + Linear(C -> 1): lane l owns channels l + 64 i
    int ch[8];
    bool on[8];
    ln_lanes64<8>(ch, on, C, lane);
    float gl[8], bl[8], wl[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      gl[i] = on[i] ? p.ln_g1[ch[i]] : 0.f;
      bl[i] = on[i] ? p.ln_b1[ch[i]] : 0.f;
      wl[i] = on[i] ? p.ln_lin_w[ch[i]] : 0.f;
    }
    float* out = p.ln_lin_out + (long long)b * p.y_rows + n0;
    for (int r0 = wave; r0 < nrow; r0 += 4 * RB) {
      float v[RB][8], o[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {  // unconditional loads at clamped rows / channels
        const T* x = Y + (long long)(n0 + min(r0 + 4 * k, nrow - 1)) * p.syr;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] = to_f32(x[min(ch[i], C - 1)]);
      }
#pragma unroll
      for (int k = 0; k < RB; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (!on[i]) v[k][i] = 0.f;
      ln_linear1_batch<T, RB, 8>(v, on, C, gl, bl, wl, p.ln_eps, p.ln_lin_b, o);
#pragma unroll
      for (int k = 0; k < RB; ++k)
        if (lane == 0 && r0 + 4 * k < nrow) out[r0 + 4 * k] = o[k];
    }
    return;
  }
  T* L = reinterpret_cast<T*>(p.ln_out) + (long long)b * p.syb;
  int ch[8];
  bool on[8];
  ln_lanes8(ch, on, C, lane);
  float g[2][8], bb[2][8];
  ln_params<8>(g, bb, ch, on, p.ln_g1, p.ln_b1, p.ln_g2, p.ln_b2);
  const int c0 = on[0] ? ch[0] : 0;  // lanes past C load a valid piece and discard it
  // the next RB rows' loads are in flight while the current RB rows are normalised (one memory
  // round trip for the tail instead of one per RB rows)
  uint4 u[2][RB];
  auto load = [&](uint4 (&d)[RB], int r0) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < RB; ++k)
      d[k] = *reinterpret_cast<const uint4*>(Y + (long long)(n0 + min(r0 + 4 * k, nrow - 1)) * p.syr + c0);
  };
  load(u[0], wave);
#pragma unroll
  for (int it = 0; it < (BN + 4 * RB - 1) / (4 * RB); ++it) {
    const int r0 = wave + it * 4 * RB;
    if (r0 >= nrow) break;  // wave-uniform
    if (it + 1 < (BN + 4 * RB - 1) / (4 * RB)) load(u[(it + 1) & 1], r0 + 4 * RB);
    float v[RB][8];
#pragma unroll
    for (int k = 0; k < RB; ++k) ln_unpack8<T>(on[0] ? u[it & 1][k] : uint4{0u, 0u, 0u, 0u}, v[k]);
#if TTS_LN_TAIL
    if (p.ln_g2) ln_batch<T, RB, 8, true>(v, on, C, g, bb, p.ln_eps);
    else ln_batch<T, RB, 8, false>(v, on, C, g, bb, p.ln_eps);
#endif
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if (on[0] && r0 + 4 * k < nrow) *reinterpret_cast<uint4*>(L + (long long)(n0 + r0 + 4 * k) * p.syr + c0) = ln_pack8<T>(v[k]);
  }
}

// XF: the group's X loads all in flight at once (one round trip instead of three), the weight
// ring primed after them so the registers fit at three blocks per CU.  Same values staged, same
// MFMA order: bit-identical.  Measured (same box, tools/ab_xres.sh): the stage 0-1 upsamplers
// 155.5 -> 145.9 us and 316.4 -> 298.2 us; the acoustic GEMMs +2 % (their MFMA loops then wait on
// the ring's first quads), so only the upsampler launches use it.
// DT > 0 (conv_xres "DMA" form, WM = 4, DT taps, 64-channel groups, no input activation): the X
// tile of channel group g + NB - 1 is copied global -> LDS by buffer_load ... lds while group g's
// MFMAs run (NB LDS buffers; no staging registers, no staging barriers besides one per group).
// Rows are 128 bytes with chunk c of row r at slot c ^ ((r >> 1) & 7) (the DMA's lane-linear LDS
// image: the swizzle goes on the source address; the B-fragment reads are conflict-free for every
// row base); rows outside the utterance read 0 through the descriptor's range.  The weight ring
// holds one quad per tap and is refilled with the next group's quads.  Same K order as the
// register-staged kernel at CG = 64 (the launcher uses CG = 64 for every launch of these layers):
// bit-identical to it.
#ifndef TTS_XDMA_NB
#define TTS_XDMA_NB 2  // LDS buffers of the DMA form (prefetch distance NB - 1 groups)
#endif
// DMA form geometry: LDS buffers (1-tap: 3, prefetch two groups ahead -- a group is a third of
// the MFMA work of a 3-tap one) and staged rows per buffer (multi-tap: a 32-row halo)
#ifndef TTS_XDMA_NB2
#define TTS_XDMA_NB2 2  // ... for the multi-tap 64-row tiles (NT = 2): small grids, one block per CU or less
#endif
#ifndef TTS_XDMA_RSL2
#define TTS_XDMA_RSL2 1  // weight ring depth (groups) of the multi-tap 64-row tiles
#endif
// (Build options for the multi-tap 64-row tiles, where the 128-row grid would leave CUs idle: the
// batch-8 decoder FFN down-projection, 336 blocks of 24 groups.  Prefetching three groups ahead
// with a two-group weight ring (NB2 = 4, RSL2 = 2; bit-identical) measured 37.5 -> 39 us per
// launch: the group round trips are not what bounds it.)
template <int DT, int NT = 4> constexpr int xdma_nb() { return DT == 1 ? 3 : NT == 2 ? TTS_XDMA_NB2 : TTS_XDMA_NB; }
template <int DT, int NT = 4> constexpr int xdma_rsl() { return DT == 1 ? 2 : NT == 2 ? TTS_XDMA_RSL2 : 1; }
template <int DT, int BN> constexpr int xdma_rows() { return BN + (DT > 1 ? 32 : 0); }
// one 16-byte-per-lane buffer load straight into LDS (lane i -> lds + 16 i), no VGPR destination
__device__ inline void lds_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

template <typename T, int NT, int WM, int OCC = TTS_XRES_OCC, bool XF = false, int DT = 0>
__global__ __launch_bounds__(256, OCC) void conv_xres_kernel(ConvParams p, int CG) {
  using MF = Mfma<T>;
  typedef typename MF::frag Frag;
  static_assert(sizeof(T) == 2, "16-bit dtypes only");
  static_assert(NT % 2 == 0 || TTS_XRES_EPI16, "fp32 staging goes in 64-row halves");
  static_assert(WM == 4 || WM == 2, "4 waves: 4 x 1 or 2 x 2");
  constexpr int WN = 4 / WM;
  constexpr int BM = 32 * WM;          // output channels per block
  constexpr int BN = 32 * NT * WN;     // output rows per block
  constexpr int OS = BM * 4 + 16;      // fp32 output staging row stride (bytes)
  constexpr int PPR = BM / 8;          // 8-channel pieces per staged row
  constexpr int NTHR = 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nh = p.nh;
  // (bx, by, bz): row tile, M block, utterance x head -- the grid's own, or decoded from the 1-D
  // XCD-ordered grid (ConvParams::xres_order)
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  int gx = gridDim.x, gy = gridDim.y;
  if (p.xres_order) {
    gx = (p.y_rows + BN - 1) / BN;
    gy = (p.M + BM - 1) / BM;
    const int total = gx * gy * p.B * nh;
    const int per = (total + 7) / 8;
    const int v = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (v >= total) return;  // padding blocks of the last XCD range (no tile, no counter)
    by = v % gy;
    const int r = v / gy;
    bx = r % gx;
    bz = r / gx;
  }
  const int b = bz / nh;
  const int hd = bz - b * nh;
  const int n0 = bx * BN;
  const int ylen = p.y_len ? min(p.y_len[b], p.y_rows) : p.y_rows;
  if (n0 >= ylen) return;
  const int xlen = p.x_len ? min(p.x_len[b], p.x_rows) : p.x_rows;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31;
  const int hh = lane >> 5;
  const int wm = wave % WM, wn = wave / WM;
#if TTS_XRES_STAMP
  const unsigned long long st0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long st1 = 0, ssum = 0;
#endif

  const T* X = reinterpret_cast<const T*>(p.x) + (long long)b * p.sxb + (long long)hd * p.sxh;
  // packed weights: [MB][taps][Cin/16][64][8]; a wave past M reads the last block (its
  // results are never stored)
  const int KST = p.Cin / 16;
  const int mb = min(by * WM + wm, (p.M + 31) / 32 - 1);
  // Weight quads stream through a bounds-checked buffer descriptor over this wave's block:
  // a reload past the group's last quad gets an out-of-range offset and fetches nothing, so
  // every ring slot is reloaded unconditionally (a branch around the reloads made the
  // waitcnt pass drain vmcnt to 0-2 every quad instead of keeping the ring's 8 younger
  // loads in flight).
  const int wbytes = __builtin_amdgcn_readfirstlane(p.taps * KST * 1024);
  const char* wblk = reinterpret_cast<const char*>(p.wpk) + (long long)mb * wbytes;
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wblk), 0, wbytes, 0x00020000);
  const int lofs = lane * 16;          // voffset: loop-invariant (the quad offset is soffset)
  const int R = BN + (p.taps - 1) * p.dil;
  const int RS = CG * 2 + 16;
  const int VPR = CG / 8;
  const int NQ = CG / 64;              // weight quads (4 k-steps of 16) per tap
  const int lnq = __builtin_ctz(NQ);
  const int QT = p.taps * NQ;          // quads per channel group
  const int x_start = n0 - p.pad;
  const int xlast = xlen > 0 ? xlen - 1 : 0;
  const int dstep = p.dil * RS;        // LDS bytes per tap
  const char* xl = smem + (wn * 32 * NT + l31) * RS + hh * 16;

  f32x16 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x16{};

  // quad qq of channel group g0: 4 contiguous 1 KiB fragments (nothing past the group's QT)
#define TTS_LOADQ(A_, QQ_)                                                                \
  do {                                                                                    \
    const int qq_ = (QQ_);                                                                \
    const int o_ = ((qq_ >> lnq) * KST + g0 / 16 + (qq_ & (NQ - 1)) * 4) * 1024 +         \
                   (((QT - 1 - qq_) >> 31) & 0x40000000); /* uniform; out of range past QT */ \
    _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_) A_[j_] =                             \
        __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lofs + j_ * 1024, o_, 0)); \
    __builtin_amdgcn_sched_barrier(0); /* issue here: the scheduler would sink reloads */  \
  } while (0)
#define TTS_MMAQ(A_, QQ_)                                                                 \
  do {                                                                                    \
    const int qq_ = (QQ_);                                                                \
    const char* bq_ = xl + (qq_ >> lnq) * dstep + (qq_ & (NQ - 1)) * 128;                 \
    _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_) {                                    \
      Frag bf_[NT];                                                                       \
      _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_)                                \
        bf_[nt_] = *reinterpret_cast<const Frag*>(bq_ + nt_ * 32 * RS + j_ * 32);         \
      _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_)                                \
        acc[nt_] = MF::mma(A_[j_], bf_[nt_], acc[nt_]);                                   \
    }                                                                                     \
  } while (0)

  if constexpr (DT > 0) {
    static_assert(WM == 4 && DT <= 3, "DMA form: 128-channel blocks, <= 3 taps (one ring slot per tap)");
    constexpr int RD = xdma_rows<DT, BN>();  // staged rows per group: the tile + a halo of (taps - 1) * dil <= 32
    constexpr int NPW = RD / 32;        // 1 KiB DMA pieces (8 rows) per wave per group
    constexpr int BUFB = RD * 128;      // bytes per LDS buffer
    constexpr int NB = xdma_nb<DT, NT>();
    constexpr int RSL = xdma_rsl<DT, NT>();  // weight ring depth in groups (one quad per tap and group)
    static_assert(RSL <= NB - 1, "the ring may not run ahead of the staged groups");
    constexpr int Q = 4 * DT;           // weight loads per group
    static_assert(NB >= 2 && NB <= 4, "2 to 4 LDS buffers");
    static_assert((NB - 2) * (RD / 32) + (NB - 1) * 4 * DT <= 63, "vmcnt wait counts fit the 6-bit field");
    // outstanding memory operations younger than group g's pieces at its wait: the DMAs of groups
    // g + 1 .. g + NB - 2 and the ring loads issued after it -- RSL groups' at g = 0, then
    // min(RSL + g, NB - 1) groups' (the smaller count of the two cases: waiting for more is safe)
    constexpr int W0 = (NB - 2) * NPW + RSL * Q;
    constexpr int W1 = (NB - 2) * NPW + (RSL + 1 < NB - 1 ? RSL + 1 : NB - 1) * Q;
    const int G = p.Cin / 64;
    // rows [0, xlen) of the utterance; anything else (rows before 0: negative offsets) reads 0
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(X), 0, xlen * p.sxr * (int)sizeof(T), 0x00020000);
    int voff[NPW];  // this lane's source bytes of its pieces for group 0 (group g: + 128 g)
#pragma unroll
    for (int q = 0; q < NPW; ++q) {
      const int row = 8 * (wave * NPW + q) + (lane >> 3);
      voff[q] = ((x_start + row) * p.sxr + 8 * ((lane & 7) ^ ((row >> 1) & 7))) * (int)sizeof(T);
    }
    // group g's X tile -> buffer g % NB; past the last group the pieces read nothing (the count of
    // outstanding memory operations stays the same every group)
    auto dma = [&](int g) __attribute__((always_inline)) {
      char* dst = smem + (g % NB) * BUFB + wave * NPW * 1024;
      const int go = g < G ? g * 64 * (int)sizeof(T) : 0x40000000;
#pragma unroll
      for (int q = 0; q < NPW; ++q)
        lds_dma16(xrs, dst + q * 1024, voff[q] + go);
      __builtin_amdgcn_sched_barrier(0);
    };
    // weight quad of (group g, tap t): k-steps t * KST + 4 g .. + 3; nothing past the last group
    auto loadq = [&](Frag (&a)[4], int g, int t) __attribute__((always_inline)) {
      const int o = (t * KST + 4 * g) * 1024 + (g < G ? 0 : 0x40000000);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a[j] = __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lofs + j * 1024, o, 0));
      __builtin_amdgcn_sched_barrier(0);
    };
    // B-fragment byte offsets of tap t, k-step j in a buffer (tile nt: + nt * 32 rows)
    int boff[DT][4];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int r = l31 + t * p.dil;
#pragma unroll
      for (int j = 0; j < 4; ++j) boff[t][j] = r * 128 + (((2 * j + hh) ^ ((r >> 1) & 7)) << 4);
    }
    Frag ra[RSL][DT][4];
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) dma(i);
#pragma unroll
    for (int s = 0; s < RSL; ++s)
#pragma unroll
      for (int t = 0; t < DT; ++t) loadq(ra[s][t], s, t);
    // one group: its pieces have landed (vmcnt: all but the youngest), then every wave's; the
    // next DMA goes into the buffer group g - 1 read (every wave is past it); the ring slot is
    // refilled with group g + RSL's quads
    auto group = [&](int g, Frag (&rs)[DT][4]) __attribute__((always_inline)) {
      if (g == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W0) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W1) : "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#if TTS_XRES_STAMP
      if (g == 0) st1 = __builtin_amdgcn_s_memtime();
#endif
      dma(g + NB - 1);
      const char* buf = smem + (g % NB) * BUFB;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          Frag bf[NT];
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) bf[nt] = *reinterpret_cast<const Frag*>(buf + boff[t][j] + nt * 32 * 128);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[nt] = MF::mma(rs[t][j], bf[nt], acc[nt]);
        }
        loadq(rs[t], g + RSL, t);
      }
    };
    for (int g = 0; g < G; g += RSL) {
      group(g, ra[0]);
      if constexpr (RSL > 1)
        if (g + 1 < G) group(g + 1, ra[1]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing pieces land before the epilogue reuses LDS
  } else {
  // X staging: thread owns 16-byte column cc of the group and rows r0, r0 + rstep, ...
  // (CG is a power of two: no per-vector division)
  const int lvpr = __builtin_ctz(VPR);
  const int cc = tid & (VPR - 1);
  const int r0 = tid >> lvpr;
  const int rstep = NTHR >> lvpr;
  // quad ring, 3 deep: quad q's weights are issued while quads q-2 and q-1 compute
  for (int g0 = 0; g0 < p.Cin; g0 += CG) {
    Frag a0[4], a1[4], a2[4];
#if TTS_XRES_STAMP
    const unsigned long long sts = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (!XF) {
      // first quads of the group in flight before the X loads (in-order vmcnt: they
      // complete first and are ready when the MFMA loop starts)
      TTS_LOADQ(a0, 0);
      TTS_LOADQ(a1, 1);
      TTS_LOADQ(a2, 2);
    }
    if (g0) __syncthreads();  // previous group's B reads are done
    const T* xg = X + g0 + cc * 8;
    constexpr int SU = XF ? XRES_SU_XF : XRES_SU;
    for (int rb = r0; rb < R; rb += SU * rstep) {
      uint4 r[SU];
#pragma unroll
      for (int i = 0; i < SU; ++i) {
        const int xr = min(max(x_start + min(rb + i * rstep, R - 1), 0), xlast);
        r[i] = *reinterpret_cast<const uint4*>(xg + xr * p.sxr);
      }
#pragma unroll
      for (int i = 0; i < SU; ++i) {
        const int rr = rb + i * rstep;
        const int xr = x_start + rr;
        // consumed unconditionally: a load consumed only under the row mask stays "pending"
        // for the waitcnt pass, whose WAW check then drains vmcnt at the MFMA loop head
        const uint4 v = act16<T>(r[i], xr >= 0 && xr < xlen, p.in_slope);
        if (rr < R) *reinterpret_cast<uint4*>(smem + rr * RS + cc * 16) = v;
      }
    }
    if constexpr (XF) {
      // the group's X rows were all in flight at once (one round trip); the ring's first quads
      // follow, issued after the X registers are written out
      TTS_LOADQ(a0, 0);
      TTS_LOADQ(a1, 1);
      TTS_LOADQ(a2, 2);
    }
    __syncthreads();
#if TTS_XRES_STAMP
    {
      const unsigned long long ste = __builtin_amdgcn_s_memtime();
      ssum += ste - sts;
      if (g0 == 0) st1 = ste;
    }
#endif
    int q = 0;
    for (; q + 3 <= QT; q += 3) {  // straight-line body
      TTS_MMAQ(a0, q);
      TTS_LOADQ(a0, q + 3);
      TTS_MMAQ(a1, q + 1);
      TTS_LOADQ(a1, q + 4);
      TTS_MMAQ(a2, q + 2);
      TTS_LOADQ(a2, q + 5);
    }
    if (q < QT) TTS_MMAQ(a0, q);
    if (q + 1 < QT) TTS_MMAQ(a1, q + 1);
  }
  }  // register-staged form
#undef TTS_LOADQ
#undef TTS_MMAQ

#if TTS_XRES_STAMP
  const unsigned long long st2 = __builtin_amdgcn_s_memtime();
#endif
  // ---- epilogue through LDS: fragments -> fp32 rows -> 8-channel row pieces ----
  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.syb + (long long)hd * p.syh;
  const T* R1 = p.r1 ? reinterpret_cast<const T*>(p.r1) + (long long)b * p.srb + (long long)hd * p.srh : nullptr;
  const T* R2 = p.r2 ? reinterpret_cast<const T*>(p.r2) + (long long)b * p.srb + (long long)hd * p.srh : nullptr;
  const int tlen = p.up_len ? min(p.up_len[b], (p.y_rows - 1) * p.up_s) : 0;
  const int cl = tid % PPR;                   // 8-channel piece of the block's BM channels
  const int m8 = by * BM + cl * 8;
  const bool mok = m8 < p.M;
  int q = 0, col = m8;
  if (p.up_s) { q = m8 / p.up_cout; col = m8 - q * p.up_cout; }
#if TTS_XRES_EPI16
  // Bias, alpha and activation applied on the fragments, rounded to T once and staged in LDS
  // as T (half the bytes of fp32; the whole tile in one round: one barrier pair).  The row
  // pass moves 16-byte pieces out; launches with residuals / an output scale add them in
  // fp32 there and round again (the pair kernels' epilogue order).
  constexpr int OS16 = BM * 2 + 16;           // staged row stride (bytes)
  constexpr int NIT = BN * PPR / NTHR;        // row pieces per thread
  static_assert(BN * PPR % NTHR == 0 && NTHR % PPR == 0, "row pass");
  // bias before the residual loads: vmcnt retires in order, so the staging's wait for the
  // bias leaves the residual loads in flight
  f32x4 bl[4];
  {  // channels past M or a null bias read 0 (descriptor range), no branch
    const auto brsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias ? p.bias : reinterpret_cast<const float*>(Y)),
                                                         0, p.bias ? p.M * 4 : 0, 0x00020000);
#pragma unroll
    for (int g = 0; g < 4; ++g)
      bl[g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            brsrc, (by * BM + wm * 32 + 8 * g + 4 * hh) * 4, 0, 0));
  }
  // first-residual rows in flight before the staging barriers, through a descriptor with no
  // records when there is no residual: the loads are unconditional (a load under `if (R1)`
  // made the waitcnt pass wait for each one right after issuing it) and fetch nothing then
  uint4 res1[NIT];
  {
    const auto r1rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(R1 ? R1 : Y), 0, R1 ? 0x7fffffff : 0,
                                                          0x00020000);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rl = tid / PPR + it * (NTHR / PPR);
      int row = min(n0 + rl, ylen - 1);
      if (p.up_s) row = min(max(row * p.up_s + q - p.up_p, 0), max(tlen - 1, 0));
      const int off = (int)(((long long)row * p.srr + (mok ? col : 0)) * (long long)sizeof(T));
      res1[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r1rsrc, off, 0, 0));
    }
  }
  __syncthreads();  // X tile no longer read
  // the activation is dispatched once for the whole tile: inside the element loop its runtime
  // switch split the staging into a basic block per element and kind (same arithmetic either way)
  auto stage_acc = [&](auto act_c) __attribute__((always_inline)) {
    constexpr int ACT = decltype(act_c)::value;
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // alpha always applied (x * 1.0f is exact): no per-group branch in the staging
        const f32x4 v0 = f32x4{acc[j][4 * g + 0], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]} + bl[g];
        f32x4 v = v0 * p.alpha;
        if constexpr (ACT != ACT_NONE) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = apply_act(v[i], ACT, p.out_slope);
        }
        *reinterpret_cast<uint2*>(smem + (wn * 32 * NT + j * 32 + l31) * OS16 + (wm * 32 + 8 * g + 4 * hh) * 2) =
            pack4<T>(v);
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
  const bool plain = !R1 && !R2 && p.out_scale == 1.0f;
  // LayerNorm in this launch (the launcher checked the shape; never the 96-row tiles, small grids
  // only, where the separate launch is faster -- and their non-inlined tail put p in scratch)
  const bool lnf = NT != 3 && p.ln_cnt != nullptr;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int rl = tid / PPR + it * (NTHR / PPR);
    const int n = n0 + rl;
    if (n >= ylen || !mok) continue;
    int row = n;
    if (p.up_s) {
      row = n * p.up_s + q - p.up_p;
      if (row < 0 || row >= tlen) continue;
    }
    uint4 y = *reinterpret_cast<const uint4*>(smem + rl * OS16 + cl * 16);
    if (!plain) {
      f32x4 v0, v1;
      ld8<T>(reinterpret_cast<const T*>(&y), v0, v1);
      if (R1) { f32x4 a, c; ld8<T>(reinterpret_cast<const T*>(&res1[it]), a, c); v0 += a; v1 += c; }
      if (R2) { f32x4 a, c; ld8<T>(R2 + (long long)row * p.srr + col, a, c); v0 += a; v1 += c; }
      if (p.out_scale != 1.0f) { v0 *= p.out_scale; v1 *= p.out_scale; }
      y = pack8<T>(v0, v1);
    }
    const int yo = (int)(((long long)row * p.syr + col) * (long long)sizeof(T));
    if (lnf) store16<16>(Y, yo, y);  // write-through: the tile's last block reads it (ln_rows.h)
    else store16<TTS_XRES_STORE>(Y, yo, y);
  }
  if (lnf) {
    // the row tile's last-arriving M block normalises rows [n0, ylen) of it over all M channels
    if (!ln_tile_last(p.ln_cnt + bz * gx + bx, gy, reinterpret_cast<int*>(smem)))
      return;
    xres_tile_ln<T, BN>(p, Y, b, n0, ylen, wave, lane);
  }
#if TTS_XRES_STAMP
  if (p.M == g_xres_stamp_target[0] && p.Cin == g_xres_stamp_target[1] && p.taps == g_xres_stamp_target[2]) {
    __syncthreads();  // every wave's epilogue issued
    if (tid == 0) {
      const unsigned long long blk = blockIdx.x + (unsigned long long)gridDim.x * (blockIdx.y + (unsigned long long)gridDim.y * blockIdx.z);
      if (blk < (1u << 17)) {
        unsigned long long* r = g_xres_stamp + blk * 8;
        r[0] = st0; r[1] = st1; r[2] = st2; r[3] = __builtin_amdgcn_s_memtime();
        r[4] = ssum; r[5] = rt0; r[6] = __builtin_amdgcn_s_memrealtime();
        r[7] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)) << 32) |
               (unsigned)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
      }
    }
  }
#endif
#else
  // staged half h holds rows wn*32*NT + 64h + [0, 64) of every N-wave, compacted to
  // staged row wn*64 + r; the row pass maps staged row sr back to its output row
  auto out_row = [&](int half, int sr) { return n0 + (sr >> 6) * (32 * NT) + half * XRES_HR + (sr & 63); };
  f32x4 bias0 = {}, bias1 = {};
  if (p.bias && mok) {
    bias0 = *reinterpret_cast<const f32x4*>(p.bias + m8);
    bias1 = *reinterpret_cast<const f32x4*>(p.bias + m8 + 4);
  }
  // every item's first-residual rows in flight before the staging barriers (the weight
  // ring is dead here, so these registers do not raise the kernel's peak; prefetching r2
  // as well would spill)
  constexpr int NIT = XRES_HR * WN * PPR / NTHR;
  uint4 res1[NT / 2][NIT];
#pragma unroll
  for (int half = 0; half < NT / 2; ++half)
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int n = out_row(half, tid / PPR + it * (NTHR / PPR));
      int row = min(n, ylen - 1);
      if (p.up_s) row = min(max(row * p.up_s + q - p.up_p, 0), max(tlen - 1, 0));
      if (R1) res1[half][it] = *reinterpret_cast<const uint4*>(R1 + (long long)row * p.srr + (mok ? col : 0));
    }
#pragma unroll
  for (int half = 0; half < NT / 2; ++half) {
    __syncthreads();  // X tile / previous half no longer read
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& a = acc[2 * half + k];
        *reinterpret_cast<f32x4*>(smem + (wn * 64 + k * 32 + l31) * OS + (wm * 32 + 8 * g + 4 * hh) * 4) =
            f32x4{a[4 * g + 0], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]};
      }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rl = tid / PPR + it * (NTHR / PPR);
      const int n = out_row(half, rl);
      if (n >= ylen || !mok) continue;
      int row = n;
      if (p.up_s) {
        row = n * p.up_s + q - p.up_p;
        if (row < 0 || row >= tlen) continue;
      }
      f32x4 v0 = *reinterpret_cast<const f32x4*>(smem + rl * OS + cl * 32);
      f32x4 v1 = *reinterpret_cast<const f32x4*>(smem + rl * OS + cl * 32 + 16);
      v0 += bias0; v1 += bias1;
      if (p.alpha != 1.0f) { v0 *= p.alpha; v1 *= p.alpha; }
      if (p.act_out) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v0[i] = apply_act(v0[i], p.act_out, p.out_slope);
          v1[i] = apply_act(v1[i], p.act_out, p.out_slope);
        }
      }
      if (R1) { f32x4 a, c; ld8<T>(reinterpret_cast<const T*>(&res1[half][it]), a, c); v0 += a; v1 += c; }
      if (R2) { f32x4 a, c; ld8<T>(R2 + (long long)row * p.srr + col, a, c); v0 += a; v1 += c; }
      if (p.out_scale != 1.0f) { v0 *= p.out_scale; v1 *= p.out_scale; }
      {
        const uint4 e8 = pack8<T>(v0, v1);
        store16<TTS_XRES_STORE>(Y, (int)(((long long)row * p.syr + col) * (long long)sizeof(T)), e8);
      }
    }
  }
#endif
}

constexpr int XRES_LDS_MAX = (160 / TTS_XRES_OCC - 1) * 1024;  // TTS_XRES_OCC blocks per CU (53 KB at 3)
#ifndef TTS_XRES_BIGCG_MIN
#define TTS_XRES_BIGCG_MIN 0           // > 0: Cin from which conv_xres stages big channel groups, one block per CU
                                       // (1024 measured slower: C3 acoustic 5.14 -> 5.51 ms, C5 acoustic +40 us)
#endif
constexpr int XRES_LDS_BIG = 159 * 1024;

// channel group for the X-resident kernel: largest power-of-two CG | Cin, CG >= 64, tile within
// XRES_LDS_MAX; 0 = not eligible
// layers the DMA form of conv_xres serves (2- and 3-tap convs: the acoustic FFN convs, the vocoder's
// stage 0-1 upsamplers); every launch of them, whichever kernel runs it, uses 64-channel groups
// (one K order: bit-identical across kernels, batch sizes and tile shapes)
#ifndef TTS_XRES_DMA
#define TTS_XRES_DMA 1
#endif
static bool xres_dma_layer(const ConvParams& p) {
  return TTS_XRES_DMA && sw(SW_XRES_DMA) != 0 && (p.taps == 2 || p.taps == 3) && p.nh == 1 && p.Cin % 64 == 0 &&
         (p.taps - 1) * p.dil <= 32 && (long long)p.x_rows * p.sxr * 2 < (1LL << 31);
}
// ... of which the DMA form runs the ones with no input activation (the DMA copies X as it is)
static int xres_dma_taps(const ConvParams& p) {
  return xres_dma_layer(p) && p.in_slope == 1.0f && sw(SW_XRES_DMA) != 2 ? p.taps : 0;
}

// ... and the 1-tap convs (the acoustic projections: Q/K/V, attention output, pointwise convs) with
// no input activation: with one tap the K order is the k-steps' own for every channel group, so
// the DMA form is bit-identical to the register-staged kernel at the group that one would use
// (TTS_XRES_DMA=3: multi-tap layers only)
static bool xres_dma1(const ConvParams& p) {
  return TTS_XRES_DMA && sw(SW_XRES_DMA) != 0 && sw(SW_XRES_DMA) != 2 && sw(SW_XRES_DMA) != 3 && p.taps == 1 &&
         p.nh == 1 && p.Cin % 64 == 0 && p.in_slope == 1.0f && p.sxr % 8 == 0 && p.sxb % 8 == 0 &&
         (long long)p.x_rows * p.sxr * 2 < (1LL << 31);
}

static int xres_group(const ConvParams& p, int BN, int lds_max = XRES_LDS_MAX) {
  if (!p.wpk || p.M < 64 || p.Cin % 64 || p.M % 8 || p.nh != 1) return 0;
  if (xres_dma_layer(p)) return 64;
  if (p.syr % 8 || p.syb % 8 || ((p.r1 || p.r2) && (p.srr % 8 || p.srb % 8))) return 0;
  if (p.up_s && p.up_cout % 8) return 0;
  const int R = BN + (p.taps - 1) * p.dil;
  for (int cg = 2048; cg >= 64; cg /= 2) {  // powers of two (division-free staging)
    if (cg > p.Cin || p.Cin % cg) continue;
    if ((size_t)R * (cg * 2 + 16) <= (size_t)lds_max) return cg;
  }
  return 0;
}


// 128-channel blocks (4 x 1 waves, BN = 128) for M >= 128; 64-channel blocks (2 x 2 waves,
// BN = 256) for M = 64 (the last upsampler)
static int xres_wm(const ConvParams& p) { return p.M >= 128 ? 4 : 2; }

#ifndef TTS_XRES_NARROW_KMIN
#define TTS_XRES_NARROW_KMIN 0         // > 0: also below 2x the block limit when Cin*taps >= this (4096 / 1024 measured neutral on C3/C5)
#endif
#ifndef TTS_XRES_NARROW_MAXBLK
#define TTS_XRES_NARROW_MAXBLK 256     // 0 disables; 512 slower for C3 (encoder at batch 32); 192 / 384 within noise
#endif
// Narrow 64 x 64 tiles (2 x 2 waves, one 32 x 32 MFMA tile each) for launches whose 128-channel
// grid would leave the chip under-filled: the small-batch acoustic passes (streaming: batch 8;
// the encoder's 144-row utterances), where an M = 384 projection over K = 4608 made 54-168
// blocks for 256 CUs.  Same channel group (K order) as the wide tiles, so a row's result does
// not depend on the choice (bit-identical; tests/test_acoustic_gpu.py).  TTS_XRES_NARROW=0/1
// forces it off / on where eligible (A/B runs and tests).
static bool xres_narrow(const ConvParams& p, int nt) {
  if (p.M % 64 || !TTS_XRES_EPI16) return false;
  if (sw(SW_XRES_NARROW) >= 0) return sw(SW_XRES_NARROW) != 0;
  const long long blocks = (long long)((p.y_rows + 32 * nt - 1) / (32 * nt)) * ((p.M + 127) / 128) * p.B * p.nh;
  if (blocks < TTS_XRES_NARROW_MAXBLK) return true;
  // long-K launches (the encoder's FFN down-projection, K = 4608) up to twice that many blocks
  return TTS_XRES_NARROW_KMIN > 0 && p.Cin * p.taps >= TTS_XRES_NARROW_KMIN && blocks < 2 * TTS_XRES_NARROW_MAXBLK;
}

#ifndef TTS_XRES_SMALL_TILES
#define TTS_XRES_SMALL_TILES 1
#endif
#ifndef TTS_XRES_NT2_MAXBLK
#define TTS_XRES_NT2_MAXBLK 400        // 0 disables the small-grid 64-row rule below
#endif
#ifndef TTS_XRES_NT3
#define TTS_XRES_NT3 1                 // 96-row tiles where they balance a small grid better (below)
#endif
// 64-row tiles (NT = 2) where 128-row tiles would leave much of the last tile of every
// utterance empty (the encoder's 144 rows: 3 x 64 = 192 rows of work instead of 2 x 128)
static int xres_nt_auto(const ConvParams& p);
// nt3: the launch has a 96-row (NT = 3) instance (the DMA forms of 1 and 3 taps)
static int xres_nt(const ConvParams& p, int wm, bool nt3 = false) {
  const int force = sw(SW_XRES_NT);  // 2 / 3 / 4 force a tile height (tests), else automatic
  if (wm != 4) return 4;
  if (force == 2 || force == 4) return force;
  if (force == 3 && nt3) return 3;
  if (!TTS_XRES_SMALL_TILES) return 4;
  const int nt = xres_nt_auto(p);
  // 96-row tiles for a grid whose blocks all fit on the chip at once but fill it unevenly: the
  // busiest CU holds ceil(blocks / 256) tiles, so the launch takes ~ceil(blocks / 256) * NT row
  // units.  The batch-8 decoder's 384-channel layers (FFN down-projection, output projection,
  // second pointwise conv; 6,912 rows): 324 blocks of 64 rows put two on 68 CUs (cost 4), 216
  // of 96 rows one per CU (cost 3).  Taken only when strictly cheaper and the 96-row grid is at
  // most one block per CU: on bigger grids (batch 32) the smaller tiles' extra weight stream per
  // row cost more than the balance gained (profiles/r05s_ab_nt3.txt).  Same channel group, so
  // the same bits.
  if (nt3 && TTS_XRES_NT3) {
    const long long mb = (long long)((p.M + 127) / 128) * p.B * p.nh;
    auto blocks = [&](int n) { return ((p.y_rows + 32 * n - 1) / (32 * n)) * mb; };
    auto cost = [&](int n) { return (blocks(n) + 255) / 256 * n; };
    if (blocks(3) <= 256 && cost(3) < cost(nt)) return 3;
  }
  return nt;
}
static int xres_nt_auto(const ConvParams& p) {
  const int r4 = (p.y_rows + 127) / 128 * 128, r2 = (p.y_rows + 63) / 64 * 64;
  if (8 * r2 <= 7 * r4) return 2;
  // small grids (the batch-8 decoder): 64-row tiles where the 128-row grid fills under ~1.5
  // blocks per CU but the 64-row one fills every CU, ahead of both the 128-row tiles and the
  // narrow 64 x 64 tiles.  Measured per launch at batch 8 (same box): the FFN down-projection
  // (M = 384, K = 4608) 63 us narrow / 57 us 128-row / 48.5 us 64-row; the pointwise conv
  // (M = 768) 14 -> 12 us; the FFN up-projection (672 blocks) and Q/K/V (504) are faster at 128
  // rows, hence the bound.  Same channel group, so the same bits.
  const long long mb = (long long)((p.M + 127) / 128) * p.B * p.nh;
  const long long b4 = (long long)(r4 / 128) * mb, b2 = (long long)(r2 / 64) * mb;
  if (b4 < TTS_XRES_NT2_MAXBLK && b2 >= 256) return 2;
  return 4;
}

// whether a conv_xres launch of row-tile height BN applies p's LayerNorm itself (ln_cnt given,
// rows of M <= 512 channels in whole 16-byte pieces, one counter per row tile)
static bool xres_ln_ok(const ConvParams& p, int BN) {
  if (!p.ln_cnt || !(p.ln_out || p.ln_lin_out) || !TTS_XRES_EPI16 || p.up_s || p.nh != 1) return false;
  if (sw(SW_LN_FUSE) > 1 && sw(SW_LN_FUSE) != 2 && sw(SW_LN_FUSE) != 7 && sw(SW_LN_FUSE) != (p.ln_lin_out ? 6 : 5))
    return false;  // (bisection: 2 = conv_xres only, 5 / 6 = its LayerNorm / LayerNorm + Linear launches only)
  // small grids: every block runs at once, so the tile's LayerNorm tail is on the critical path
  // and costs more than the separate launch (the result is the same either way)
  if (sw(SW_LN_FUSE) != 7 && (long long)((p.y_rows + BN - 1) / BN) * p.B * ((p.M + 127) / 128) < TTS_LN_FUSE_MINBLK)
    return false;  // (TTS_LN_FUSE=7: every eligible launch, tests)
  if (p.M > 512 || p.M % 8 || (p.ln_lin_out && p.syb != (long long)p.y_rows * p.syr)) return false;
  return (long long)((p.y_rows + BN - 1) / BN) * p.B <= p.ln_cnt_n;
}

#ifndef TTS_XRES_ORDER_DEFAULT
#define TTS_XRES_ORDER_DEFAULT 2
#endif

template <typename T, int WM, int NT = 4, int OCC = TTS_XRES_OCC, bool XF = false, int DT = 0>
static hipError_t launch_xres_wm(const ConvParams& p, int cg, hipStream_t s, bool* ln_done) {
  constexpr int BM = 32 * WM, BN = 32 * NT * (4 / WM);
  const size_t xt = DT ? (size_t)xdma_nb<DT, NT>() * xdma_rows<DT, BN>() * 128 : (size_t)(BN + (p.taps - 1) * p.dil) * (cg * 2 + 16);
  const size_t lds = std::max(xt, TTS_XRES_EPI16 ? (size_t)BN * (BM * 2 + 16) : (size_t)XRES_HR * (4 / WM) * (BM * 4 + 16));
  dim3 grid((p.y_rows + BN - 1) / BN, (p.M + BM - 1) / BM, p.B * p.nh);
  ConvParams q = p;
  // XCD-ordered 1-D grid (TTS_XRES_ORDER=1: the multi-tap DMA launches, the decoder FFN convs and
  // the stage 0-1 upsamplers; =2, the default: every conv_xres launch; 0: the 3-D grid).  Same-box
  // A/B (profiles/r04e_ab_xres_order.txt): batch-32 acoustic 5.83 -> 5.67 ms, C5 3.52 -> 3.43 ms,
  // C2 unchanged; bit-identical (tests/test_acoustic_gpu.py).
  const int ord = sw(SW_XRES_ORDER) < 0 ? TTS_XRES_ORDER_DEFAULT : sw(SW_XRES_ORDER);
  q.xres_order = (ord == 2 || (ord == 1 && DT > 1)) ? 1 : 0;
  if (q.xres_order) grid = dim3(8 * ((grid.x * grid.y * grid.z + 7) / 8), 1, 1);
  if (NT == 3 || !xres_ln_ok(q, BN)) q.ln_cnt = nullptr;  // the kernel's LayerNorm switch
  if (ln_done) *ln_done = q.ln_cnt != nullptr;
  hipLaunchKernelGGL((conv_xres_kernel<T, NT, WM, OCC, XF, DT>), grid, dim3(256), lds, s, q, cg);
  return hipGetLastError();
}

template <typename T>
static bool launch_xres(const ConvParams& p, hipStream_t s, hipError_t* err, bool* ln_done) {
  const int wm = xres_wm(p);
  const bool big = TTS_XRES_BIGCG_MIN > 0 && wm == 4 && p.Cin >= TTS_XRES_BIGCG_MIN;
  const bool dma3 = xres_dma_taps(p) == 3, dma1 = xres_dma_taps(p) != 2 && !dma3 && xres_dma1(p);
  // (the 96-row option never displaces the narrow tiles: they are decided at the other heights)
  const int nt0 = xres_nt(p, wm);
  const bool narrow = xres_narrow(p, nt0);
  const int nt = narrow ? nt0 : xres_nt(p, wm, !big && (dma3 || dma1));
  // channel group sized for 128-row tiles whatever the tile height: the group fixes the K
  // order of the accumulation, so a row's result does not depend on the tiling (streamed
  // chunks stay bit-identical to the full pass)
  // long-K convs (Cin >= TTS_XRES_BIGCG_MIN: the FFN down-projections) stage 4x larger channel
  // groups at one block per CU: a quarter of the single-buffered group stagings, each a full
  // HBM/L2 round trip.  The choice depends on the layer shape only, so the K order is still
  // the same for every batch size and tile shape.
  const int cg = xres_group(p, 32 * 4 * (4 / wm), big ? XRES_LDS_BIG : XRES_LDS_MAX);
  if (!cg) return false;
  if (wm == 2)  // (the postnet's 80-channel output conv)
    *err = launch_xres_wm<T, 2>(p, cg, s, ln_done);
  else if (big)
    *err = narrow    ? launch_xres_wm<T, 2, 1, 1>(p, cg, s, ln_done)
           : nt == 2          ? launch_xres_wm<T, 4, 2, 1>(p, cg, s, ln_done)
                              : launch_xres_wm<T, 4, 4, 1>(p, cg, s, ln_done);
  else if (narrow)
    *err = launch_xres_wm<T, 2, 1>(p, cg, s, ln_done);
  else if (dma3)  // (TTS_XRES_DMA=2: the same layers, K order and bits, register-staged)
    *err = nt == 2   ? launch_xres_wm<T, 4, 2, TTS_XRES_OCC, false, 3>(p, cg, s, ln_done)
           : nt == 3 ? launch_xres_wm<T, 4, 3, TTS_XRES_OCC, false, 3>(p, cg, s, ln_done)
                     : launch_xres_wm<T, 4, 4, TTS_XRES_OCC, false, 3>(p, cg, s, ln_done);
  else if (xres_dma_taps(p) == 2)  // the polyphase upsamplers (k = 2 s): 2 taps
    *err = nt == 2 ? launch_xres_wm<T, 4, 2, TTS_XRES_OCC, false, 2>(p, cg, s, ln_done)
                   : launch_xres_wm<T, 4, 4, TTS_XRES_OCC, false, 2>(p, cg, s, ln_done);
  else if (xres_dma1(p))
    *err = nt == 2   ? launch_xres_wm<T, 4, 2, TTS_XRES_OCC, false, 1>(p, cg, s, ln_done)
           : nt == 3 ? launch_xres_wm<T, 4, 3, TTS_XRES_OCC, false, 1>(p, cg, s, ln_done)
                     : launch_xres_wm<T, 4, 4, TTS_XRES_OCC, false, 1>(p, cg, s, ln_done);
  else if (TTS_XRES_UPFIRST && p.up_s)
    *err = nt == 2 ? launch_xres_wm<T, 4, 2, TTS_XRES_OCC, true>(p, cg, s, ln_done)
                   : launch_xres_wm<T, 4, 4, TTS_XRES_OCC, true>(p, cg, s, ln_done);
  else
    *err = nt == 2 ? launch_xres_wm<T, 4, 2>(p, cg, s, ln_done) : launch_xres_wm<T, 4>(p, cg, s, ln_done);
  return true;
}

template <typename T, int MT, int NT, int WM, int WN, int CK>
static hipError_t launch_cfg(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 32 * MT * WM;
  constexpr int BN = 32 * NT * WN;
  constexpr int LDSR = CK + 16 / (int)sizeof(T);
  const int R = BN + (p.taps - 1) * p.dil;
  const int nchunks = (p.Cin + CK - 1) / CK;
  const size_t lds = (size_t)R * LDSR * sizeof(T) * (nchunks > 1 ? 2 : 1);
  dim3 grid((p.y_rows + BN - 1) / BN, (p.M + BM - 1) / BM, p.B * p.nh * std::max(p.kslices, 1));
  hipLaunchKernelGGL((conv_gemm_kernel<T, MT, NT, WM, WN, CK>), grid, dim3(64 * WM * WN), lds, s, p);
  return hipGetLastError();
}

#ifndef TTS_F32_SK_MINM
#define TTS_F32_SK_MINM 64  // fp32 split-K only above this many output channels (A/B builds: 32 -- C1's stage-2 convs)
#endif
#ifndef TTS_F32_SLICE_CH
#define TTS_F32_SLICE_CH 32  // fp32 split-K: input channels per slice at least (C1: 32 beat 64, profiles/r05zm)
#endif
#ifndef TTS_F32_SK_SMAX
#define TTS_F32_SK_SMAX 16  // fp32 split-K: at most this many slices (a cap keeps batch-invariant bits)
#endif
#ifndef TTS_F32_CK
#define TTS_F32_CK 16  // fp32 channel chunk (A/B builds: 32 -- half the staging rounds and barriers)
#endif
static int f32_ck(int Cin) { return Cin % TTS_F32_CK == 0 ? TTS_F32_CK : 16; }

// fp32 split-K: slices of >= TTS_F32_SLICE_CH input channels (every tap of them), at most 16, dividing the
// 16-channel chunk count -- from Cin only (ConvParams::f32_splitk), so layers that differ only in
// zero-padded taps (the batched variance predictors) still sum in the same order.  At batch 1 (C1)
// the fp32 acoustic model's FFN convs ran on 3 (encoder) / 12 (decoder) blocks of 128 x 128 for
// 565 us each, every block walking K = 4608 chunk by chunk with one HBM round trip per chunk.
int f32_kslices(int taps, int Cin) {
  const int ck = f32_ck(Cin);
  const int nch = (Cin + ck - 1) / ck;
  int S = taps > 0 ? std::min(TTS_F32_SK_SMAX, Cin / TTS_F32_SLICE_CH) : 1;
  while (S > 1 && nch % S) --S;
  return std::max(S, 1);
}

long long f32_splitk_ws_bytes(int taps, int Cin, int M, long long rows) {
  const int S = f32_kslices(taps, Cin);
  return S > 1 ? (long long)S * rows * M * 4 : 0;
}

static thread_local int g_f32sk_kernels = 0;

// the split-K form of an fp32 launch, or false when p does not take it
static bool launch_f32_splitk(const ConvParams& p, hipStream_t s, hipError_t* e, bool* ln_done) {
  if (!p.f32_splitk || p.up_s || p.nh != 1 || p.xres_order || p.M <= TTS_F32_SK_MINM) return false;
  const int S = f32_kslices(p.taps, p.Cin);
  if (S <= 1) return false;
  g_f32sk_kernels = 0;
  if (!p.ws || (long long)S * p.B * p.y_rows * p.M * 4 > p.ws_bytes) {  // the caller sized ws for its layers
    *e = hipErrorInvalidValue;
    return true;
  }
  ConvParams q = p;
  q.kslices = S;
  if (p.M <= 64)  // (launch_t's M <= 64 tile)
    *e = launch_cfg<float, 1, 2, 2, 2, 16>(q, s);
  else
    *e = f32_ck(p.Cin) == 16 ? launch_cfg<float, 1, 4, 4, 1, 16>(q, s) : launch_cfg<float, 1, 4, 4, 1, TTS_F32_CK>(q, s);
  if (*e != hipSuccess) return true;
  ConvParams r = p;
  r.x_rows = p.y_rows;  // the partials' rows per utterance
  *e = split_reduce_launch(r, S, s, ln_done);
  g_f32sk_kernels = 2;
  return true;
}

template <typename T>
static hipError_t launch_t(const ConvParams& p, hipStream_t s) {
  constexpr int CKW = 64 / (int)sizeof(T);   // 32 x 16-bit / 16 x f32 (64-byte rows)
  if constexpr (sizeof(T) == 4 && TTS_F32_CK != 16)
    if (p.nh == 1 && f32_ck(p.Cin) == TTS_F32_CK) {
      if (p.M <= 32) return launch_cfg<T, 1, 2, 1, 4, TTS_F32_CK>(p, s);
      if (p.M <= 64) return launch_cfg<T, 1, 2, 2, 2, TTS_F32_CK>(p, s);
      return launch_cfg<T, 1, 4, 4, 1, TTS_F32_CK>(p, s);
    }
  // fp32 head-batched attention products of the exact-duration encoder (M = 144-288 keys /
  // 192 channels, K = 144-192, 144 query rows, batch x heads): when the 128 x 128 grid would
  // fill under half the CUs (batch 8: 64 blocks), 64 x 64 tiles with 128-byte channel chunks,
  // one 32 x 32 MFMA tile per wave.  Measured at batch 8: the 12 launches 443 -> 289 us; at
  // batch 32 (256 blocks) the small tiles were slower (522 -> 585 us), so the rule.
  if constexpr (sizeof(T) == 4)
    if (p.nh > 1 && (long long)((p.y_rows + 127) / 128) * ((p.M + 127) / 128) * p.B * p.nh < 128)
      return p.Cin % 32 == 0 ? launch_cfg<T, 1, 1, 2, 2, 32>(p, s) : launch_cfg<T, 1, 1, 2, 2, CKW>(p, s);
  if (p.M <= 32) {
    return launch_cfg<T, 1, 2, 1, 4, CKW>(p, s);
  }
  if (p.M <= 64) {
    return launch_cfg<T, 1, 2, 2, 2, CKW>(p, s);
  }
  // M >= 128: 4 waves stacked along M, 32 x 128 per wave.  (A 32 x 256 strip per wave
  // cuts the L2-served weight bytes per MFMA in half but needs 235 VGPRs -> 2 waves/SIMD,
  // and measured 1.8x slower: the kernel is latency/issue-bound, not weight-bandwidth-bound.)
  return launch_cfg<T, 1, 4, 4, 1, CKW>(p, s);
}

#if TTS_XRES_STAMP
extern "C" int tts_debug_xres_target(int M, int Cin, int taps) {
  const int t[3] = {M, Cin, taps};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_xres_stamp_target), t, sizeof(t)) == hipSuccess ? 0 : -1;
}
extern "C" int tts_debug_xres_stamps(unsigned long long* host, long long words) {
  const long long n = words < (1LL << 20) ? words : (1LL << 20);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_xres_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

int conv_gemm_check(const ConvParams& p, int dtype, const char** why) {
  const int epv = dtype == DT_F32 ? 4 : 8;
  if (p.M <= 0 || p.Cin <= 0 || p.taps <= 0 || p.dil <= 0 || p.B <= 0) { *why = "bad dims"; return -1; }
  if (p.M % 4) { *why = "M must be a multiple of 4"; return -1; }
  if (p.Cin % epv) { *why = "Cin must be a multiple of 16 bytes"; return -1; }
  if (p.sxr % epv || p.w_ld % epv || p.sxb % epv || p.swb % epv) {
    *why = "X/W strides must be 16-byte multiples"; return -1;
  }
  if (p.syr % 4 || p.syb % 4 || ((p.r1 || p.r2) && (p.srr % 4 || p.srb % 4))) {
    *why = "Y/R strides must be multiples of 4 elements"; return -1;
  }
  if ((p.taps - 1) * p.dil > HALO_MAX) { *why = "receptive field (taps-1)*dil > 64"; return -1; }
  if (p.up_s && (p.up_cout % 4 || !p.up_len)) { *why = "bad transposed mapping"; return -1; }
  if (p.x_rows <= 0 || p.y_rows <= 0) { *why = "empty rows"; return -1; }
  if (p.nh < 1 || p.sxh % epv || p.swh % epv || p.syh % 4 || p.srh % 4) { *why = "bad head batching"; return -1; }
  if (dtype == DT_F32 && p.f32_splitk && !p.up_s && p.nh == 1 && !p.xres_order && p.M > TTS_F32_SK_MINM && !conv_split_eligible(p)) {
    const int S = f32_kslices(p.taps, p.Cin);
    if (S > 1 && (!p.ws || (long long)S * p.B * p.y_rows * p.M * 4 > p.ws_bytes)) {
      *why = "fp32 split-K workspace smaller than this layer's partials (reserve with the caller's batch / rows)";
      return -1;
    }
  }
  return 0;
}

int conv_gemm_kind(int dtype, const ConvParams& p) {
  if (dtype == DT_F32) return conv_split_eligible(p) ? PK_CONV_SPLIT : PK_CONV_GEMM;
  return (dtype != DT_F32 && xres_group(p, 32 * 4 * (4 / xres_wm(p)))) ? PK_CONV_XRES : PK_CONV_GEMM;
}

static hipError_t conv_gemm_launch_noln(int dtype, const ConvParams& p, hipStream_t s, bool* ln_done) {
  switch (dtype) {
    case DT_F32: {
      if (conv_split_eligible(p)) return conv_split_launch(p, s, ln_done);
      hipError_t e;
      if (launch_f32_splitk(p, s, &e, ln_done)) return e;
      return launch_t<float>(p, s);
    }
    case DT_F16: {
      hipError_t e;
      if (launch_xres<half_t>(p, s, &e, ln_done)) return e;
      return launch_t<half_t>(p, s);
    }
    case DT_BF16: {
      hipError_t e;
      if (launch_xres<bf16_t>(p, s, &e, ln_done)) return e;
      return launch_t<bf16_t>(p, s);
    }
  }
  return hipErrorInvalidValue;
}

static thread_local int g_conv_kernels = 0;
int conv_last_kernels() { return g_conv_kernels; }

hipError_t conv_gemm_launch(int dtype, const ConvParams& p, hipStream_t s) {
  bool ln_done = false;
  g_conv_kernels = 1;
  const hipError_t e = conv_gemm_launch_noln(dtype, p, s, &ln_done);
  if (dtype == DT_F32 && conv_split_eligible(p)) g_conv_kernels = conv_split_last_kernels();
  else if (dtype == DT_F32 && g_f32sk_kernels) g_conv_kernels = g_f32sk_kernels, g_f32sk_kernels = 0;
  if (e != hipSuccess || !(p.ln_out || p.ln_lin_out) || ln_done) return e;
  ++g_conv_kernels;
  // LayerNorm as its own launch over the [B][y_rows] output (contiguous rows of M); rows past an
  // utterance's length are skipped (no consumer reads them)
  if (p.syr != p.M || p.syb != (long long)p.y_rows * p.syr || p.nh != 1) return hipErrorInvalidValue;
  if (p.ln_lin_out)
    return launch_ln_linear1(dtype, p.y, p.B * p.y_rows, p.M, p.ln_g1, p.ln_b1, p.ln_eps, p.ln_lin_w, p.ln_lin_b,
                             p.ln_lin_out, s);
  return launch_layernorm(dtype, p.y, p.ln_out, p.B * p.y_rows, p.M, p.ln_g1, p.ln_b1, p.ln_g2, p.ln_b2, p.ln_eps, s,
                          p.y_len, p.y_rows);
}

}  // namespace tts
