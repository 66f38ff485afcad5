// fp32 implicit-GEMM conv computed as three f16 MFMAs ("split precision"), gfx950.
//
// gfx950 has no xf32 and its native fp32 MFMA (v_mfma_f32_32x32x2_f32) peaks at 1/16 of the
// 16-bit rate.  An fp32 value a is split into two f16 terms,
//     a_hi = f16(a),   a_lo = f16(a - a_hi)        (a ~= a_hi + a_lo),
// a_hi carrying the top 11 significand bits and a_lo the next 11 (a_lo is subnormal for |a| below
// ~2^-3 and then keeps fewer bits: an absolute error under 2^-25 per element, below the fp32
// rounding of the sums it enters), and
//     sum a*b ~= sum a_hi*b_hi + a_hi*b_lo + a_lo*b_hi
// runs as three v_mfma_f32_32x32x16_f16 into ONE fp32 accumulator.  The weights are stored scaled
// by a power of two 2^s per layer (frag_pack_split: max|w| 2^s in [2^14, 2^15), so the weights' lo
// plane stays normal) and the sums are multiplied by ConvParams::w_unscale = 2^-s, exactly.  The
// dropped a_lo*b_lo term and the representation errors are ~2^-21 relative per product: ~8x the
// fp32 rounding of one product, 1000x below bf16.  Effective fp32 throughput is 1/3 of the f16
// peak: ~5x the native fp32 MFMA.  Range: |a| < 65504 (f16); the encoder's activations are O(100).
//
// Used for the acoustic encoder + variance predictors in "exact" encoder precision (the
// integer durations of HF:181-183 then match the fp32 oracle, SURVEY.md §8c "durations: exact
// integer match"; the decoder and postnet stay 16-bit).
//
// Layout: X fp32 [B][rows][Cin] channels-last; weights packed by frag_pack_split (runtime.h):
// two planes of f16 fragments [M/32][taps][Cin/16][64 lanes][8] (hi, then lo * 2^11), so a
// wave's A fragment is one contiguous 1 KiB read.  Block: 4 waves along M (128 output
// channels), NT 32-row MFMA tiles along time.  A channel group CG of the block's X rows (every
// tap's halo included) is split once into two LDS planes (row stride CG*2+16 bytes: an odd
// number of 16-byte slots, conflict-free ds_read_b128 over 32 consecutive rows); the weight
// quads (4 k-steps, hi + lo = 8 fragments) stream through a 2-deep register ring over a
// bounds-checked buffer descriptor (a load past the group's last quad fetches nothing, so the
// ring reloads unconditionally).  The epilogue is conv_gemm's (bias, alpha, activation,
// residuals, scale; fp32 rows).
#include "common.h"
#include "conv_epilogue.h"
#include "kernels.h"
#include "ln_rows.h"
#include "switches.h"

#ifndef TTS_LN_FUSE_MINBLK
#define TTS_LN_FUSE_MINBLK 512  // GEMM blocks from which a launch applies its post-LN itself (same-box A/B: 0 slower at batch 8)
#endif
#ifndef TTS_SPLIT_STAMP
#define TTS_SPLIT_STAMP 0  // diagnostic builds: per-block phase timestamps of one launch shape (tools/xres_stamps.py)
#endif
#ifndef TTS_SPLIT_NT1_MAXBLK
#define TTS_SPLIT_NT1_MAXBLK 128  // 64-row grids below this many blocks run 32-row tiles (0: never)
#endif
#ifndef TTS_SPLIT_PROBE
#define TTS_SPLIT_PROBE 0  // timing-only probe builds: every weight quad read from the first (L1/L2-hot, wrong results)
#endif
#ifndef TTS_SPLIT_WHOLE_MAXBLK
#define TTS_SPLIT_WHOLE_MAXBLK 256  // packed split GEMMs of at most this many blocks stage their K slice at once
#endif
#ifndef TTS_SPLIT_NT4_MINBLK
#define TTS_SPLIT_NT4_MINBLK 320  // 128-row split GEMM tiles from this many blocks (~1.25 per CU)
#endif
#ifndef TTS_SPLIT_KQ4
#define TTS_SPLIT_KQ4 1  // k-steps per weight-ring slot of the 128-row tiles (register budget)
#endif
#ifndef TTS_LN_TAIL
#define TTS_LN_TAIL 1  // 0: timing-only probe builds -- fused post-LN tails load their rows but compute nothing
#endif

#include <algorithm>
#include <cstdlib>

namespace tts {

constexpr int SPLIT_SU = 4;            // X staging loads (x2) in flight per thread

// 8 fp32 -> (hi, lo) f16 x 8
__device__ inline void split8(f32x4 a, f32x4 b, uint4& hi, uint4& lo) {
  const half4 ha = __builtin_convertvector(a, half4), hb = __builtin_convertvector(b, half4);
  const f32x4 ra = a - __builtin_convertvector(ha, f32x4);
  const f32x4 rb = b - __builtin_convertvector(hb, f32x4);
  const half4 la = __builtin_convertvector(ra, half4), lb = __builtin_convertvector(rb, half4);
  const uint2 h0 = __builtin_bit_cast(uint2, ha), h1 = __builtin_bit_cast(uint2, hb);
  const uint2 l0 = __builtin_bit_cast(uint2, la), l1 = __builtin_bit_cast(uint2, lb);
  hi = uint4{h0.x, h0.y, h1.x, h1.y};
  lo = uint4{l0.x, l0.y, l1.x, l1.y};
}

// KQ: k-steps per weight-ring slot -- 4, or 2 / 1 for 64- / 32-channel groups (the fp32 vocoder's
// stage-2 / stage-3 convs), so a group always has an even number of slots.  (At M = 32 -- stage 3 --
// three of the four waves recompute the one 32-channel block and store nothing: the split form is
// still ~5x the fp32 MFMA's rate per product, and each wave has a SIMD of its own.)
template <int NT, int UW, int KQ = 4>
__global__ __launch_bounds__(256, 2) void conv_split_kernel(ConvParams p, int CG) {
  typedef half8 Frag;
  constexpr int WM = 4 / UW;  // waves along M; UW waves along utterances (same weights)
  constexpr int BN = 32 * NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // XCD-aware order (cdna_hip_programming.md T1): blocks are dealt round-robin over the 8 XCDs,
  // so work item w = (M block, utterance group, row tile), M block slowest, is given to block
  // ids such that each XCD runs one contiguous range of w -- one or two M blocks.
  const int ntx = (p.y_rows + BN - 1) / BN;
  const int nbz = (p.B + UW - 1) / UW;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int w = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int tx = w % ntx;
  const int bz = (w / ntx) % nbz;
  const int by = w / (ntx * nbz);
  const int n0 = tx * BN;
  auto ylen_of = [&](int bb) { return bb < p.B ? (p.y_len ? min(p.y_len[bb], p.y_rows) : p.y_rows) : 0; };
  auto xlen_of = [&](int bb) { return bb < p.B ? (p.x_len ? min(p.x_len[bb], p.x_rows) : p.x_rows) : 0; };
  {
    int ymax = 0;
#pragma unroll
    for (int u = 0; u < UW; ++u) ymax = max(ymax, ylen_of(bz * UW + u));
    if (n0 >= ymax) return;  // uniform over the block
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wu = wave / WM;
  const int b = bz * UW + wu;  // this wave's utterance (>= B: computed, never stored)
  const int l31 = lane & 31;
  const int hh = lane >> 5;

  const int KST = p.Cin / 16;
  const int MB = (p.M + 31) / 32;
  const int mb = min(by * WM + wm, MB - 1);  // a wave past M recomputes the last block (not stored)
  const int wbytes = __builtin_amdgcn_readfirstlane(p.taps * KST * 1024);
  const char* whi = reinterpret_cast<const char*>(p.wpk) + (long long)mb * wbytes;
  const char* wlo = whi + (long long)MB * wbytes;
  const auto rs_hi = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(whi), 0, wbytes, 0x00020000);
  const auto rs_lo = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wlo), 0, wbytes, 0x00020000);
  const int lofs = lane * 16;

  const int R = BN + (p.taps - 1) * p.dil;  // staged rows per utterance
  const int RU = UW * R;
  const int RS = CG * 2 + 16;
  const int PL = RU * RS;                // bytes per LDS plane
  const int KS = CG / 16;                // k-steps per tap and group
  const int lks = __builtin_ctz(KS);
  const int QT = p.taps * KS / KQ;       // weight-ring slots per group (even: 8 per 128 channels / 4 per 64)
  const int x_start = n0 - p.pad;
  const char* xl = smem + (wu * R + l31) * RS + hh * 16;

  f32x16 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x16{};
  unsigned rng = 0;  // range guard over the staged hi halves (common.h f16x2_nonfinite)

  // staging: thread owns 8-channel column cc of the group and staged rows r0, r0 + rstep, ...
  // (staged row rr = utterance u * R + local row), SPLIT_SU loads in flight per batch
  const int VPR = CG / 8;
  const int lvpr = __builtin_ctz(VPR);
  const int cc = tid & (VPR - 1);
  const int r0 = tid >> lvpr;
  const int rstep = 256 >> lvpr;
  auto stage = [&](int g) {
    for (int rb = r0; rb < RU; rb += SPLIT_SU * rstep) {
      f32x4 xa[SPLIT_SU], xb[SPLIT_SU];
      bool ok[SPLIT_SU];
#pragma unroll
      for (int i = 0; i < SPLIT_SU; ++i) {  // unconditional, clamped addresses (masked below)
        const int rr = min(rb + i * rstep, RU - 1);
        const int u = rr / R;
        const int bu = min(bz * UW + u, p.B - 1);
        const int xl_ = xlen_of(bz * UW + u);
        const int xrow = x_start + rr - u * R;
        ok[i] = xrow >= 0 && xrow < xl_;
        const float* src = reinterpret_cast<const float*>(p.x) + (long long)bu * p.sxb +
                           (long long)min(max(xrow, 0), max(xl_ - 1, 0)) * p.sxr + g + cc * 8;
        xa[i] = *reinterpret_cast<const f32x4*>(src);
        xb[i] = *reinterpret_cast<const f32x4*>(src + 4);
      }
#pragma unroll
      for (int i = 0; i < SPLIT_SU; ++i) {
        const int rr = rb + i * rstep;
        f32x4 va = xa[i], vb = xb[i];
        if (!ok[i]) { va = f32x4{}; vb = f32x4{}; }
        if (p.in_slope != 1.0f) {
#pragma unroll
          for (int e = 0; e < 4; ++e) { va[e] = leaky(va[e], p.in_slope); vb[e] = leaky(vb[e], p.in_slope); }
        }
        uint4 hi, lo;
        split8(va, vb, hi, lo);
        rng |= f16x2_nonfinite(hi.x) | f16x2_nonfinite(hi.y) | f16x2_nonfinite(hi.z) | f16x2_nonfinite(hi.w);
        if (rr < RU) {
          *reinterpret_cast<uint4*>(smem + rr * RS + cc * 16) = hi;
          *reinterpret_cast<uint4*>(smem + PL + rr * RS + cc * 16) = lo;
        }
      }
    }
  };

  for (int g0 = 0; g0 < p.Cin; g0 += CG) {
    Frag a0[2 * KQ], a1[2 * KQ];  // slot ring: [0, KQ) hi, [KQ, 2 KQ) lo
    // quad qq of this group: k-steps 4qq .. 4qq+3 (never across a tap: KS % 4 == 0)
#define TTS_SPLIT_LOADQ(A_, QQ_)                                                                     \
    do {                                                                                             \
      const int kq_ = KQ * (QQ_);                                                                    \
      const int o_ = (((kq_ >> lks) * KST + g0 / 16 + (kq_ & (KS - 1))) * 1024) +                    \
                     (((QT - 1 - (QQ_)) >> 31) & 0x40000000); /* out of range past the group */      \
      _Pragma("unroll") for (int j_ = 0; j_ < KQ; ++j_) {                                            \
        A_[j_] = __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(rs_hi, lofs + j_ * 1024, o_, 0)); \
        A_[KQ + j_] = __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(rs_lo, lofs + j_ * 1024, o_, 0)); \
      }                                                                                              \
      __builtin_amdgcn_sched_barrier(0);                                                             \
    } while (0)
#define TTS_SPLIT_MMAQ(A_, QQ_)                                                                      \
    do {                                                                                             \
      const int kq_ = KQ * (QQ_);                                                                    \
      const char* bq_ = xl + (kq_ >> lks) * p.dil * RS + (kq_ & (KS - 1)) * 32;                      \
      _Pragma("unroll") for (int j_ = 0; j_ < KQ; ++j_) {                                            \
        Frag bh_[NT], bl_[NT];                                                                       \
        _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_) {                                       \
          bh_[nt_] = *reinterpret_cast<const Frag*>(bq_ + nt_ * 32 * RS + j_ * 32);                  \
          bl_[nt_] = *reinterpret_cast<const Frag*>(bq_ + PL + nt_ * 32 * RS + j_ * 32);             \
        }                                                                                            \
        _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_) {                                       \
          acc[nt_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A_[j_], bh_[nt_], acc[nt_], 0, 0, 0);    \
          acc[nt_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A_[j_], bl_[nt_], acc[nt_], 0, 0, 0);    \
          acc[nt_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A_[KQ + j_], bh_[nt_], acc[nt_], 0, 0, 0); \
        }                                                                                            \
      }                                                                                              \
    } while (0)

    int q = 0;
    if constexpr (NT == 1) {
      // 4-slot quad ring: the quad three ahead goes into the slot consumed one quad earlier (two
      // quads of MFMAs cover its latency, and no load lands in a register an MFMA of the quad
      // just issued still reads -- a 2-slot ring at one row tile was register-renamed by the
      // compiler, whose copies then waited for every load at the end of each iteration)
      Frag a2[2 * KQ], a3[2 * KQ];
      TTS_SPLIT_LOADQ(a0, 0);
      TTS_SPLIT_LOADQ(a1, 1);
      TTS_SPLIT_LOADQ(a2, 2);
      if (g0) __syncthreads();  // the previous group's tile is no longer read
      stage(g0);
      __syncthreads();
      for (; q < QT; q += 4) {  // the quads past QT load nothing and are skipped
        TTS_SPLIT_MMAQ(a0, q);
        TTS_SPLIT_LOADQ(a3, q + 3);
        TTS_SPLIT_MMAQ(a1, q + 1);
        TTS_SPLIT_LOADQ(a0, q + 4);
        if (q + 2 < QT) {
          TTS_SPLIT_MMAQ(a2, q + 2);
          TTS_SPLIT_LOADQ(a1, q + 5);
          TTS_SPLIT_MMAQ(a3, q + 3);
          TTS_SPLIT_LOADQ(a2, q + 6);
        } else {
          TTS_SPLIT_LOADQ(a1, q + 5);
          TTS_SPLIT_LOADQ(a2, q + 6);
        }
      }
    } else {
      TTS_SPLIT_LOADQ(a0, 0);
      TTS_SPLIT_LOADQ(a1, 1);
      if (g0) __syncthreads();
      stage(g0);
      __syncthreads();
      for (; q < QT; q += 2) {
        TTS_SPLIT_MMAQ(a0, q);
        TTS_SPLIT_LOADQ(a0, q + 2);
        TTS_SPLIT_MMAQ(a1, q + 1);
        TTS_SPLIT_LOADQ(a1, q + 3);
      }
    }
#undef TTS_SPLIT_LOADQ
#undef TTS_SPLIT_MMAQ
  }

  range_report(p.range_flag, rng);
  if (b >= p.B) return;
  f32x16 out[1][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) out[0][j] = acc[j] * p.w_unscale;
  conv_epilogue<float, 1, NT>(p, out, b, 0, n0, (by * WM + wm) * 32, ylen_of(b), l31, hh);
}

// ---------------------------------------------------------------------------------------
// Packed-row form (ConvParams::rows_pad): the batch is one flat sequence of B * x_rows rows, an
// utterance's rows followed by >= rows_pad masked rows, so a 128-row tile may hold the end of
// one utterance and the start of the next (every staged row is masked by its own utterance's
// length; a conv tap never reaches past the masked gap).  Block: 4 waves along M (128 output
// channels) x 128 rows (each wave 4 MFMA row tiles; each weight quad feeds 12 MFMAs, a quarter
// of the per-CU weight stream of 32-row tiles, with no row cover beyond the 32-row padding).
// K is optionally split into S slices of whole channel groups (S from the layer shape only, so a
// row's accumulation order never depends on the batch): each slice writes fp32 partial sums to
// ConvParams::ws and split_reduce_kernel adds them in slice order and applies the epilogue.
constexpr int SPK_NT = 2;   // 32-row MFMA tiles per wave: 64-row blocks
constexpr int SPK_SU = 9;   // X prefetch registers (16 B each) per thread: 66-72 rows x 128 channels
constexpr int SPK_SU4 = 17; // the same for 128-row blocks (NT = 4): 130-136 rows
__host__ __device__ constexpr int spk_su(int nt) { return nt >= 4 ? SPK_SU4 : SPK_SU; }

__device__ inline int packed_valid(const ConvParams& p, const int* lens, int f, int F) {
  if (f < 0 || f >= F) return 0;
  const int b = f / p.x_rows;
  const int r = f - b * p.x_rows;
  return r < (lens ? min(lens[b], p.x_rows) : p.x_rows);
}

// The fused post-LN of a one-slice conv_splitp launch (ConvParams::ln_cnt): the valid rows among
// flat rows [f0, f0 + BN) of the fp32 output y (all M <= 512 channels), one wave per row;
// layernorm_kernel / ln_linear1_kernel arithmetic (ln_rows.h), lane l owning channels l + 64 i.
__device__ inline void splitp_tile_ln(const ConvParams& p, int f0, int BN, int F, int wave, int lane) {
  const int C = p.M;
  constexpr int RB = 4;  // rows per wave in flight and normalised together
  int ch[8];
  bool on[8];
  ln_lanes64<8>(ch, on, C, lane);
  float g[2][8], bb[2][8], wl[8];
  ln_params<8>(g, bb, ch, on, p.ln_g1, p.ln_b1, p.ln_g2, p.ln_b2);
#pragma unroll
  for (int i = 0; i < 8; ++i) wl[i] = on[i] && p.ln_lin_w ? p.ln_lin_w[ch[i]] : 0.f;
  const auto ylrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.y_len ? p.y_len : reinterpret_cast<const int*>(p.y)),
                                                      0, p.y_len ? p.B * 4 : 0, 0x00020000);
  for (int r0 = wave; r0 < BN; r0 += 4 * RB) {
    float v[RB][8];
    long long ro[RB];
    bool ok[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {  // unconditional loads at clamped rows / channels
      const int f = min(f0 + min(r0 + 4 * k, BN - 1), F - 1);
      const int b = f / p.x_rows, r = f - b * p.x_rows;
      // (the length through a descriptor, OR-ed to "no limit" when absent: an unconditional load)
      const int L = __builtin_amdgcn_raw_buffer_load_b32(ylrs, b * 4, 0, 0) | (p.y_len ? 0 : 0x7fffffff);
      ok[k] = r0 + 4 * k < BN && f0 + r0 + 4 * k < F && r < min(L, p.y_rows);
      ro[k] = p.ln_lin_out ? (long long)b * p.y_rows + r : (long long)b * p.syb + (long long)r * p.syr;
      const float* x = reinterpret_cast<const float*>(p.y) + (long long)b * p.syb + (long long)r * p.syr;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[k][i] = x[min(ch[i], C - 1)];
    }
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (!on[i]) v[k][i] = 0.f;
#if TTS_LN_TAIL
    if (p.ln_lin_out) {
      float o[RB];
      ln_linear1_batch<float, RB, 8>(v, on, C, g[0], bb[0], wl, p.ln_eps, p.ln_lin_b, o);
#pragma unroll
      for (int k = 0; k < RB; ++k)
        if (lane == 0 && ok[k]) p.ln_lin_out[ro[k]] = o[k];
      continue;
    }
    if (p.ln_g2) ln_batch<float, RB, 8, true>(v, on, C, g, bb, p.ln_eps);
    else ln_batch<float, RB, 8, false>(v, on, C, g, bb, p.ln_eps);
#endif
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if (ok[k] && !p.ln_lin_out) {
        float* o = reinterpret_cast<float*>(p.ln_out) + ro[k];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (on[i]) o[ch[i]] = v[k][i];
      }
  }
}

// one flat row f of the split-K reduce + LayerNorm, by one wave (rows past an utterance: nothing).
// Every load is unconditional (clamped channels, the length through a descriptor) and the slices
// go one at a time with all of the lane's channels in flight: the first form returned early on
// the row's length and loaded each channel's slices under its own branch -- a wait per load.
__device__ inline void split_reduce_ln_row(const ConvParams& p, int S, int F, int f, int lane) {
  constexpr int PER = 8;
  const int b = f / p.x_rows;
  const int r = f - b * p.x_rows;
  const auto ylrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.y_len ? p.y_len : reinterpret_cast<const int*>(p.ws)),
                                                      0, p.y_len ? p.B * 4 : 0, 0x00020000);
  const int ylen = min(__builtin_amdgcn_raw_buffer_load_b32(ylrs, b * 4, 0, 0) | (p.y_len ? 0 : 0x7fffffff), p.y_rows);
  const int C = p.M;
  const long long ro = (long long)b * p.srb + (long long)r * p.srr;
  int ch[PER];
  bool on[PER];
  ln_lanes64<PER>(ch, on, C, lane);
  float g[2][PER], bb[2][PER], v[1][PER];
  ln_params<PER>(g, bb, ch, on, p.ln_g1, p.ln_b1, p.ln_g2, p.ln_b2);
  float x[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) x[i] = p.ws[(long long)f * C + min(ch[i], C - 1)];
  for (int sl = 1; sl < S; ++sl) {
    float w[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) w[i] = p.ws[((long long)sl * F + f) * C + min(ch[i], C - 1)];
#pragma unroll
    for (int i = 0; i < PER; ++i) x[i] += w[i];
  }
  // bias / residuals through descriptors with no records when absent (unconditional loads, the
  // adds selected by the uniform flags: the same operations as the branches they replace)
  const auto mk = [&](const void* q, long long n) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(q ? q : (const void*)p.ws), 0, q ? (int)min(n, 0x7fffffffLL) : 0, 0x00020000);
  };
  const auto bs = mk(p.bias, (long long)C * 4), r1s = mk(p.r1, 0x7fffffffLL), r2s = mk(p.r2, 0x7fffffffLL);
  float bv[PER], r1v[PER], r2v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = min(ch[i], C - 1);
    bv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bs, c * 4, 0, 0));
    r1v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1s, (int)((ro + c) * 4), 0, 0));
    r2v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2s, (int)((ro + c) * 4), 0, 0));
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    float y = x[i];
    if (p.bias) y += bv[i];
    if (p.alpha != 1.0f) y *= p.alpha;
    if (p.r1) y += r1v[i];
    if (p.r2) y += r2v[i];
    if (p.out_scale != 1.0f) y *= p.out_scale;
    v[0][i] = on[i] ? y : 0.f;
  }
  if (p.ln_g2) ln_batch<float, 1, PER, true>(v, on, C, g, bb, p.ln_eps);
  else ln_batch<float, 1, PER, false>(v, on, C, g, bb, p.ln_eps);
  if (r >= ylen) return;
  float* o = reinterpret_cast<float*>(p.ln_out) + (long long)b * p.syb + (long long)r * p.syr;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (on[i]) o[ch[i]] = v[0][i];
}

// WHOLE: every channel group of the block's K slice (at most SPK_WG) is staged at once, their X
// loads all in flight together, into LDS regions of their own (one block per CU), and the MFMA
// loop runs over the groups with no restaging -- for grids of at most one block per CU (the
// batch-8 encoder), where each group's load round trip and barriers were the block's critical
// path.  Same groups, quads and MFMA order: bit-identical to the group-by-group form.
constexpr int SPK_WG = 3;
#if TTS_SPLIT_STAMP
// records of the launches whose (M, Cin, taps) match g_split_stamp_target: conv_xres's layout
// (st0, staging done, MFMA loop done, row pass done, staging cycles, realtime start / end, hw id)
__device__ int g_split_stamp_target[3];
__device__ unsigned long long g_split_stamp[1 << 18];
#endif
// NT: 32-row MFMA tiles per wave (SPK_NT; 1 for grids the 64-row tiles leave under-filled, 4 for
// grids that fill the chip with 128-row tiles: half the weight stream and X staging per MFMA)
template <bool WHOLE, int NT = SPK_NT>
__global__ __launch_bounds__(256, 2) void conv_splitp_kernel(ConvParams p, int CG, int S, int gps) {
  typedef half8 Frag;
  constexpr int BN = 32 * NT;
  constexpr int SU = spk_su(NT);
  static_assert(!(WHOLE && NT >= 4), "whole-slice staging is for small grids");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int F = p.B * p.x_rows;  // flat rows
  const int ntx = (F + BN - 1) / BN;
  const int nmb = (p.M + 127) / 128;
  // XCD-aware order (T1): work w = (slice, M block, row tile), row tile fastest, contiguous per XCD
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xq = nwg / 8, xr = nwg % 8, xcd = orig % 8;
  const int w = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + orig / 8;
  const int tx = w % ntx;
  const int by = (w / ntx) % nmb;
  const int sl = w / (ntx * nmb);
  const int f0 = tx * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31;
  const int hh = lane >> 5;

  const int KST = p.Cin / 16;
  const int MB = (p.M + 31) / 32;
  const int mb = min(by * 4 + wave, MB - 1);
  const int wbytes = __builtin_amdgcn_readfirstlane(p.taps * KST * 1024);
  const char* whi = reinterpret_cast<const char*>(p.wpk) + (long long)mb * wbytes;
  const char* wlo = whi + (long long)MB * wbytes;
  const auto rs_hi = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(whi), 0, wbytes, 0x00020000);
  const auto rs_lo = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wlo), 0, wbytes, 0x00020000);
  const int lofs = lane * 16;

  const int R = BN + (p.taps - 1) * p.dil;
  const int RS = CG * 2 + 16;
  const int PL = R * RS;
  const int KS = CG / 16;
  const int lks = __builtin_ctz(KS);
  // weight ring slots of KQ k-steps (hi + lo fragments each): 4, or 2 at 128-row tiles, whose
  // accumulators and X prefetch leave no room for 4-step slots at two waves per SIMD
  constexpr int KQ = NT >= 4 ? TTS_SPLIT_KQ4 : 4;
  const int QT = p.taps * KS / KQ;  // even (CG >= 128)
  const int x_start = f0 - p.pad;
  const char* xl = smem + l31 * RS + hh * 16;
  const float* X = reinterpret_cast<const float*>(p.x);
#if TTS_SPLIT_STAMP
  const unsigned long long st0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long st1 = 0, st2 = 0;
  auto stamp = [&]() __attribute__((always_inline)) {
    if (p.M == g_split_stamp_target[0] && p.Cin == g_split_stamp_target[1] && p.taps == g_split_stamp_target[2]) {
      __syncthreads();
      if (tid == 0 && blockIdx.x < (1u << 15)) {
        unsigned long long* r = g_split_stamp + blockIdx.x * 8;
        r[0] = st0; r[1] = st1; r[2] = st2; r[3] = __builtin_amdgcn_s_memtime();
        r[4] = st1 - st0; r[5] = rt0; r[6] = __builtin_amdgcn_s_memrealtime();
        r[7] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)) << 32) |
               (unsigned)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
      }
    }
  };
#endif

  f32x16 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x16{};
  unsigned rng = 0;  // range guard over the staged hi halves (common.h f16x2_nonfinite)

  // X staging: thread owns 4-channel column c4 of the group and staged rows r0, r0 + rstep, ...
  // (at most SU: split_group sizes CG for that).  The next group's rows are loaded into
  // registers while the current group's MFMAs run (issued two weight quads into the group, so
  // the first wait on a younger weight load finds them landed) and split into LDS after them.
  const int VPR = CG / 4;
  const int lvpr = __builtin_ctz(VPR);
  const int c4 = tid & (VPR - 1);
  const int r0 = tid >> lvpr;
  const int rstep = 256 >> lvpr;
  f32x4 xv[SU];
  // Validity of this thread's staged rows (the same rows for every group), bit i for row
  // r0 + i * rstep: computed once, after the first group's X loads are issued, with the length
  // loads through a descriptor (no branch around them).  Computing it per row inside the LDS
  // stores made the compiler wait for every outstanding load (vmcnt(0)) once per staged row:
  // at batch 8, 27 serialized round trips, 59 % of a K = 384 block's time (tools/xres_stamps.py).
  int vm = 0;
  auto row_mask = [&]() __attribute__((always_inline)) {
    const auto lrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.x_len ? p.x_len : reinterpret_cast<const int*>(X)),
                                                       0, p.x_len ? p.B * 4 : 0, 0x00020000);
    int m = 0;
#pragma unroll
    for (int i = 0; i < SU; ++i) {
      const int f = x_start + r0 + i * rstep;
      const int fc = min(max(f, 0), F - 1);
      const int b = fc / p.x_rows, r = fc - b * p.x_rows;
      // (no length array: the descriptor reads 0 and the OR makes the limit x_rows -- the load
      // stays unconditional, not sunk into a branch with a wait of its own)
      const int L = __builtin_amdgcn_raw_buffer_load_b32(lrs, b * 4, 0, 0) | (p.x_len ? 0 : 0x7fffffff);
      const int lim = min(L, p.x_rows);
      m |= (f >= 0 && f < F && r < lim ? 1 : 0) << i;
    }
    return m;
  };
  auto load_x_to = [&](int g, f32x4 (&xd)[SU]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < SU; ++i) {
      const int f = x_start + min(r0 + i * rstep, R - 1);
      xd[i] = *reinterpret_cast<const f32x4*>(X + (long long)min(max(f, 0), F - 1) * p.sxr + g + c4 * 4);
    }
  };
  auto load_x = [&](int g) __attribute__((always_inline)) { load_x_to(g, xv); };
  auto store_x_from = [&](const f32x4 (&xs)[SU], char* base) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < SU; ++i) {
      const int rr = r0 + i * rstep;
      f32x4 v = xs[i];
      if (!((vm >> i) & 1)) v = f32x4{};
      if (p.in_slope != 1.0f) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = leaky(v[e], p.in_slope);
      }
      const half4 h = __builtin_convertvector(v, half4);
      const half4 l = __builtin_convertvector(v - __builtin_convertvector(h, f32x4), half4);
      const uint2 hb = __builtin_bit_cast(uint2, h);
      rng |= f16x2_nonfinite(hb.x) | f16x2_nonfinite(hb.y);
      if (rr < R) {
        *reinterpret_cast<uint2*>(base + rr * RS + c4 * 8) = __builtin_bit_cast(uint2, h);
        *reinterpret_cast<uint2*>(base + PL + rr * RS + c4 * 8) = __builtin_bit_cast(uint2, l);
      }
    }
  };
  auto store_x = [&]() __attribute__((always_inline)) { store_x_from(xv, smem); };

  const int gbeg = sl * gps * CG, gend = min(p.Cin, (sl + 1) * gps * CG);
  // Weight quads form one ring over the slice: the two quads past a group's last are the next
  // group's first two (issued before the group-change barriers, so their latency overlaps the
  // X restaging); past the slice's last group they fall outside the descriptor and fetch nothing.
  Frag a0[2 * KQ], a1[2 * KQ];
  int g0 = gbeg;
#define TTS_SPLIT_LOADQ(A_, QQ_)                                                                     \
    do {                                                                                             \
      const int nx_ = (QQ_) >= QT;                                                                   \
      const int kq_ = KQ * ((QQ_) - nx_ * QT);                                                       \
      const int gg_ = g0 + nx_ * CG;                                                                 \
      const int o_ = TTS_SPLIT_PROBE ? 0 : (((kq_ >> lks) * KST + gg_ / 16 + (kq_ & (KS - 1))) * 1024) + \
                     (gg_ < gend ? 0 : 0x40000000);                                                  \
      _Pragma("unroll") for (int j_ = 0; j_ < KQ; ++j_) {                                            \
        A_[j_] = __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(rs_hi, lofs + j_ * 1024, o_, 0)); \
        A_[KQ + j_] = __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(rs_lo, lofs + j_ * 1024, o_, 0)); \
      }                                                                                              \
      __builtin_amdgcn_sched_barrier(0);                                                             \
    } while (0)
#define TTS_SPLIT_MMAQ(A_, QQ_)                                                                      \
    do {                                                                                             \
      const int kq_ = KQ * (QQ_);                                                                    \
      const char* bq_ = xg + (kq_ >> lks) * p.dil * RS + (kq_ & (KS - 1)) * 32;                      \
      _Pragma("unroll") for (int j_ = 0; j_ < KQ; ++j_) {                                            \
        _Pragma("unroll") for (int nt_ = 0; nt_ < NT; ++nt_) {                                       \
          const Frag bh_ = *reinterpret_cast<const Frag*>(bq_ + nt_ * 32 * RS + j_ * 32);            \
          const Frag bl_ = *reinterpret_cast<const Frag*>(bq_ + PL + nt_ * 32 * RS + j_ * 32);       \
          acc[nt_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A_[j_], bh_, acc[nt_], 0, 0, 0);         \
          acc[nt_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A_[j_], bl_, acc[nt_], 0, 0, 0);         \
          acc[nt_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A_[KQ + j_], bh_, acc[nt_], 0, 0, 0);    \
        }                                                                                            \
      }                                                                                              \
    } while (0)
  TTS_SPLIT_LOADQ(a0, 0);
  TTS_SPLIT_LOADQ(a1, 1);
  const char* xg = xl;  // the current group's LDS tile
  if constexpr (WHOLE) {
    // every group's X loads in flight at once, then split into the groups' own LDS regions
    f32x4 xw[SPK_WG][SU];
    const int ng = (gend - gbeg) / CG;  // <= SPK_WG (launcher)
#pragma unroll
    for (int i = 0; i < SPK_WG; ++i) load_x_to(gbeg + min(i, ng - 1) * CG, xw[i]);
    __builtin_amdgcn_sched_barrier(0);  // the X loads issue before the length loads
    vm = row_mask();
#pragma unroll
    for (int i = 0; i < SPK_WG; ++i)
      if (i < ng) store_x_from(xw[i], smem + i * 2 * PL);
  } else {
    load_x(gbeg);
    __builtin_amdgcn_sched_barrier(0);
    vm = row_mask();
    store_x();
  }
  __syncthreads();
#if TTS_SPLIT_STAMP
  st1 = __builtin_amdgcn_s_memtime();
#endif
  for (; g0 < gend; g0 += CG) {
    const bool more = g0 + CG < gend;
    TTS_SPLIT_MMAQ(a0, 0);
    TTS_SPLIT_LOADQ(a0, 2);
    if constexpr (!WHOLE) load_x(more ? g0 + CG : g0);  // unconditional (a load under a branch is waited on at once)
    TTS_SPLIT_MMAQ(a1, 1);
    TTS_SPLIT_LOADQ(a1, 3);
    for (int q = 2; q < QT; q += 2) {
      TTS_SPLIT_MMAQ(a0, q);
      TTS_SPLIT_LOADQ(a0, q + 2);
      TTS_SPLIT_MMAQ(a1, q + 1);
      TTS_SPLIT_LOADQ(a1, q + 3);
    }
#undef TTS_SPLIT_LOADQ
#undef TTS_SPLIT_MMAQ
    if constexpr (WHOLE) {
      xg += 2 * PL;  // the next group's region
    } else if (more) {
      __syncthreads();  // every wave is done with this group's tile
      store_x();
      __syncthreads();
    }
  }
  if constexpr (WHOLE) __syncthreads();  // (the epilogue reuses LDS: every wave is past its MFMAs)
  range_report(p.range_flag, rng);
#if TTS_SPLIT_STAMP
  st2 = __builtin_amdgcn_s_memtime();
#endif

  const int m_w0 = (by * 4 + wave) * 32;
  if (S == 1) {
    // epilogue through LDS: fp32 tile [BN rows][128 channels] (row stride 528 B), then a row pass
    // of 16-byte pieces -- bias, alpha, activation, residuals (prefetched before the staging
    // barrier), scale -- with coalesced row stores (fragment-shaped stores were ~1/3 of a small
    // launch's time)
    constexpr int OSR = 128 * 4 + 16;
    constexpr int NIT = BN * 32 / 256;  // 4-channel pieces per thread
    const int pc = tid & 31;            // piece: channels by*128 + 4*pc .. +3
    const int m4 = by * 128 + pc * 4;
    const bool mok = m4 < p.M;
    f32x4 res[NIT];
    // row-pass validity, bit it (rows inside F and the utterance's output length): the length
    // loads go with the residual prefetch, not one wait per row in the row pass
    int ym = 0;
    // (the record count stops short of the 0x7ffffff0 offset that lanes past M load from: they read 0.
    // At 0x7fffffff that offset was in range -- a real load 2 GB past r1, which faulted on the first
    // layer whose M is not a multiple of 128: the fp32 postnet's 80-channel last conv)
    const auto r1rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.r1 ? p.r1 : p.y), 0, p.r1 ? 0x7ffffff0 : 0, 0x00020000);
    const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias ? p.bias : reinterpret_cast<const float*>(X)), 0,
                                                       p.bias ? p.M * 4 : 0, 0x00020000);
    const auto ylrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.y_len ? p.y_len : reinterpret_cast<const int*>(X)),
                                                        0, p.y_len ? p.B * 4 : 0, 0x00020000);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rl = (tid >> 5) + it * 8;
      const int f = min(f0 + rl, F - 1);
      const int b = f / p.x_rows, r = f - b * p.x_rows;
      const int L = __builtin_amdgcn_raw_buffer_load_b32(ylrs, b * 4, 0, 0) | (p.y_len ? 0 : 0x7fffffff);
      ym |= ((int)(f0 + rl < F) & (int)(r < min(L, p.y_rows))) << it;  // (no short-circuit: no branch)
      // the first residual (0 when absent or past M), through a descriptor: an unconditional load
      const long long ro = (long long)b * p.srb + (long long)r * p.srr + m4;
      res[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r1rs, mok ? (int)(ro * 4) : 0x7ffffff0, 0, 0));
    }
    const f32x4 bias = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(brs, m4 * 4, 0, 0));  // 0 past M
    __syncthreads();  // X tile no longer read
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const f32x16 v = acc[nt] * p.w_unscale;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(smem + (nt * 32 + l31) * OSR + (wave * 32 + 8 * g + 4 * hh) * 4) =
            f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
    }
    __syncthreads();
    const bool lnf = p.ln_cnt != nullptr;  // LayerNorm in this launch (the launcher checked the shape)
    const auto yrsrc = __builtin_amdgcn_make_buffer_rsrc(p.y, 0, 0x7fffffff, 0x00020000);
    // the activation kind is dispatched once, outside the row loop (conv_xres's epilogue)
    auto row_pass = [&](auto act_c) __attribute__((always_inline)) {
      constexpr int ACT = decltype(act_c)::value;
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int rl = (tid >> 5) + it * 8;
        const int f = f0 + rl;
        if (!((ym >> it) & 1) || !mok) continue;
        const int b = f / p.x_rows, r = f - b * p.x_rows;
        f32x4 v = (*reinterpret_cast<const f32x4*>(smem + rl * OSR + pc * 16) + bias) * p.alpha;  // x * 1.0f exact
        if constexpr (ACT != ACT_NONE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], ACT, p.out_slope);
        }
        const long long ro = (long long)b * p.srb + (long long)r * p.srr + m4;
        v += res[it];
        if (p.r2) v += *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.r2) + ro);
        v *= p.out_scale;  // exact for 1.0f: no branch
        const long long yo = (long long)b * p.syb + (long long)r * p.syr + m4;
        if (lnf)  // write-through: the row tile's last block reads it (ln_rows.h)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrsrc, (int)(yo * 4), 0, 16);
        else
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.y) + yo) = v;
      }
    };
    switch (p.act_out) {
      case ACT_RELU: row_pass(ActC<ACT_RELU>{}); break;
      case ACT_TANH: row_pass(ActC<ACT_TANH>{}); break;
      case ACT_LRELU: row_pass(ActC<ACT_LRELU>{}); break;
      case ACT_SILU: row_pass(ActC<ACT_SILU>{}); break;
      default: row_pass(ActC<ACT_NONE>{}); break;
    }
#if TTS_SPLIT_STAMP
    stamp();
#endif
    // the row tile's last-arriving M block normalises its valid flat rows over all M channels
    if (lnf && ln_tile_last(p.ln_cnt + tx, nmb, reinterpret_cast<int*>(smem))) splitp_tile_ln(p, f0, BN, F, wave, lane);
    return;
  }
  // partial sums of slice sl: ws[sl][f][M] (rows past F and channels past M are not stored);
  // split_reduce(_ln)_kernel adds them in slice order
  float* P = p.ws + (long long)sl * F * p.M;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int f = f0 + nt * 32 + l31;
    if (f >= F) continue;
    const f32x16 v = acc[nt] * p.w_unscale;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int m = m_w0 + 8 * g + 4 * hh;
      if (m >= p.M) continue;
      *reinterpret_cast<f32x4*>(P + (long long)f * p.M + m) = f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
    }
  }
#if TTS_SPLIT_STAMP
  stamp();
#endif
}

// y[f][m] = epilogue(sum over slices of ws[s][f][m]) for every valid flat row (conv_epilogue's
// arithmetic: ((alpha * (acc + bias)) -> act) + r1 + r2, times out_scale)
template <int ACT>
__device__ inline void split_reduce(const ConvParams& p, int S) {
  const int F = p.B * p.x_rows;
  const int M4 = p.M / 4;
  const long long n = (long long)F * M4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int f = (int)(i / M4);
    const int m = (int)(i - (long long)f * M4) * 4;
    const int b = f / p.x_rows;
    const int r = f - b * p.x_rows;
    const int ylen = p.y_len ? min(p.y_len[b], p.y_rows) : p.y_rows;
    if (r >= ylen) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(p.ws + (long long)f * p.M + m);
    for (int s = 1; s < S; ++s) v += *reinterpret_cast<const f32x4*>(p.ws + ((long long)s * F + f) * p.M + m);
    if (p.bias) v += *reinterpret_cast<const f32x4*>(p.bias + m);
    if (p.alpha != 1.0f) v *= p.alpha;
    if constexpr (ACT != ACT_NONE) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], ACT, p.out_slope);
    }
    const long long ro = (long long)b * p.srb + (long long)r * p.srr + m;
    if (p.r1) v += *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.r1) + ro);
    if (p.r2) v += *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.r2) + ro);
    if (p.out_scale != 1.0f) v *= p.out_scale;
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.y) + (long long)b * p.syb + (long long)r * p.syr + m) = v;
  }
}

__global__ __launch_bounds__(256) void split_reduce_kernel(ConvParams p, int S) {
  switch (p.act_out) {  // the activation kind dispatched once, outside the loop
    case ACT_RELU: split_reduce<ACT_RELU>(p, S); break;
    case ACT_TANH: split_reduce<ACT_TANH>(p, S); break;
    case ACT_LRELU: split_reduce<ACT_LRELU>(p, S); break;
    case ACT_SILU: split_reduce<ACT_SILU>(p, S); break;
    default: split_reduce<ACT_NONE>(p, S); break;
  }
}

// The same reduce with the post-LN of a residual block fused (ConvParams::ln_out): one wave per
// row of M <= 512 channels, lane l owning channels l + 64 i.  Each element is summed over the
// slices in slice order with the epilogue applied as split_reduce does, then the row is
// normalised exactly as layernorm_kernel<float, 8> does it (two-pass fp32, the same lane layout
// and wave reduction, the optional second LayerNorm on the first's output), so ln_out equals
// split_reduce + launch_layernorm bit for bit on every valid row; y is not written and rows past
// an utterance are left alone (the separate LayerNorm also normalised their stale contents,
// which no consumer reads: every kernel masks rows >= len on load).
__global__ __launch_bounds__(256) void split_reduce_ln_kernel(ConvParams p, int S) {
  const int F = p.B * p.x_rows;
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= F) return;
  split_reduce_ln_row(p, S, F, f, threadIdx.x & 63);
}

// The reduce of a split-K launch whose partials are ws[S][B * p.x_rows][M] (the fp32
// conv_gemm_kernel's slices, conv_gemm.hip; the packed form below launches the same kernels):
// the post-LN fused when the row fits one wave and there is no activation before it
hipError_t split_reduce_launch(const ConvParams& p, int S, hipStream_t s, bool* ln_done) {
  const int F = p.B * p.x_rows;
  if (ln_done) *ln_done = false;
  if (p.ln_out && p.M <= 512 && p.act_out == ACT_NONE) {
    hipLaunchKernelGGL(split_reduce_ln_kernel, dim3((F + 3) / 4), dim3(256), 0, s, p, S);
    if (ln_done) *ln_done = true;
  } else {
    const long long n = (long long)F * (p.M / 4);
    const unsigned g = (unsigned)std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(split_reduce_kernel, dim3(g), dim3(256), 0, s, p, S);
  }
  return hipGetLastError();
}

constexpr int SPLIT_LDS_MAX = 76 * 1024;  // two blocks per CU

// channel group: largest power of two dividing Cin with both planes of UW utterances' rows within
// SPLIT_LDS_MAX; >= 32 (64- / 32-channel groups run 2- / 1-k-step ring slots, KQ = 2 / 1)
static int split_group(const ConvParams& p, int BN, int UW) {
  const int R = BN + (p.taps - 1) * p.dil;
  for (int cg = 512; cg >= 32; cg /= 2) {
    if (cg > p.Cin || p.Cin % cg) continue;
    if ((size_t)2 * UW * R * (cg * 2 + 16) <= (size_t)SPLIT_LDS_MAX) return cg;
  }
  return 0;
}

bool conv_split_eligible(const ConvParams& p) {
  return !p.no_split && p.wpk && p.Cin % 32 == 0 && p.M % 4 == 0 && p.nh == 1 && p.sxr % 4 == 0 && p.sxb % 4 == 0 &&
         split_group(p, 64, 1) > 0 && split_group(p, 32, 1) > 0;
}

// Per-utterance form (callers without the packed-row promise: the fp32 vocoder's resblock convs,
// an fp32 decoder's short-K GEMMs): 128 channels x 64 rows of one utterance (NT = 2) when that grid
// has at least one block per CU, else 32 rows (twice the blocks); the K order is the same.
#ifndef TTS_SPLIT_TILE_MINBLK
#define TTS_SPLIT_TILE_MINBLK 256  // 64-row tiles from this many blocks (C1: 256 beat 1024 and 0, profiles/r06t/)
#endif
static int split_tile(const ConvParams& p) {
  const long long blocks2 = (long long)((p.y_rows + 63) / 64) * ((p.M + 127) / 128) * p.B;
  return blocks2 >= TTS_SPLIT_TILE_MINBLK ? 2 : 1;
}

template <int NT>
static hipError_t launch_tile(const ConvParams& p, hipStream_t s) {
  constexpr int BN = 32 * NT;
  const int cg = split_group(p, BN, 1);
  if (!cg) return hipErrorInvalidValue;
  const size_t lds = (size_t)2 * (BN + (p.taps - 1) * p.dil) * (cg * 2 + 16);
  const int nwg = (p.y_rows + BN - 1) / BN * ((p.M + 127) / 128) * p.B;
  if (cg >= 128) hipLaunchKernelGGL((conv_split_kernel<NT, 1, 4>), dim3(nwg), dim3(256), lds, s, p, cg);
  else if (cg == 64) hipLaunchKernelGGL((conv_split_kernel<NT, 1, 2>), dim3(nwg), dim3(256), lds, s, p, cg);
  else hipLaunchKernelGGL((conv_split_kernel<NT, 1, 1>), dim3(nwg), dim3(256), lds, s, p, cg);
  return hipGetLastError();
}

// packed-row channel group: 128 when every thread's share of the (32 nt + halo)-row tile fits its
// spk_su(nt) prefetch registers and both planes fit LDS at two blocks per CU
static int packed_group(const ConvParams& p, int nt = SPK_NT) {
  const int R = 32 * nt + (p.taps - 1) * p.dil;
  const int cg = 128, rstep = 256 / (cg / 4);
  if (p.Cin % cg || (R + rstep - 1) / rstep > spk_su(nt) || (size_t)2 * R * (cg * 2 + 16) > SPLIT_LDS_MAX) return 0;
  return cg;
}

// whether a one-slice packed launch over F flat rows applies p's LayerNorm itself: a counter per
// BN-row tile, rows of M <= 512 channels, y / ln_out in the packed [B][x_rows][M] layout
static bool splitp_ln_ok(const ConvParams& p, int F, int BN) {
  if (!p.ln_cnt || !(p.ln_out || p.ln_lin_out) || p.M > 512) return false;
  // small grids: the tile's LayerNorm tail is on the critical path (the same bits either way)
  if (sw(SW_LN_FUSE) != 7 && (long long)((F + BN - 1) / BN) * ((p.M + 127) / 128) < TTS_LN_FUSE_MINBLK)
    return false;  // (TTS_LN_FUSE=7: every eligible launch, tests)
  return (F + BN - 1) / BN <= p.ln_cnt_n;
}

// packed-row form: usable when the caller promises enough masked rows after every utterance for
// this conv's taps, the row stride is a multiple of 32 rows, and the buffers are contiguous
static bool packed_ok(const ConvParams& p) {
  const int right = (p.taps - 1) * p.dil - p.pad;
  return p.rows_pad > 0 && p.rows_pad >= p.pad && p.rows_pad >= right && p.x_rows == p.y_rows &&
         p.x_rows % 32 == 0 && p.sxb == (long long)p.x_rows * p.sxr && p.syb == (long long)p.y_rows * p.syr &&
         (!(p.r1 || p.r2) || p.srb == (long long)p.y_rows * p.srr) && !p.up_s && p.M % 4 == 0;
}

// split-K slices from the layer shape only (batch-independent accumulation order): one slice per
// ~1152 of K (taps * Cin), whole channel groups each, while the workspace holds the partials
static int split_slices(const ConvParams& p, int cg) {
  const int groups = p.Cin / cg;
  int S = std::max(1, std::min(groups, p.taps * p.Cin / 1152));
  while (S > 1 && groups % S) --S;
  const long long need = (long long)S * p.B * p.x_rows * p.M * 4;
  return (S > 1 && p.ws && need <= p.ws_bytes) ? S : 1;
}

long long conv_split_ws_bytes(int taps, int Cin, int M, int rows) {
  ConvParams q = conv_params_default();
  q.taps = taps; q.Cin = Cin; q.M = M; q.B = 1; q.x_rows = rows; q.ws = reinterpret_cast<float*>(16);
  q.ws_bytes = 1LL << 62;
  const int cg = packed_group(q);
  return cg ? (long long)split_slices(q, cg) * rows * M * 4 : 0;
}

// The packed kernel and the reduce + LayerNorm kernels it hands to address y, the residuals and
// the split-K partials through buffer descriptors with 32-bit byte offsets (num_records
// 0x7fffffff): past 2 GiB a load would read 0 and a store would be dropped.  Launches whose
// arrays reach that take the per-utterance kernel (64-bit pointer arithmetic) instead.
static bool packed_i32_ok(const ConvParams& p, int S) {
  const long long lim = 0x7fffff00LL;
  const long long F = (long long)p.B * p.x_rows;
  if ((long long)S * F * p.M * 4 >= lim) return false;             // split-K partials ws[S][F][M]
  if ((long long)p.B * p.syb * 4 >= lim) return false;             // y / ln_out
  if ((p.r1 || p.r2) && (long long)p.B * p.srb * 4 >= lim) return false;  // residuals
  return true;
}

static thread_local int g_split_kernels = 1;
int conv_split_last_kernels() { return g_split_kernels; }

hipError_t conv_split_launch(const ConvParams& p, hipStream_t s, bool* ln_done) {
  if (ln_done) *ln_done = false;
  g_split_kernels = 1;
  if (packed_ok(p)) {
    const int cg = packed_group(p);
    if (cg && packed_i32_ok(p, split_slices(p, cg))) {
      const int S = split_slices(p, cg);
      const int gps = p.Cin / cg / S;
      const int F = p.B * p.x_rows;
      // 32-row tiles where the 64-row grid would leave most CUs idle (the batch-8 encoder's
      // M = 384 projections: 60 blocks): twice the blocks, each with half the staging and MFMA
      // latency.  A row's K order does not depend on the tile: bit-identical.
      // 128-row tiles where even they fill the chip (TTS_SPLIT_NT4_MINBLK blocks: the batch-32
      // FFN / Q|K|V / pointwise-1 GEMMs): each weight quad feeds twice the MFMAs, and X is staged
      // once per 128 rows.  TTS_SPLIT_NT1: 0 = 64-row tiles, 1 = 32-row, 4 = 128-row wherever
      // eligible; unset = by grid.
      const int mbs = (p.M + 127) / 128 * S;
      const int ntsw = sw(SW_SPLIT_NT1);
      int nt = ntsw == 1 || (ntsw < 0 && (F + 63) / 64 * mbs < TTS_SPLIT_NT1_MAXBLK) ? 1 : SPK_NT;
      if (packed_group(p, 4) && (ntsw == 4 || (ntsw < 0 && (long long)(F + 127) / 128 * mbs >= TTS_SPLIT_NT4_MINBLK))) nt = 4;
      const int nwg = (F + 32 * nt - 1) / (32 * nt) * mbs;
      const size_t lds = std::max((size_t)2 * (32 * nt + (p.taps - 1) * p.dil) * (cg * 2 + 16),
                                  (size_t)32 * nt * (128 * 4 + 16));  // X planes / epilogue tile
      // one block per CU or fewer: stage the K slice's groups at once (no restaging; bit-identical)
      const int ngs = gps;  // groups per slice
      const bool whole = sw(SW_SPLIT_WHOLE) != 0 && ngs <= SPK_WG && nwg <= TTS_SPLIT_WHOLE_MAXBLK && nt < 4;
      const size_t ldsw = whole ? std::max((size_t)ngs * 2 * (32 * nt + (p.taps - 1) * p.dil) * (cg * 2 + 16),
                                           (size_t)32 * nt * (128 * 4 + 16))
                                : lds;
      ConvParams q = p;
      // the kernel's LayerNorm switch: its epilogue applies the post-LN in one-slice launches
      // (ln_rows.h hand-off); split-K launches reduce and normalise in split_reduce_ln_kernel.
      // (Round 4 also built an in-launch split-K reduce; its run-to-run bit difference did not
      // reproduce -- profiles/r04c_splitk_stability.txt -- and it was never faster, so round 6
      // removed it.)
      bool fuse = splitp_ln_ok(p, F, 32 * nt) && S == 1;
      if (sw(SW_LN_FUSE) > 1 && sw(SW_LN_FUSE) != 7 && sw(SW_LN_FUSE) != 3) fuse = false;  // (bisection: 3 = one slice)
      if (!fuse) q.ln_cnt = nullptr;
      if (whole && ldsw <= 160 * 1024) {
        if (nt == 1) hipLaunchKernelGGL((conv_splitp_kernel<true, 1>), dim3(nwg), dim3(256), ldsw, s, q, cg, S, gps);
        else hipLaunchKernelGGL((conv_splitp_kernel<true, SPK_NT>), dim3(nwg), dim3(256), ldsw, s, q, cg, S, gps);
      } else {
        if (nt == 1) hipLaunchKernelGGL((conv_splitp_kernel<false, 1>), dim3(nwg), dim3(256), lds, s, q, cg, S, gps);
        else if (nt == 4) hipLaunchKernelGGL((conv_splitp_kernel<false, 4>), dim3(nwg), dim3(256), lds, s, q, cg, S, gps);
        else hipLaunchKernelGGL((conv_splitp_kernel<false, SPK_NT>), dim3(nwg), dim3(256), lds, s, q, cg, S, gps);
      }
      if (q.ln_cnt) {
        if (ln_done) *ln_done = true;
        return hipGetLastError();
      }
      if (S > 1 && p.ln_out && p.M <= 512 && p.act_out == ACT_NONE) {
        hipLaunchKernelGGL(split_reduce_ln_kernel, dim3((F + 3) / 4), dim3(256), 0, s, p, S);
        g_split_kernels = 2;
        if (ln_done) *ln_done = true;
      } else if (S > 1) {
        const long long n = (long long)F * (p.M / 4);
        const unsigned g = (unsigned)std::min<long long>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(split_reduce_kernel, dim3(g), dim3(256), 0, s, p, S);
        g_split_kernels = 2;
      }
      return hipGetLastError();
    }
  }
  return split_tile(p) == 2 ? launch_tile<2>(p, s) : launch_tile<1>(p, s);
}

#if TTS_SPLIT_STAMP
extern "C" int tts_debug_split_target(int M, int Cin, int taps) {
  const int t[3] = {M, Cin, taps};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_split_stamp_target), t, sizeof(t)) == hipSuccess ? 0 : -1;
}
extern "C" int tts_debug_split_stamps(unsigned long long* host, long long words) {
  const long long n = words < (1LL << 18) ? words : (1LL << 18);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_split_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace tts
