// Fused relative-position self-attention of the conformer layers (HF:396-452), flash style:
//
//   S[i][j] = (Qu[i] . K[j] + Qv[i] . R[i - j]) / sqrt(dk),   Qu = q + pos_bias_u, Qv = q + pos_bias_v
//   O[i]    = softmax_j<len(S[i]) . V           R[m] = linear_pos(pe)[rel = m]  (HF:419)
//
// replacing four launches per layer (Qu.K^T and Qv.P^T head-batched GEMMs, the shift +
// masked softmax, P.V) that moved three [B][H][T][T..2T] score matrices through HBM.  The
// matrix_bd "shift" (HF:381-393) becomes an index map: for a 16-query x 32-key step the
// needed R rows m = i - j span 47 consecutive rows of the precomputed table, so the wave
// computes G = Qv . R_win^T (3 16x16 tiles) and gathers G[q][slot(q, key)] through a
// per-wave LDS scratch.
//
// Block = (utterance, head, 64 queries); 4 waves x 16 queries; keys in 32-key steps with
// an online softmax.  MFMA v_mfma_f32_16x16x32_{bf16,f16}, every product transposed so the
// softmax statistics, P and O share one lane <-> query map (query = lane & 15):
//   S^T = K . Qu^T     A = K rows (LDS),       B = Qu^T (registers, whole dk)
//   G^T = R . Qv^T     A = R window (LDS),     B = Qv^T (registers)
//   O^T += Vt . P^T    A = Vt (LDS, V rows read transposed), B = P^T: the lane's own 8 probabilities
// P^T's k index is permuted (keys 4g..4g+3, 16+4g..16+4g+3 for lane group g) and the Vt
// fragment is read with the same permutation, so no cross-lane move is needed.
//
// V is staged as it lies in QKV, [32 keys][dk] rows like K, and the A fragment of O^T is taken
// with two ds_read_b64_tr_b16 per 16-row tile: lane group g reads the 4 x 16 block (keys 4g..4g+3
// or 16+4g..16+4g+3, channels 16t..16t+15) and lane q receives channel 16t + q of those 4 keys --
// exactly the Vt row piece the lane needs.  (Round 4 wrote Vt with a transpose launch per layer.)
// LDS images (MI355X_MICROARCH.md §LDS bank model), all conflict-free:
//   * K / V / R rows at a stride of dk*2 + 32 bytes (dk/8 + 2 16-byte slots, = 2 mod 4): the
//     ds_read_b128 fragment reads (16 rows x 2 lane groups per 16-lane bank group) take 16
//     distinct slots; the odd-slot stride of round 4 (dk*2 + 16) was 2-way there;
//   * the transposed V reads: 8 keys x 4 column pieces per 32-lane half on 64 distinct banks;
//   * the per-wave G scratch (48 slots x 16 queries, f32): slot s is stored at row
//     s ^ ((s >> 2) & 1), so the two lane groups of a 32-lane half (slots 4 apart) land in
//     opposite bank halves for the writes and for the diagonal gather.
//
// Three forms share that schedule: rel_attn_kernel (16-bit stacks: the decoder, and the whole
// model with encoder_precision "fast"), rel_attn_split_kernel (fp32 stacks of a 16-bit model:
// the exact-duration encoder, each product as three f16 MFMAs) and rel_attn_f32_kernel (fp32
// models, v_mfma_f32_16x16x4_f32).
#include <type_traits>

#include "acoustic_kernels.h"
#include "common.h"
#include "ln_rows.h"
#include "mrf_tile.h"
#include "switches.h"

namespace tts {

namespace {

// Row statistics over the 4 lanes of a query (q, q+16, q+32, q+48) with gfx950's VALU lane
// swaps instead of LDS-routed ds_bpermute: each swap returns the lane's own value in one result
// and its partner's in the other, so max / sum of the two is the xor-16 / xor-32 reduction (the
// same operands, so bit-identical to the shuffle form)
__device__ inline float at_xor16_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ inline float at_xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ inline float at_xor16_sum(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float at_xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// 2^x on v_exp_f32 (arguments <= 0 here; -inf -> 0), without exp2f's denormal-range fixup
__device__ inline float at_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// K / V / R row stride in LDS (bytes): dk/8 + 2 16-byte slots for 16-bit rows (see the header),
// dk + 4 dwords for fp32 rows (the f32 kernel's scalar V reads: lane groups 16 dwords apart)
template <typename T>
constexpr int at_kr(int dk) { return sizeof(T) == 2 ? dk * 2 + 32 : dk * 4 + 16; }
// G scratch row of slot s (see the header)
__device__ inline int at_gslot(int s) { return s ^ ((s >> 2) & 1); }
// byte offset, within the V rows, of lane (g, q)'s transposed read of tile 0's keys 4g .. 4g + 3:
// lane 4a + c of the 16-lane group supplies key 4g + a, channels 4c .. 4c + 3
__device__ inline int at_tr_addr(int kr, int g, int q) { return (4 * g + (q >> 2)) * kr + (q & 3) * 8; }
// ds_read_b64_tr_b16 (all 64 lanes active: the loop has no divergence)
__device__ inline uint2 at_tr16(const char* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)const_cast<char*>(p));
  return __builtin_bit_cast(uint2, v);
}

constexpr int AT_BQ = 64;   // queries per block
constexpr int AT_BK = 32;   // keys per step
constexpr int AT_RW = AT_BQ + AT_BK;  // R window rows per block (95 used)
// fp32 attention key chunk (keys per block; rel_attn_f32_kernel), TTS_ATTN_F32_KC (0: off).
// C1 (same box, profiles/r06ab/): 64 beat 128 by 40-75 us per sentence and 256 by ~170; 32 ties 64
constexpr int AT_F32_KC = 64;
// Key chunk of the split-precision form (the exact encoder), a multiple of AT_BK; 0: one pass.
// A build-time choice (A/B variant builds): see DESIGN §11 for the batch-8 / batch-32 trade.
#ifndef TTS_ATTN_SPLIT_KC
#define TTS_ATTN_SPLIT_KC 0
#endif
static_assert(TTS_ATTN_SPLIT_KC % AT_BK == 0, "split key chunk: whole key steps");
// Lazy online-softmax rescale (16-bit kernel): a row's reference max moves only when a step's
// max exceeds it by more than AT_LAZY (log2 units), so P = 2^(s - m) stays <= 2^AT_LAZY (f16 /
// bf16 hold it exactly as well as any P <= 1: same relative precision) and the O^T rescale of
// DT tiles is skipped on every step where no row of the wave moved -- after the first steps,
// nearly all.  0: eager (a row moves whenever its max grows; the skipped multiplies are by
// exactly 1, so the result equals the eager form's bits).
#ifndef TTS_ATTN_LAZY
#define TTS_ATTN_LAZY 8
#endif
constexpr float AT_LAZY = TTS_ATTN_LAZY;

// KH = 2: 8 waves, the block's keys split into two groups of whole 32-key steps, one per 4
// waves (each group with its own K / Vt / R staging), merged through LDS at the end -- twice
// the waves per SIMD where the grid has about one block per CU.  The split point depends only
// on the utterance's length, so a row's result does not depend on the batch.
template <typename T, int DK, int KH>
__global__ __launch_bounds__(256 * KH, KH == 1 ? 2 : 1) void rel_attn_kernel(const float* __restrict__ pu, const float* __restrict__ pv,
                                                         const T* __restrict__ qkv,
                                                         const T* __restrict__ ptab, const int* __restrict__ lens,
                                                         int Tp, int D, int H, int rmax, float scale,
                                                         T* __restrict__ out, int nqb, int nbatch) {
  using MF = Mfma16<T>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int KS = DK / 32;         // k-steps over dk
  constexpr int DT = DK / 16;         // 16-row tiles of dk (O^T)
  constexpr int KR = at_kr<T>(DK);    // K / V / R row stride in LDS (bytes)
  constexpr int HALF = 2 * AT_BK * KR + AT_RW * KR;  // one key group's staging bytes
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int kh = KH > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 8) : 0;  // key group
  char* Ks = smem + kh * HALF;                      // [32 keys][DK]
  char* Vs = Ks + AT_BK * KR;                       // [32 keys][DK]
  char* Rs = Vs + AT_BK * KR;                       // [96 slots][DK]
  float* Gs = reinterpret_cast<float*>(smem + KH * HALF);  // [KH][4 waves][48 slots][16 q]

  // 1-D grid, XCD-grouped: the query blocks of one (utterance, head) -- which all stream the
  // same K / Vt / R rows -- run on one XCD, so those rows come from its L2 after the first
  int bh, qb;
  if (!xcd_tile(nqb, H * nbatch, bh, qb)) return;
  const int b = bh / H, h = bh - b * H;
  const int i0 = qb * AT_BQ;
  const int len = lens[b];
  if (i0 >= len) return;
  const int tid = threadIdx.x & 255, lane = tid & 63;  // thread / wave within the key group
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 15, g = lane >> 4;
  const int i0w = i0 + 16 * w;
  const long long rowD = D;
  // this group's keys: whole 32-key steps, the same step count for both groups
  const int khalf = KH > 1 ? (len + 2 * AT_BK - 1) / (2 * AT_BK) * AT_BK : len;
  const int kbeg = kh * khalf, kend = min(len, kbeg + khalf);
  // this lane's query row (clamped into the buffer; rows >= len are computed, not stored)
  const int iq = min(i0w + q, Tp - 1);
  // Qu = q + pos_bias_u, Qv = q + pos_bias_v (HF:420-423), formed here from the q slice of
  // QKV and rounded to T once, exactly as the separate pos_bias_kernel materialised them
  Frag bu[KS], bv[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int c = h * DK + ks * 32 + 8 * g;
    const uint4 qw = *reinterpret_cast<const uint4*>(qkv + ((long long)b * Tp + iq) * 3 * rowD + c);
    f32x4 q0, q1;
    pair_ld8<T>(reinterpret_cast<const T*>(&qw), q0, q1);
    const f32x4 u0 = *reinterpret_cast<const f32x4*>(pu + c), u1 = *reinterpret_cast<const f32x4*>(pu + c + 4);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(pv + c), v1 = *reinterpret_cast<const f32x4*>(pv + c + 4);
    bu[ks] = __builtin_bit_cast(Frag, pack8<T>(q0 + u0, q1 + u1));
    bv[ks] = __builtin_bit_cast(Frag, pack8<T>(q0 + v0, q1 + v1));
  }
  f32x4 oacc[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) oacc[t] = f32x4{};
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = scale * 1.4426950408889634f;  // scores in log2 units
  float* gw = Gs + (kh * 4 + w) * 48 * 16;

  // Staging.  K[j0 .. j0+32) and Vt[:, j0 .. j0+32) per step; the R window (block slot sb <->
  // m = i0 - j0 - 31 + sb, 96 rows) lives in a 96-row ring indexed by m mod 96: a step shifts the
  // window by 32, so only the 32 rows entering it are loaded, into the slots of the 32 that left.
  // Loads for step s+1 are issued before step s's MFMAs (registers, pinned there by a scheduling
  // barrier) and written to LDS after the barrier that ends step s -- on every step, the last one
  // included, so the loads are consumed unconditionally (consumed only under a branch, they were
  // sunk into it and their latency was exposed once per step).
  // The per-step loads go through buffer descriptors whose base moves with j0 (scalar arithmetic)
  // and whose range ends at the utterance's last key (K rows >= len read 0: no clamp, no mask),
  // at the end of the (utterance, head) Vt block, and at the position table's last row; each
  // thread's byte offsets, LDS destinations and ring slots are fixed or stepped by one unsigned
  // min, so the staging costs no index arithmetic per step (it was ~40 % of the loop's VALU).
  constexpr int KP = AT_BK * (DK / 8) / 256;   // 16-byte pieces per thread: K, V, new R rows
  static_assert(AT_BK * (DK / 8) % 256 == 0, "staging split");
  constexpr unsigned RING = AT_RW * KR;        // R ring bytes
  auto rslot = [](int m) { const int r = m % AT_RW; return r < 0 ? r + AT_RW : r; };
  auto rrow = [&](int m) { return min(max(rmax - 1 - m, 0), 2 * rmax - 1); };
  // next ring slot, 32 rows back (mod 96), of a byte address slot * KR + col (col < KR)
  auto ring_back = [](unsigned a) { return min(a - AT_BK * KR, a + (AT_RW - AT_BK) * KR); };
  const int rowB = 3 * D * (int)sizeof(T);     // QKV row bytes
  int kofs[KP], rofs[KP];
  unsigned kdst[KP], rdst[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    const int p = tid + 256 * i;
    const int r = p / (DK / 8), c = p - r * (DK / 8);
    kofs[i] = r * rowB + c * 16;  // K and V rows: the same pieces of the row's two slices
    kdst[i] = r * KR + c * 16;
    // position-table row row0 + r <-> m = i0 - j0 - r; the first prefetch is for j0 = kbeg + 32
    rofs[i] = r * D * (int)sizeof(T) + c * 16;
    rdst[i] = rslot(i0 - kbeg - AT_BK - r) * KR + c * 16;
  }
  u32x4 pkv[KP], pvt[KP], prr[KP];
  auto load_kv = [&](int j0) __attribute__((always_inline)) {
    // K and V rows >= len read 0 (the descriptors' range ends at the utterance's last key):
    // those keys are masked out of the softmax, and V = 0 keeps 0 * V finite
    const T* krow = qkv + ((long long)b * Tp + j0) * 3 * rowD + D + h * DK;
    const auto kr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(krow), 0, max(len - j0, 0) * rowB, 0x00020000);
    const auto vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(krow + D), 0, max(len - j0, 0) * rowB, 0x00020000);
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      pkv[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(kr, kofs[i], 0, 0));
      pvt[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vr, kofs[i], 0, 0));
    }
  };
  auto load_r = [&](int j0) __attribute__((always_inline)) {
    // R rows entering the window: table rows rmax - 1 - i0 + j0 + [0, 32) (m = i0 - j0 - [0, 32));
    // rows past the table's last (m < -(rmax - 1), only masked keys use them) read 0
    const int row0 = rmax - 1 - i0 + j0;  // >= 0: i0 < len <= Tm <= rmax
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(ptab + (long long)row0 * rowD + h * DK), 0,
                                                      max(rmax + i0 - j0, 0) * D * (int)sizeof(T), 0x00020000);
#pragma unroll
    for (int i = 0; i < KP; ++i)
      prr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, rofs[i], 0, 0));
  };
  auto write_kv = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      *reinterpret_cast<u32x4*>(Ks + kdst[i]) = pkv[i];
      *reinterpret_cast<u32x4*>(Vs + kdst[i]) = pvt[i];
    }
  };
  auto write_r = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      *reinterpret_cast<u32x4*>(Rs + rdst[i]) = prr[i];
      rdst[i] = ring_back(rdst[i]);
    }
  };
  // first step: the whole 96-row R window
  for (int p = tid; p < AT_RW * (DK / 8); p += 256) {
    const int sb = p / (DK / 8), c = p - sb * (DK / 8);
    const int m = i0 - kbeg - (AT_BK - 1) + sb;
    *reinterpret_cast<uint4*>(Rs + rslot(m) * KR + c * 16) =
        *reinterpret_cast<const uint4*>(ptab + (long long)rrow(m) * rowD + h * DK + c * 8);
  }
  load_kv(kbeg);
  write_kv();
  __syncthreads();
  // this lane's R fragment rows: slot of m = i0w - j0 - 31 + q (+ 16 t per tile), plus its column
  unsigned ra = rslot(i0w - kbeg - (AT_BK - 1) + q) * KR + 16 * g;
  const int vta = at_tr_addr(KR, g, q);  // this lane's transposed-read address in the V rows (tile 0)

  // one 32-key step; MASK: a step with keys past the group's end
  auto key_step = [&](const int j0, auto MASK) __attribute__((always_inline)) {
    load_kv(j0 + AT_BK);  // in flight during this step's MFMAs (the last step's are written, unused)
    load_r(j0 + AT_BK);
    __builtin_amdgcn_sched_barrier(0);
    // S^T tiles (keys 16 kt + 4g + e, query q) and G^T tiles (slots 16 t + 4g + e)
    f32x4 sacc[2] = {f32x4{}, f32x4{}};
    f32x4 gacc[3] = {f32x4{}, f32x4{}, f32x4{}};
    unsigned rt[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const unsigned y = ra + 16 * t * KR;
      rt[t] = t ? min(y, y - RING) : y;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const Frag a = *reinterpret_cast<const Frag*>(Ks + (16 * kt + q) * KR + (ks * 32 + 8 * g) * 2);
        sacc[kt] = MF::mma(a, bu[ks], sacc[kt]);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const Frag a = *reinterpret_cast<const Frag*>(Rs + rt[t] + ks * 64);
        gacc[t] = MF::mma(a, bv[ks], gacc[t]);
      }
    }
    ra = ring_back(ra);
    // G^T -> wave scratch [slot][q]; gather G[q][q - key + 31] for the lane's 8 keys
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) gw[at_gslot(16 * t + 4 * g + e) * 16 + q] = gacc[t][e];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's scratch writes landed
    __builtin_amdgcn_wave_barrier();
    float sv[8];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = 16 * kt + 4 * g + e;
        const float bd = gw[at_gslot(q - kk + AT_BK - 1) * 16 + q];
        sv[4 * kt + e] = (sacc[kt][e] + bd) * sl2;
      }
    __builtin_amdgcn_wave_barrier();
    if constexpr (decltype(MASK)::value) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (j0 + 16 * kt + 4 * g + e >= kend) sv[4 * kt + e] = -INFINITY;
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) mloc = fmaxf(mloc, sv[e]);
    mloc = at_xor32_max(at_xor16_max(mloc));
    // (m_run = -inf: -inf + AT_LAZY = -inf, so the first step with a key moves the row)
    const bool grow = mloc > m_run + AT_LAZY;
    const float m_new = grow ? mloc : m_run;
    // a step with every key masked (the second key group of a short utterance) keeps m = -inf:
    // exponents are then taken against 0, so alpha and P stay 0 instead of NaN
    const float m_ref = KH > 1 && m_new == -INFINITY ? 0.f : m_new;
    const float alpha = at_exp2(m_run - m_ref);  // m_run = -inf on the first step: alpha = 0
    // alpha is exactly 1 for a row that did not move (or 0 with O^T and l still 0): the rescale
    // runs only when some row of the wave moved
    const bool rescale = __builtin_amdgcn_ballot_w64(grow) != 0;
    float lsum = 0.f;
    f32x4 pe0, pe1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pe0[e] = at_exp2(sv[e] - m_ref);
      pe1[e] = at_exp2(sv[4 + e] - m_ref);
    }
    // normalise with the rounded probabilities P.V uses (keys in the order e = 0 .. 7), read back
    // from the packed P fragment (the same round-to-nearest conversion, done once)
    uint4 pk = pack8<T>(pe0, pe1);
    // (keeps the unpack below on these bits: else the compiler converts each value again)
    asm volatile("" : "+v"(pk.x), "+v"(pk.y), "+v"(pk.z), "+v"(pk.w));
    const Frag bp = __builtin_bit_cast(Frag, pk);
    {
      float pr[8];
      ln_unpack8<T>(pk, pr);
#pragma unroll
      for (int e = 0; e < 8; ++e) lsum += pr[e];
    }
    lsum = at_xor32_sum(at_xor16_sum(lsum));
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    if (rescale) {
#pragma unroll
      for (int t = 0; t < DT; ++t) oacc[t] *= alpha;
    }
    // O^T += Vt . P^T with the permuted key order of bp: the Vt fragment by transposed reads
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const uint2 lo = at_tr16(Vs + vta + t * 32);
      const uint2 hi = at_tr16(Vs + vta + 16 * KR + t * 32);
      const uint4 av = uint4{lo.x, lo.y, hi.x, hi.y};
      oacc[t] = MF::mma(*reinterpret_cast<const Frag*>(&av), bp, oacc[t]);
    }
    __syncthreads();  // every wave is done with this step's K / Vt and the leaving R rows
    write_kv();
    write_r();
    __syncthreads();
  };
  // steps whose 32 keys all lie before the group's end run without the per-key compares; the
  // rest (KH = 1: at most the last; KH = 2: the second group of a short utterance may have several
  // past its end) with them
  const int nsteps = (khalf + AT_BK - 1) / AT_BK;  // (KH = 1: khalf = len)
  const int nfull = min(nsteps, max(0, (kend - kbeg) / AT_BK));
  for (int st = 0; st < nfull; ++st) key_step(kbeg + st * AT_BK, std::false_type{});
  for (int st = nfull; st < nsteps; ++st) key_step(kbeg + st * AT_BK, std::true_type{});
  if constexpr (KH > 1) {
    // merge the two key groups: group 1 leaves (m, l, O^T) in LDS, group 0 rescales both
    constexpr int MS = 2 + 4 * DT + 2;  // floats per lane (padded)
    float* mg = reinterpret_cast<float*>(smem) + (w * 64 + lane) * MS;
    __syncthreads();  // staging tiles no longer read
    if (kh == 1) {
      mg[0] = m_run;
      mg[1] = l_run;
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) mg[2 + 4 * t + e] = oacc[t][e];
    }
    __syncthreads();
    if (kh == 1) return;
    const float mb = mg[0], lb = mg[1];
    const float mm = fmaxf(m_run, mb);
    const float sa = m_run == -INFINITY ? 0.f : at_exp2(m_run - mm);
    const float sb = mb == -INFINITY ? 0.f : at_exp2(mb - mm);
    l_run = l_run * sa + lb * sb;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) oacc[t][e] = oacc[t][e] * sa + mg[2 + 4 * t + e] * sb;
  }
  // O[i][h*dk + d] = O^T[d][i] / l
  const int i = i0w + q;
  if (i < len) {
    const float inv = 1.f / l_run;
    T* orow = out + ((long long)b * Tp + i) * rowD + h * DK;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const f32x4 v = oacc[t] * inv;
      const T o4[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
      *reinterpret_cast<uint2*>(orow + 16 * t + 4 * g) = *reinterpret_cast<const uint2*>(o4);
    }
  }
}

// fp32 form (the exact-duration encoder, acoustic.cpp): the same flash schedule and index map
// on v_mfma_f32_16x16x4_f32 (exact f32 products, fp32 accumulation -- the unfused fp32 path's
// arithmetic up to summation order), P kept in fp32.  The dk index of each 4-deep k-step is
// permuted (lane group g holds d = 16u + 4g + e for k-step 4u + e) so every A fragment of four
// k-steps is one 16-byte LDS read and every Q fragment one 16-byte global load.  LDS holds fp32
// K / Vt / R (140 KB): one block per CU.
//
// Key chunks (kc > 0, fp32 models): block (query tile, chunk c) runs keys [c kc, min(len, (c+1) kc))
// and writes its unnormalised O^T rows with the row's (max, sum) to `po` / `pml`;
// rel_attn_merge_kernel combines an utterance's ceil(len / kc) chunks.  A batch-1 decoder
// (C1: 7 query tiles x 2 heads = 14 blocks, one wave per SIMD on 14 of 256 CUs) gets
// ceil(len / kc) times the blocks (98 at kc = 64), each with 1 / that of the serial key loop.  The chunking
// depends on the utterance's length only (batch invariant), and a one-chunk row merges to the
// direct form's bits (x * exp2(0) = x, then the same O * (1 / l)).
template <int DK>
__global__ __launch_bounds__(256, 1) void rel_attn_f32_kernel(const float* __restrict__ pu, const float* __restrict__ pv,
                                                             const float* __restrict__ qkv,
                                                             const float* __restrict__ ptab, const int* __restrict__ lens,
                                                             int Tp, int D, int H, int rmax, float scale,
                                                             float* __restrict__ out, int nqb, int nbatch,
                                                             int kc, int nks, float* __restrict__ po,
                                                             float* __restrict__ pml) {
  constexpr int KU = DK / 16;         // 16-wide dk chunks (4 k-steps each); also O^T tiles
  constexpr int KR = at_kr<float>(DK);  // K / V / R row stride in LDS (bytes; odd 16-byte slots)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;                                  // [32 keys][DK]
  char* Vs = Ks + AT_BK * KR;                       // [32 keys][DK]
  char* Rs = Vs + AT_BK * KR;                       // [96 slots][DK]
  float* Gs = reinterpret_cast<float*>(Rs + AT_RW * KR);  // [4 waves][48 slots][16 q]

  int bh, qt;
  if (!xcd_tile(nqb * nks, H * nbatch, bh, qt)) return;
  const int kcn = qt / nqb, qb = qt - kcn * nqb;  // key chunk, query tile
  const int b = bh / H, h = bh - b * H;
  const int i0 = qb * AT_BQ;
  const int len = lens[b];
  if (i0 >= len) return;
  const int kbeg = kcn * kc;  // (kc = 0: one chunk, all keys)
  if (kbeg >= len) return;
  const int kend = kc > 0 ? min(len, kbeg + kc) : len;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 15, g = lane >> 4;
  const int i0w = i0 + 16 * w;
  const long long rowD = D;
  const int iq = min(i0w + q, Tp - 1);
  // Qu = q + pos_bias_u, Qv = q + pos_bias_v (HF:420-423) in fp32, as pos_bias_kernel<float>
  f32x4 bu[KU], bv[KU];
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    const int c = h * DK + 16 * u + 4 * g;
    const f32x4 qv = *reinterpret_cast<const f32x4*>(qkv + ((long long)b * Tp + iq) * 3 * rowD + c);
    bu[u] = qv + *reinterpret_cast<const f32x4*>(pu + c);
    bv[u] = qv + *reinterpret_cast<const f32x4*>(pv + c);
  }
  f32x4 oacc[KU];
#pragma unroll
  for (int t = 0; t < KU; ++t) oacc[t] = f32x4{};
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = scale * 1.4426950408889634f;
  float* gw = Gs + w * 48 * 16;

  // staging as the 16-bit kernel: loads for step s+1 in flight during step s, written after
  // the barrier that ends it (every step), masks applied at the write
  constexpr int KP = AT_BK * (DK / 4) / 256;  // 16-byte pieces per thread: K, V, new R rows
  static_assert(AT_BK * (DK / 4) % 256 == 0, "staging split");
  auto rslot = [](int m) { const int r = m % AT_RW; return r < 0 ? r + AT_RW : r; };
  auto rrow = [&](int m) { return min(max(rmax - 1 - m, 0), 2 * rmax - 1); };
  f32x4 pkv[KP], pvt[KP], prr[KP];
  auto load_kv = [&](int j0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int p = tid + 256 * i;
      const int r = p / (DK / 4), c = p - r * (DK / 4);
      const float* kv = qkv + ((long long)b * Tp + min(j0 + r, Tp - 1)) * 3 * rowD + D + h * DK + c * 4;
      pkv[i] = *reinterpret_cast<const f32x4*>(kv);
      pvt[i] = *reinterpret_cast<const f32x4*>(kv + D);
    }
  };
  auto load_r = [&](int j0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int p = tid + 256 * i;
      const int r = p / (DK / 4), c = p - r * (DK / 4);
      prr[i] = *reinterpret_cast<const f32x4*>(ptab + (long long)rrow(i0 - j0 - (AT_BK - 1) + r) * rowD + h * DK + c * 4);
    }
  };
  auto write_kv = [&](int j0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int p = tid + 256 * i;
      const int r = p / (DK / 4), c = p - r * (DK / 4);
      *reinterpret_cast<f32x4*>(Ks + r * KR + c * 16) = j0 + r < kend ? pkv[i] : f32x4{};
      *reinterpret_cast<f32x4*>(Vs + r * KR + c * 16) = j0 + r < kend ? pvt[i] : f32x4{};  // 0 * V finite
    }
  };
  auto write_r = [&](int j0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int p = tid + 256 * i;
      const int r = p / (DK / 4), c = p - r * (DK / 4);
      *reinterpret_cast<f32x4*>(Rs + rslot(i0 - j0 - (AT_BK - 1) + r) * KR + c * 16) = prr[i];
    }
  };
  for (int p = tid; p < AT_RW * (DK / 4); p += 256) {
    const int sb = p / (DK / 4), c = p - sb * (DK / 4);
    const int m = i0 - kbeg - (AT_BK - 1) + sb;
    *reinterpret_cast<f32x4*>(Rs + rslot(m) * KR + c * 16) =
        *reinterpret_cast<const f32x4*>(ptab + (long long)rrow(m) * rowD + h * DK + c * 4);
  }
  load_kv(kbeg);
  write_kv(kbeg);
  __syncthreads();

  for (int j0 = kbeg; j0 < kend; j0 += AT_BK) {
    load_kv(j0 + AT_BK);
    load_r(j0 + AT_BK);
    __builtin_amdgcn_sched_barrier(0);
    const int mbw = i0w - j0 - (AT_BK - 1);
    f32x4 sacc[2] = {f32x4{}, f32x4{}};
    f32x4 gacc[3] = {f32x4{}, f32x4{}, f32x4{}};
    int rs[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) rs[t] = rslot(mbw + 16 * t + q) * KR;
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      f32x4 a[5];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) a[kt] = *reinterpret_cast<const f32x4*>(Ks + (16 * kt + q) * KR + (16 * u + 4 * g) * 4);
#pragma unroll
      for (int t = 0; t < 3; ++t) a[2 + t] = *reinterpret_cast<const f32x4*>(Rs + rs[t] + (16 * u + 4 * g) * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) sacc[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kt][e], bu[u][e], sacc[kt], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 3; ++t) gacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2 + t][e], bv[u][e], gacc[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) gw[at_gslot(16 * t + 4 * g + e) * 16 + q] = gacc[t][e];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's scratch writes landed
    __builtin_amdgcn_wave_barrier();
    float sv[8];
    float mloc = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = 16 * kt + 4 * g + e;
        const float bd = gw[at_gslot(q - kk + AT_BK - 1) * 16 + q];
        float sc = (sacc[kt][e] + bd) * sl2;
        if (j0 + kk >= kend) sc = -INFINITY;
        sv[4 * kt + e] = sc;
        mloc = fmaxf(mloc, sc);
      }
    __builtin_amdgcn_wave_barrier();
    mloc = at_xor32_max(at_xor16_max(mloc));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = at_exp2(m_run - m_new);
    f32x4 pe[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) pe[kt][e] = at_exp2(sv[4 * kt + e] - m_new);
    float lsum = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) lsum += pe[e >> 2][e & 3];
    lsum = at_xor32_sum(at_xor16_sum(lsum));
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    // O^T += Vt . P^T: k-step (kt, e) has lane group g on key 16 kt + 4 g + e, the lane's own pe
#pragma unroll
    for (int t = 0; t < KU; ++t) {
      f32x4 o = oacc[t] * alpha;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        // Vt[16t + q][16kt + 4g + e] = V[16kt + 4g + e][16t + q]: four dword reads down the V rows
        // (the two lane groups of a 32-lane half are 4 rows = 16 banks apart: conflict-free)
        const float* vc = reinterpret_cast<const float*>(Vs + (16 * kt + 4 * g) * KR) + 16 * t + q;
#pragma unroll
        for (int e = 0; e < 4; ++e) o = __builtin_amdgcn_mfma_f32_16x16x4f32(vc[e * (KR / 4)], pe[kt][e], o, 0, 0, 0);
      }
      oacc[t] = o;
    }
    __syncthreads();
    write_kv(j0 + AT_BK);
    write_r(j0 + AT_BK);
    __syncthreads();
  }
  const int i = i0w + q;
  if (i < len) {
    if (po != nullptr) {  // key chunk: unnormalised rows and the row's (max, sum)
      const long long prow = ((long long)(kcn * nbatch + b) * H + h) * Tp + i;
      float* orow = po + prow * DK;
#pragma unroll
      for (int t = 0; t < KU; ++t) *reinterpret_cast<f32x4*>(orow + 16 * t + 4 * g) = oacc[t];
      if (g == 0) *reinterpret_cast<float2*>(pml + 2 * prow) = float2{m_run, l_run};
      return;
    }
    const float inv = 1.f / l_run;
    float* orow = out + ((long long)b * Tp + i) * rowD + h * DK;
#pragma unroll
    for (int t = 0; t < KU; ++t) *reinterpret_cast<f32x4*>(orow + 16 * t + 4 * g) = oacc[t] * inv;
  }
}

// Merge of the key chunks (rel_attn_f32_kernel, kc > 0): O = sum_c 2^(m_c - M) O_c,
// l = sum_c 2^(m_c - M) l_c, M = max_c m_c, out = O * (1 / l).  One thread per (row, 4 channels).
template <int DK>
__global__ __launch_bounds__(192) void rel_attn_merge_kernel(const float* __restrict__ po, const float* __restrict__ pml,
                                                            const int* __restrict__ lens, int Tp, int D, int H, int kc,
                                                            int nbatch, float* __restrict__ out) {
  const int r = blockIdx.x * 2 + threadIdx.x / 96;
  const int c4 = threadIdx.x % 96;
  if (4 * c4 >= D || r >= nbatch * Tp) return;
  const int b = r / Tp, i = r - b * Tp;
  const int len = lens[b];
  if (i >= len) return;
  const int h = 4 * c4 / DK, d = 4 * c4 - h * DK;
  const int n = (len + kc - 1) / kc;
  auto prow = [&](int c) { return ((long long)(c * nbatch + b) * H + h) * Tp + i; };
  float M = -INFINITY;
  for (int c = 0; c < n; ++c) M = fmaxf(M, pml[2 * prow(c)]);
  f32x4 o = f32x4{};
  float l = 0.f;
  for (int c = 0; c < n; ++c) {
    const float2 ml = *reinterpret_cast<const float2*>(pml + 2 * prow(c));
    const float wgt = at_exp2(ml.x - M);
    o += *reinterpret_cast<const f32x4*>(po + prow(c) * DK + d) * wgt;
    l += ml.y * wgt;
  }
  const float inv = 1.f / l;
  *reinterpret_cast<f32x4*>(out + (long long)r * D + h * DK + d) = o * inv;
}

// Split-precision form (the fp32 encoder of a 16-bit model, acoustic.cpp): every fp32 operand
// x is staged as two f16 planes, x_hi = f16(x) and x_lo = f16((x - x_hi) * 2^11), and each
// product runs as three v_mfma_f32_16x16x32_f16 (hi.hi into one accumulator, hi.lo + lo.hi
// into a second, scaled by 2^-11 when read) -- conv_split.hip's scheme, ~2^-21 relative per
// product, at 126 MFMA issues of 16 cycles per 32-key step where the f32 form needs 336 of 32.
// P is split the same way (P.V keeps fp32 accuracy); the softmax statistics are fp32.  Same
// schedule, index map and operand layouts as the 16-bit kernel; LDS holds both planes of K /
// Vt / R (142 KB): one block per CU.
constexpr float AT_SPLIT = 2048.f;  // 2^11

__device__ inline void at_split4(f32x4 v, uint2& hi, uint2& lo) {
  const half4 h = __builtin_convertvector(v, half4);
  const half4 l = __builtin_convertvector((v - __builtin_convertvector(h, f32x4)) * AT_SPLIT, half4);
  hi = __builtin_bit_cast(uint2, h);
  lo = __builtin_bit_cast(uint2, l);
}

__device__ inline void at_split8(f32x4 a, f32x4 b, half8& hi, half8& lo) {
  uint2 h0, l0, h1, l1;
  at_split4(a, h0, l0);
  at_split4(b, h1, l1);
  hi = __builtin_bit_cast(half8, uint4{h0.x, h0.y, h1.x, h1.y});
  lo = __builtin_bit_cast(half8, uint4{l0.x, l0.y, l1.x, l1.y});
}

template <int DK>
__global__ __launch_bounds__(256, 1) void rel_attn_split_kernel(const float* __restrict__ pu, const float* __restrict__ pv,
                                                               const float* __restrict__ qkv,
                                                               const float* __restrict__ ptab, const int* __restrict__ lens,
                                                               int Tp, int D, int H, int rmax, float scale,
                                                               float* __restrict__ out, int nqb, int nbatch,
                                                               int* __restrict__ range_flag, int kc, int nks,
                                                               float* __restrict__ po, float* __restrict__ pml) {
  using MF = Mfma16<half_t>;
  typedef half8 Frag;
  constexpr int KS = DK / 32;         // k-steps over dk
  constexpr int DT = DK / 16;         // 16-row tiles of dk (O^T)
  constexpr int KR = at_kr<half_t>(DK);  // K / V / R plane row stride (bytes)
  constexpr int KPL = AT_BK * KR, RPL = AT_RW * KR;  // plane sizes (lo = hi + size)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;                                        // 2 x [32 keys][DK]
  char* Vs = Ks + 2 * KPL;                                // 2 x [32 keys][DK]
  char* Rs = Vs + 2 * KPL;                                // 2 x [96 slots][DK]
  float* Gs = reinterpret_cast<float*>(Rs + 2 * RPL);     // [4 waves][48 slots][16 q]

  int bh, qt;
  if (!xcd_tile(nqb * nks, H * nbatch, bh, qt)) return;
  const int kcn = qt / nqb, qb = qt - kcn * nqb;  // key chunk, query tile (rel_attn_f32_kernel's map)
  const int b = bh / H, h = bh - b * H;
  const int i0 = qb * AT_BQ;
  const int len = lens[b];
  if (i0 >= len) return;
  const int kbeg = kcn * kc;  // (kc = 0: one chunk, all keys; kc a multiple of AT_BK)
  if (kbeg >= len) return;
  const int kend = kc > 0 ? min(len, kbeg + kc) : len;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 15, g = lane >> 4;
  const int i0w = i0 + 16 * w;
  const long long rowD = D;
  const int iq = min(i0w + q, Tp - 1);
  // Qu = q + pos_bias_u, Qv = q + pos_bias_v (HF:420-423) in fp32, then split
  Frag bu[KS], bul[KS], bv[KS], bvl[KS];
  unsigned rng = 0;  // range guard over the split operands' hi halves (common.h f16x2_nonfinite)
  auto guard8 = [&](const Frag& f) __attribute__((always_inline)) {
    const uint4 u = __builtin_bit_cast(uint4, f);
    rng |= f16x2_nonfinite(u.x) | f16x2_nonfinite(u.y) | f16x2_nonfinite(u.z) | f16x2_nonfinite(u.w);
  };
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int c = h * DK + ks * 32 + 8 * g;
    const float* qr = qkv + ((long long)b * Tp + iq) * 3 * rowD + c;
    const f32x4 q0 = *reinterpret_cast<const f32x4*>(qr), q1 = *reinterpret_cast<const f32x4*>(qr + 4);
    at_split8(q0 + *reinterpret_cast<const f32x4*>(pu + c), q1 + *reinterpret_cast<const f32x4*>(pu + c + 4), bu[ks], bul[ks]);
    at_split8(q0 + *reinterpret_cast<const f32x4*>(pv + c), q1 + *reinterpret_cast<const f32x4*>(pv + c + 4), bv[ks], bvl[ks]);
    guard8(bu[ks]);
    guard8(bv[ks]);
  }
  f32x4 oacc[DT], oaccx[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) { oacc[t] = f32x4{}; oaccx[t] = f32x4{}; }
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = scale * 1.4426950408889634f;
  float* gw = Gs + w * 48 * 16;

  // staging: fp32 pieces loaded for step s+1 during step s, split into the two planes after
  // the barrier that ends it (every step).  As in rel_attn_kernel: buffer descriptors stepped by
  // scalar base arithmetic (K and V rows >= len read 0, table rows past the last read 0 -- only
  // masked keys use them), per-thread offsets and LDS destinations fixed, ring slots stepped by
  // one unsigned min, masks only on the last key step
  constexpr int KP = AT_BK * (DK / 4) / 256;
  static_assert(AT_BK * (DK / 4) % 256 == 0, "staging split");
  constexpr unsigned RING = AT_RW * KR;
  auto rslot = [](int m) { const int r = m % AT_RW; return r < 0 ? r + AT_RW : r; };
  auto rrow = [&](int m) { return min(max(rmax - 1 - m, 0), 2 * rmax - 1); };
  auto ring_back = [](unsigned a) { return min(a - AT_BK * KR, a + (AT_RW - AT_BK) * KR); };
  auto put = [&rng](char* plane_hi, int plane, int off, f32x4 v) __attribute__((always_inline)) {
    uint2 hi, lo;
    at_split4(v, hi, lo);
    rng |= f16x2_nonfinite(hi.x) | f16x2_nonfinite(hi.y);
    *reinterpret_cast<uint2*>(plane_hi + off) = hi;
    *reinterpret_cast<uint2*>(plane_hi + plane + off) = lo;
  };
  const int rowB = 3 * D * 4;  // QKV row bytes
  int kofs[KP], rofs[KP];
  unsigned kdst[KP], rdst[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) {
    const int p = tid + 256 * i;
    const int r = p / (DK / 4), c = p - r * (DK / 4);
    kofs[i] = r * rowB + c * 16;                         // K and V rows
    kdst[i] = r * KR + c * 8;
    rofs[i] = r * D * 4 + c * 16;                        // table row row0 + r <-> m = i0 - j0 - r
    rdst[i] = rslot(i0 - kbeg - AT_BK - r) * KR + c * 8;  // slot for the first prefetch (j0 = kbeg + 32)
  }
  f32x4 pkv[KP], pvt[KP], prr[KP];
  auto load_kv = [&](int j0) __attribute__((always_inline)) {
    const float* krow = qkv + ((long long)b * Tp + j0) * 3 * rowD + D + h * DK;
    const auto kr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(krow), 0, max(len - j0, 0) * rowB, 0x00020000);
    const auto vr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(krow + D), 0, max(len - j0, 0) * rowB, 0x00020000);
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      pkv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(kr, kofs[i], 0, 0));
      pvt[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(vr, kofs[i], 0, 0));
    }
  };
  auto load_r = [&](int j0) __attribute__((always_inline)) {
    const int row0 = rmax - 1 - i0 + j0;  // >= 0: i0 < len <= Tm <= rmax
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptab + (long long)row0 * rowD + h * DK), 0,
                                                      max(rmax + i0 - j0, 0) * D * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < KP; ++i)
      prr[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, rofs[i], 0, 0));
  };
  auto write_kv = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      put(Ks, KPL, kdst[i], pkv[i]);
      put(Vs, KPL, kdst[i], pvt[i]);
    }
  };
  auto write_r = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      put(Rs, RPL, rdst[i], prr[i]);
      rdst[i] = ring_back(rdst[i]);
    }
  };
  for (int p = tid; p < AT_RW * (DK / 4); p += 256) {
    const int sb = p / (DK / 4), c = p - sb * (DK / 4);
    const int m = i0 - kbeg - (AT_BK - 1) + sb;
    put(Rs, RPL, rslot(m) * KR + c * 8, *reinterpret_cast<const f32x4*>(ptab + (long long)rrow(m) * rowD + h * DK + c * 4));
  }
  load_kv(kbeg);
  write_kv();
  __syncthreads();
  unsigned ra = rslot(i0w - kbeg - (AT_BK - 1) + q) * KR + 16 * g;  // this lane's R rows (slot of m + 16 t) and column
  const int vta = at_tr_addr(KR, g, q);  // this lane's transposed-read address in the V planes (tile 0)

  // (the last-step peel of rel_attn_kernel pushed this kernel past 256 VGPRs: kept as one loop).
  // Only the last chunk's last step has keys past len (kc is a multiple of AT_BK): the mask below.
  for (int j0 = kbeg; j0 < kend; j0 += AT_BK) {
    load_kv(j0 + AT_BK);
    load_r(j0 + AT_BK);
    __builtin_amdgcn_sched_barrier(0);
    f32x4 sacc[2] = {f32x4{}, f32x4{}}, saccx[2] = {f32x4{}, f32x4{}};
    f32x4 gacc[3] = {f32x4{}, f32x4{}, f32x4{}}, gaccx[3] = {f32x4{}, f32x4{}, f32x4{}};
    unsigned rs[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const unsigned y = ra + 16 * t * KR;
      rs[t] = t ? min(y, y - RING) : y;
    }
    ra = ring_back(ra);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int co = (ks * 32 + 8 * g) * 2;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const char* kr = Ks + (16 * kt + q) * KR + co;
        const Frag ah = *reinterpret_cast<const Frag*>(kr), al = *reinterpret_cast<const Frag*>(kr + KPL);
        sacc[kt] = MF::mma(ah, bu[ks], sacc[kt]);
        saccx[kt] = MF::mma(ah, bul[ks], saccx[kt]);
        saccx[kt] = MF::mma(al, bu[ks], saccx[kt]);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const char* rr = Rs + rs[t] + ks * 64;
        const Frag ah = *reinterpret_cast<const Frag*>(rr), al = *reinterpret_cast<const Frag*>(rr + RPL);
        gacc[t] = MF::mma(ah, bv[ks], gacc[t]);
        gaccx[t] = MF::mma(ah, bvl[ks], gaccx[t]);
        gaccx[t] = MF::mma(al, bv[ks], gaccx[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const f32x4 gv = gacc[t] + gaccx[t] * (1.f / AT_SPLIT);
#pragma unroll
      for (int e = 0; e < 4; ++e) gw[at_gslot(16 * t + 4 * g + e) * 16 + q] = gv[e];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's scratch writes landed
    __builtin_amdgcn_wave_barrier();
    float sv[8];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const f32x4 s4 = sacc[kt] + saccx[kt] * (1.f / AT_SPLIT);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = 16 * kt + 4 * g + e;
        const float bd = gw[at_gslot(q - kk + AT_BK - 1) * 16 + q];
        sv[4 * kt + e] = (s4[e] + bd) * sl2;
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (j0 + AT_BK > len) {  // wave-uniform: only the last step has keys past len
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (j0 + 16 * kt + 4 * g + e >= len) sv[4 * kt + e] = -INFINITY;
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) mloc = fmaxf(mloc, sv[e]);
    mloc = at_xor32_max(at_xor16_max(mloc));
    // lazy rescale as in rel_attn_kernel (P <= 2^AT_LAZY: its hi / lo planes keep their range)
    const bool grow = mloc > m_run + AT_LAZY;
    const float m_new = grow ? mloc : m_run;
    const float alpha = at_exp2(m_run - m_new);
    if (__builtin_amdgcn_ballot_w64(grow) != 0) {
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        oacc[t] *= alpha;
        oaccx[t] *= alpha;
      }
    }
    f32x4 pe0, pe1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pe0[e] = at_exp2(sv[e] - m_new);
      pe1[e] = at_exp2(sv[4 + e] - m_new);
    }
    float lsum = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) lsum += pe0[e];
#pragma unroll
    for (int e = 0; e < 4; ++e) lsum += pe1[e];
    lsum = at_xor32_sum(at_xor16_sum(lsum));
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    Frag bp, bpl;
    at_split8(pe0, pe1, bp, bpl);
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const char* vr = Vs + vta + t * 32;
      const uint2 h0 = at_tr16(vr), h1 = at_tr16(vr + 16 * KR);
      const uint2 l0 = at_tr16(vr + KPL), l1 = at_tr16(vr + KPL + 16 * KR);
      const Frag ah = __builtin_bit_cast(Frag, uint4{h0.x, h0.y, h1.x, h1.y});
      const Frag al = __builtin_bit_cast(Frag, uint4{l0.x, l0.y, l1.x, l1.y});
      oacc[t] = MF::mma(ah, bp, oacc[t]);
      f32x4 ox = MF::mma(ah, bpl, oaccx[t]);
      oaccx[t] = MF::mma(al, bp, ox);
    }
    __syncthreads();
    write_kv();
    write_r();
    __syncthreads();
  }
  const int i = i0w + q;
  if (i < len) {
    if (po != nullptr) {  // key chunk: unnormalised rows and the row's (reference max, sum), merged
                          // by rel_attn_merge_kernel (the lazy reference max is a valid one)
      const long long prow = ((long long)(kcn * nbatch + b) * H + h) * Tp + i;
      float* orow = po + prow * DK;
#pragma unroll
      for (int t = 0; t < DT; ++t) *reinterpret_cast<f32x4*>(orow + 16 * t + 4 * g) = oacc[t] + oaccx[t] * (1.f / AT_SPLIT);
      if (g == 0) *reinterpret_cast<float2*>(pml + 2 * prow) = float2{m_run, l_run};
    } else {
      const float inv = 1.f / l_run;
      float* orow = out + ((long long)b * Tp + i) * rowD + h * DK;
#pragma unroll
      for (int t = 0; t < DT; ++t)
        *reinterpret_cast<f32x4*>(orow + 16 * t + 4 * g) = (oacc[t] + oaccx[t] * (1.f / AT_SPLIT)) * inv;
    }
  }
  range_report(range_flag, rng);
}

template <int DK>
size_t rel_attn_split_lds() {
  return (size_t)2 * (2 * AT_BK + AT_RW) * at_kr<half_t>(DK) + (size_t)4 * 48 * 16 * 4;
}

template <int DK>
size_t rel_attn_f32_lds() {
  return (size_t)(2 * AT_BK + AT_RW) * at_kr<float>(DK) + (size_t)4 * 48 * 16 * 4;
}

template <int DK>
size_t rel_attn_lds(int kh) {
  return (size_t)kh * ((2 * AT_BK + AT_RW) * at_kr<half_t>(DK) + (size_t)4 * 48 * 16 * 4);
}
// two 16-bit blocks per CU (rel_attn_kernel's launch bounds)
static_assert((2 * AT_BK + AT_RW) * at_kr<half_t>(192) + 4 * 48 * 16 * 4 <= 160 * 1024 / 2, "LDS");

}  // namespace

bool rel_attn_supported(int dt, int D, int H) {
  return (dt == DT_F16 || dt == DT_BF16 || dt == DT_F32) && H > 0 && D % H == 0 && D / H == 192;
}

int rel_attn_f32_kc() {
  const int v = sw(SW_ATTN_F32_KC);
  if (v < 0) return AT_F32_KC;
  return v == 0 ? 0 : std::max(AT_BK, v / AT_BK * AT_BK);
}

long long rel_attn_split_ws_bytes(int B, int Tm, int Tp, int D, int H) {
  const int kc = TTS_ATTN_SPLIT_KC;
  if (kc == 0 || Tm <= kc) return 0;
  const long long nks = (Tm + kc - 1) / kc;
  return nks * B * Tp * ((long long)D + 2 * H) * 4;
}

long long rel_attn_f32_ws_bytes(int B, int Tm, int Tp, int D, int H) {
  const int kc = rel_attn_f32_kc();
  if (kc == 0 || Tm <= kc) return 0;
  const long long nks = (Tm + kc - 1) / kc;
  return nks * B * Tp * ((long long)D + 2 * H) * 4;
}

hipError_t launch_rel_attn(int dt, bool split, const float* pos_u, const float* pos_v, const void* qkv,
                           const void* ptab, const int* lens, int B, int Tm, int Tp, int D, int H, int rmax,
                           float scale, void* out, hipStream_t s, int* range_flag, float* ws, long long ws_bytes) {
  if (!rel_attn_supported(dt, D, H) || Tm > rmax) return hipErrorInvalidValue;
  const int nqb = (Tm + AT_BQ - 1) / AT_BQ;
  dim3 grid(xcd_grid(nqb, H * B));
  if (dt == DT_F32 && split) {
    // key chunks of TTS_ATTN_SPLIT_KC keys when the workspace holds them (as the fp32 form below)
    const int kc = TTS_ATTN_SPLIT_KC;
    const long long need = rel_attn_split_ws_bytes(B, Tm, Tp, D, H);
    if (need > 0 && ws != nullptr && need <= ws_bytes) {
      const int nks = (Tm + kc - 1) / kc;
      float* po = ws;
      float* pml = ws + (long long)nks * B * Tp * D;
      hipLaunchKernelGGL((rel_attn_split_kernel<192>), dim3(xcd_grid(nqb * nks, H * B)), dim3(256), rel_attn_split_lds<192>(), s,
                         pos_u, pos_v, (const float*)qkv, (const float*)ptab, lens, Tp, D, H, rmax, scale,
                         (float*)out, nqb, B, range_flag, kc, nks, po, pml);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((rel_attn_merge_kernel<192>), dim3((B * Tp + 1) / 2), dim3(192), 0, s, po, pml, lens, Tp, D, H,
                         kc, B, (float*)out);
      return hipGetLastError();
    }
    hipLaunchKernelGGL((rel_attn_split_kernel<192>), grid, dim3(256), rel_attn_split_lds<192>(), s, pos_u, pos_v,
                       (const float*)qkv, (const float*)ptab, lens, Tp, D, H, rmax, scale,
                       (float*)out, nqb, B, range_flag, 0, 1, nullptr, nullptr);
    return hipGetLastError();
  }
  if (dt == DT_F32) {
    // key chunks when the workspace holds them (fp32 models; the merge is skipped when every
    // utterance fits one chunk: that row's merge would reproduce the direct bits)
    const int kc = rel_attn_f32_kc();
    const long long need = rel_attn_f32_ws_bytes(B, Tm, Tp, D, H);
    if (need > 0 && ws != nullptr && need <= ws_bytes) {
      const int nks = (Tm + kc - 1) / kc;
      float* po = ws;
      float* pml = ws + (long long)nks * B * Tp * D;
      hipLaunchKernelGGL((rel_attn_f32_kernel<192>), dim3(xcd_grid(nqb * nks, H * B)), dim3(256), rel_attn_f32_lds<192>(), s,
                         pos_u, pos_v, (const float*)qkv, (const float*)ptab, lens, Tp, D, H, rmax, scale,
                         (float*)out, nqb, B, kc, nks, po, pml);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((rel_attn_merge_kernel<192>), dim3((B * Tp + 1) / 2), dim3(192), 0, s, po, pml, lens, Tp, D, H,
                         kc, B, (float*)out);
      return hipGetLastError();
    }
    hipLaunchKernelGGL((rel_attn_f32_kernel<192>), grid, dim3(256), rel_attn_f32_lds<192>(), s, pos_u, pos_v,
                       (const float*)qkv, (const float*)ptab, lens, Tp, D, H, rmax, scale,
                       (float*)out, nqb, B, 0, 1, nullptr, nullptr);
    return hipGetLastError();
  }
  // two key groups per block (TTS_ATTN_KSPLIT=1): batch 8 287 -> 248 us per forward, batch 32
  // 757 -> 934 us (one block per CU).  Off by default: a batch-dependent choice would make a
  // row's bits depend on the batch (the merge rounds differently from one online softmax)
  const int kh = sw(SW_ATTN_KSPLIT) == 1 ? 2 : 1;
  const size_t lds = rel_attn_lds<192>(kh);
#define TTS_ATTN_LAUNCH(TT_, KH_)                                                                  \
  hipLaunchKernelGGL((rel_attn_kernel<TT_, 192, KH_>), grid, dim3(256 * KH_), lds, s, pos_u, pos_v, \
                     (const TT_*)qkv, (const TT_*)ptab, lens, Tp, D, H, rmax, scale,                     \
                     (TT_*)out, nqb, B)
  if (dt == DT_F16) {
    if (kh == 2) TTS_ATTN_LAUNCH(half_t, 2); else TTS_ATTN_LAUNCH(half_t, 1);
  } else {
    if (kh == 2) TTS_ATTN_LAUNCH(bf16_t, 2); else TTS_ATTN_LAUNCH(bf16_t, 1);
  }
#undef TTS_ATTN_LAUNCH
  return hipGetLastError();
}

}  // namespace tts
