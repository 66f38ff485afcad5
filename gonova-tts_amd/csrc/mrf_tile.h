// ResBlock tile machinery shared by the pair kernel (mrf_pair.hip) and the resblock chain
// kernel (mrf_chain.hip): LDS activation-tile geometry and swizzle, the 16x16x32 MFMA
// wrappers, epilogue arithmetic, and the weight-ring conv loop over 16-row tiles.
#pragma once
#include "common.h"

namespace tts {

template <int C>
struct PairGeom;
// Activation tiles in LDS: unpadded rows (RS = C*2 bytes), 16-byte chunk c of row r stored
// at chunk c ^ (((r * SW_MUL) >> SW_S) & SW_M).  Chosen with an LDS bank model of every access
// (MI355X_MICROARCH.md §LDS lane groups): the MFMA B-fragment ds_read_b128 (16 rows x 4
// chunks per lane group) and the staging ds_write_b128 are conflict-free; the once-per-tile
// 8-byte epilogue accesses are 2-way.  (Padded rows of 80/144 B made the B reads 2-way:
// measured 43-47 % of LDS cycles were bank conflicts.)  The swizzle depends on r mod 8
// only, so it is shared by every 16-row tile and computed once per tap.  At C = 128 the
// 256-byte rows are one LDS bank row each; chunk ^ ((2r) & 15) keeps the B reads
// conflict-free for every tap offset (exhaustive check over r mod 16).
// MT: 16-channel M tiles per wave (a wave owns 16*MT output channels); D: weight-ring depth
// (k-steps); OCC: blocks per CU the register budget is sized for.
#ifndef TTS_P32_D
#define TTS_P32_D 4
#endif
#ifndef TTS_P64_D
#define TTS_P64_D 4
#endif
#ifndef TTS_P32_OCC
#define TTS_P32_OCC 3
#endif
template <>
struct PairGeom<32> {
  static constexpr int BN = 512, WM = 1, WN = 4, RS = 64, SW_MUL = 1, SW_S = 1, SW_M = 3, D = TTS_P32_D, MT = 2, OCC = TTS_P32_OCC;
};
#ifndef TTS_P64_OCC
#define TTS_P64_OCC 3
#endif
#ifndef TTS_P64_WM
#define TTS_P64_WM 2  // 1: 64-channel wave tiles (MT = 4, 4 waves along the rows)
#endif
template <>
struct PairGeom<64> {
  static constexpr int BN = 256, WM = TTS_P64_WM, WN = 4 / TTS_P64_WM, RS = 128, SW_MUL = 1, SW_S = 0, SW_M = 7,
                       D = TTS_P64_D, MT = 4 / TTS_P64_WM, OCC = TTS_P64_OCC;
};
#ifndef TTS_P128_WM
#define TTS_P128_WM 4
#endif
#ifndef TTS_P128_D
#define TTS_P128_D 4
#endif
#ifndef TTS_P128_OCC
#define TTS_P128_OCC 3
#endif
#ifndef TTS_P256_D
#define TTS_P256_D 2
#endif
template <>
struct PairGeom<128> {
  static constexpr int BN = 128, WM = TTS_P128_WM, WN = 4 / WM, RS = 256, SW_MUL = 2, SW_S = 0, SW_M = 15,
                       D = TTS_P128_D, MT = 8 / WM, OCC = TTS_P128_OCC;
};
// C = 256 (HiFi-GAN stage 0): 64-row tiles, 64 channels per wave, two blocks per CU.  The
// 512-byte rows span two LDS bank rows; the same chunk ^ ((2r) & 15) keeps the B reads
// conflict-free (the XOR never leaves a chunk's 256-byte half).  Weights streamed per row
// equal conv_xres's 128-channel x 128-row blocks (both read 2*C*C*k / 64 B per output row
// and conv), but t never leaves the block.
#ifndef TTS_P256_WN
#define TTS_P256_WN 1  // 2: 8-wave blocks of 128 rows (half the weight stream per row, one block per CU)
#endif
template <>
struct PairGeom<256> {
  static constexpr int BN = 64 * TTS_P256_WN, WM = 4, WN = TTS_P256_WN, RS = 512, SW_MUL = 2, SW_S = 0, SW_M = 15,
                       D = TTS_P256_D, MT = 4, OCC = TTS_P256_WN == 1 ? 2 : 1;
};

template <typename T>
struct Mfma16;
template <>
struct Mfma16<half_t> {
  __device__ static inline f32x4 mma(half8 a, half8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Mfma16<bf16_t> {
  __device__ static inline f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};

#ifndef TTS_PAIR_SU
#define TTS_PAIR_SU 12
#endif
#ifndef TTS_ROW_STORE
#define TTS_ROW_STORE 2  // cache policy of the pair / chain output stores (store16, common.h)
#endif
#ifndef TTS_XCD_REMAP
#define TTS_XCD_REMAP 1
#endif
// XCD-aware tile order for a 1-D grid of nx row tiles x B utterances.  Workgroups are dealt to
// the 8 XCDs round robin in dispatch order, so adjacent row tiles (which share halo rows)
// would land on 8 different L2s; here XCD x gets the contiguous tile range
// [x * per, (x + 1) * per) of the (utterance, tile) sequence.  Returns false for the padding
// workgroups of the last range.
__device__ inline bool xcd_tile(int nx, int B, int& b, int& tile) {
  const int total = nx * B;
  int v = blockIdx.x;
#if TTS_XCD_REMAP
  const int per = (total + 7) / 8;
  v = (v & 7) * per + (v >> 3);
#endif
  if (v >= total) return false;
  b = v / nx;
  tile = v - b * nx;
  return true;
}
inline int xcd_grid(int nx, int B) {
#if TTS_XCD_REMAP
  return 8 * ((nx * B + 7) / 8);
#else
  return nx * B;
#endif
}

constexpr int PAIR_SU = TTS_PAIR_SU;  // input-tile loads in flight per thread (one round for every pair shape up to k = 11)

template <typename T>
__device__ inline void pair_ld8(const T* p, f32x4& a, f32x4& b) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const T* e = reinterpret_cast<const T*>(&u);
  a = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
  b = f32x4{(float)e[4], (float)e[5], (float)e[6], (float)e[7]};
}
// Bias in the accumulator (TTS_BIAS_ACC, default): every conv's accumulators start at its bias
// (the first MFMA reads the bias registers as its C operand), so the epilogues add nothing --
// 2 packed f16 adds (f16) or 4 f32 adds (bf16) fewer per accumulator quad, and for f16 one
// rounding of acc + bias instead of f16(acc) + f16(bias).  Pair, chain and pipelined kernels all
// use it, so they stay bit-identical to each other.
#ifndef TTS_BIAS_ACC
#define TTS_BIAS_ACC 1
#endif
__device__ inline f32x4 acc_init(f32x4 bias) {
#if TTS_BIAS_ACC
  return bias;
#else
  (void)bias;
  return f32x4{};
#endif
}

// Epilogue arithmetic.  f16: packed half math after one cvt_pk per pair of accumulators
// (v_pk_add/mul/max_f16: a fraction of the f32 instruction count; a sum of two f16 values
// is correctly rounded either way, the bias/slope products differ by <= 1 ulp).  bf16:
// f32 math, one rounding at the end.
template <typename T>
__device__ inline uint2 epi_conv1(f32x4 acc, f32x4 bias, float slope) {  // lrelu(acc + b) -> 4 x T
  if constexpr (__is_same(T, half_t)) {
#if TTS_BIAS_ACC
    (void)bias;
    half4 h = __builtin_convertvector(acc, half4);
#else
    half4 h = __builtin_convertvector(acc, half4) + __builtin_convertvector(bias, half4);
#endif
    const half4 m = h * (half_t)slope;
    const uint2 hu = __builtin_bit_cast(uint2, h), mu = __builtin_bit_cast(uint2, m);
    return uint2{pk_max_f16(hu.x, mu.x), pk_max_f16(hu.y, mu.y)};
  } else {
#if TTS_BIAS_ACC
    (void)bias;
    f32x4 v = acc;
#else
    f32x4 v = acc + bias;
#endif
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaxf(v[e], v[e] * slope);  // 0 <= slope <= 1
    return pack4<T>(v);
  }
}
template <typename T>
__device__ inline uint2 epi_conv2(f32x4 acc, f32x4 bias) {  // acc + b -> 4 x T
#if TTS_BIAS_ACC
  (void)bias;
  return pack4<T>(acc);
#else
  if constexpr (__is_same(T, half_t)) {
    half4 h = __builtin_convertvector(acc, half4) + __builtin_convertvector(bias, half4);
    return *reinterpret_cast<const uint2*>(&h);
  } else {
    return pack4<T>(acc + bias);
  }
#endif
}
// row pass: (y + h (+ s)) * scale on 8 elements
template <typename T>
__device__ inline uint4 epi_row(uint4 y, uint4 h, bool acc, uint4 s, float scale) {
  if constexpr (__is_same(T, half_t)) {
    half8 v = *reinterpret_cast<const half8*>(&y) + *reinterpret_cast<const half8*>(&h);
    if (acc) v += *reinterpret_cast<const half8*>(&s);
    if (scale != 1.0f) v *= (half_t)scale;
    return *reinterpret_cast<const uint4*>(&v);
  } else if constexpr (__is_same(T, bf16_t)) {
    const unsigned* yw = reinterpret_cast<const unsigned*>(&y);
    const unsigned* hw = reinterpret_cast<const unsigned*>(&h);
    const unsigned* sw = reinterpret_cast<const unsigned*>(&s);
    unsigned o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x2 v = bf16x2_unpack(yw[i]) + bf16x2_unpack(hw[i]);
      if (acc) v += bf16x2_unpack(sw[i]);
      o[i] = bf16x2_pack(v * scale);
    }
    return uint4{o[0], o[1], o[2], o[3]};
  } else {
    const T* ye = reinterpret_cast<const T*>(&y);
    const T* he = reinterpret_cast<const T*>(&h);
    const T* se = reinterpret_cast<const T*>(&s);
    T o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = (float)ye[e] + (float)he[e];
      if (acc) v += (float)se[e];
      o[e] = (T)(v * scale);
    }
    return *reinterpret_cast<const uint4*>(o);
  }
}

// row pass on 4 elements (one lane's MFMA output quad), rounded exactly as epi_row rounds them
template <typename T>
__device__ inline uint2 epi_row4(uint2 y, uint2 h, bool acc, uint2 s, float scale) {
  if constexpr (__is_same(T, half_t)) {
    half4 v = __builtin_bit_cast(half4, y) + __builtin_bit_cast(half4, h);
    if (acc) v += __builtin_bit_cast(half4, s);
    if (scale != 1.0f) v *= (half_t)scale;
    return __builtin_bit_cast(uint2, v);
  } else {
    f32x2 v0 = bf16x2_unpack(y.x) + bf16x2_unpack(h.x);
    f32x2 v1 = bf16x2_unpack(y.y) + bf16x2_unpack(h.y);
    if (acc) {
      v0 += bf16x2_unpack(s.x);
      v1 += bf16x2_unpack(s.y);
    }
    return uint2{bf16x2_pack(v0 * scale), bf16x2_pack(v1 * scale)};
  }
}

// the same, branch-free for the pipelined kernels (a uniform branch would split the basic block
// their MFMAs and epilogues are interleaved in): s is 0 when the launch does not accumulate (a
// zero-record descriptor) and scale 1 multiplies exactly, so the values equal epi_row4's (a
// -0 sum may come out as +0)
template <typename T>
__device__ inline uint2 epi_row4_nb(uint2 y, uint2 h, uint2 s, float scale) {
  if constexpr (__is_same(T, half_t)) {
    half4 v = __builtin_bit_cast(half4, y) + __builtin_bit_cast(half4, h);
    v += __builtin_bit_cast(half4, s);
    v *= (half_t)scale;
    return __builtin_bit_cast(uint2, v);
  } else {
    const f32x2 v0 = bf16x2_unpack(y.x) + bf16x2_unpack(h.x) + bf16x2_unpack(s.x);
    const f32x2 v1 = bf16x2_unpack(y.y) + bf16x2_unpack(h.y) + bf16x2_unpack(s.y);
    return uint2{bf16x2_pack(v0 * scale), bf16x2_pack(v1 * scale)};
  }
}

template <typename T>
__device__ inline void pair_st8(T* p, f32x4 a, f32x4 b) {
  *reinterpret_cast<uint4*>(p) = pack8<T>(a, b);
}

// One conv of the pair over NU 16-row tiles per wave: acc[u][mt] += W[mt] x tile u.
// S = k * KS k-steps, weights streamed through the D-slot register ring (ring[i] holds step
// i on entry).  The step sequence is compile-time: full groups of D steps in a counted loop
// (every step reloads its slot D steps ahead), then a peeled last group whose reloads stop
// at S, then the S % D tail.  Straight-line bodies let the waitcnt pass keep the ring's
// 2*(D-1) younger loads in flight (a conditional reload made it drain vmcnt to 0 every step).
// lb: this lane's LDS base for its wave's first tile (row rb of it, tap 0); the wave's tile u
// sits TU bytes after tile u - 1 (TU = 16 rows x WN waves x row bytes: the waves' tiles are
// dealt round robin), a compile-time immediate of the LDS reads -- no per-tile address
// arithmetic -- except for the last tile, at last_off bytes: a wave whose share is one short
// repeats the block's last tile there (straight-line, result not stored).
// tstep: LDS bytes per tap; trow: rows per tap (swizzle); rb: the lane's row mod 8 in tile 0.
// MTO: MFMA order within a step -- M tile outer (each A fragment feeds NU MFMAs back to
// back) or row tile outer.  Same-box A/B: M-outer 1-3 % faster for the C = 64 / 128 / 256
// pairs, slower for C = 32 and the chains.
// RB0 / TROW (the chain kernel, whose row offsets and dilations are compile-time): rb = l15 + RB0
// and trow = TROW, so a step's row phase (r mod 8, which fixes the swizzle) is a compile-time
// index into sw8 (pair_sw8) and its chunk offset one register -- no swizzle arithmetic per step.
// Used where every step is unrolled (fewer than two full groups of D steps).
template <typename T, int C, int S, int NU, int D, int MT = 2, bool MTO = false, int TU = 0, int RB0 = -1, int TROW = 0>
__device__ __forceinline__ void pair_conv(f32x4 (&acc)[NU][MT], typename Mfma<T>::frag (&ring)[D][MT],
                                          const char* __restrict__ wp, const char* lb, int tstep, int trow,
                                          int rb, int lq, int last_off, const int* sw8 = nullptr) {
  using G = PairGeom<C>;
  using MF = Mfma16<T>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int KS = C / 32;
  constexpr int NG = S / D, REM = S % D;
  constexpr bool TABLE = RB0 >= 0 && NG < 2;
  auto step = [&](const int s, const int slot, const bool reload) __attribute__((always_inline)) {
    const int tap = KS == 1 ? s : s / KS, ks = KS == 1 ? 0 : s % KS;
    const char* bp;
    if constexpr (TABLE) {
      // (lq + 4 ks) ^ sw = (lq ^ sw) ^ 4 ks: lq < 4, so the k-step only flips chunk bits >= 2
      bp = lb + tap * TROW * G::RS + (sw8[(RB0 + tap * TROW) & 7] ^ (ks << 6));
    } else {
      const int r = rb + tap * trow;
      bp = lb + tap * tstep + (((lq + 4 * ks) ^ (((r * G::SW_MUL) >> G::SW_S) & G::SW_M)) << 4);
    }
    Frag bf[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) bf[u] = *reinterpret_cast<const Frag*>(bp + (u + 1 < NU ? u * TU : last_off));
    if constexpr (MTO) {  // one A fragment held across the NU tiles
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int u = 0; u < NU; ++u) acc[u][mt] = MF::mma(ring[slot][mt], bf[u], acc[u][mt]);
    } else {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[u][mt] = MF::mma(ring[slot][mt], bf[u], acc[u][mt]);
    }
    if (reload) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        ring[slot][mt] = *reinterpret_cast<const Frag*>(wp + ((long long)mt * S + s + D) * 1024);
      __builtin_amdgcn_sched_barrier(0);  // issue the reload here, D steps ahead of its use
    }
  };
  if constexpr (NG >= 2) {
#pragma nounroll
    for (int g = 0; g < NG - 1; ++g) {
#pragma unroll
      for (int i = 0; i < D; ++i) step(g * D + i, i, true);
    }
  }
  if constexpr (NG >= 1) {
#pragma unroll
    for (int i = 0; i < D; ++i) step((NG - 1) * D + i, i, i < REM);
  }
#pragma unroll
  for (int i = 0; i < REM; ++i) step(NG * D + i, i, false);
}

// sw8[j]: the B-fragment chunk byte offset (k-step 0) of a lane whose tile row is l15 + j (mod 8)
template <int C>
__device__ inline void pair_sw8(int (&sw8)[8], int l15, int lq) {
  using G = PairGeom<C>;
#pragma unroll
  for (int j = 0; j < 8; ++j) sw8[j] = (lq ^ ((((l15 + j) * G::SW_MUL) >> G::SW_S) & G::SW_M)) << 4;
}
// ep8[j]: pair_lds4's chunk bytes for row l15 + j (mod 8) and channels 4 lq .. 4 lq + 3; channel
// c0 = 4 lq + 16 m (m = 2 wm + mt) adds m to the chunk's bits >= 1, i.e. ep8[j] ^ (m << 5)
template <int C>
__device__ inline void pair_ep8(int (&ep8)[8], int l15, int lq) {
  using G = PairGeom<C>;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    ep8[j] = (((lq >> 1) ^ ((((l15 + j) * G::SW_MUL) >> G::SW_S) & G::SW_M)) << 4) + 8 * (lq & 1);
}

// byte offset of this lane's 4 channels (c0 .. c0+3) in LDS row r of a PairGeom<C> tile; the
// swizzle depends on r mod 8 only, so row r + 16 t is the same offset + 16 t rows
template <int C>
__device__ inline int pair_lds4(int r, int c0) {
  using G = PairGeom<C>;
  const int cb = c0 * 2;
  return r * G::RS + ((((cb >> 4) ^ (((r * G::SW_MUL) >> G::SW_S) & G::SW_M))) << 4) + (cb & 15);
}

}  // namespace tts
