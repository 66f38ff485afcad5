// Shared device/host helpers for the gfx950 (CDNA4) TTS kernels.
//
// Everything here is written for MI355X directly: 64-lane wavefronts, the
// gfx950 MFMA builtins (32x32x16 f16/bf16, 32x32x2 f32) and 16-byte vector
// memory accesses.  No portability layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tts {

enum DType : int { DT_F32 = 0, DT_F16 = 1, DT_BF16 = 2 };

typedef _Float16 half_t;
typedef __bf16 bf16_t;

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// 16-byte staging registers: a native vector, so a global -> register -> LDS copy is a plain
// load / store pair (a uint4 struct copy becomes a memcpy that can land in scratch)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// MFMA traits: one 32x32 output tile per wave-instruction.
//   16-bit: v_mfma_f32_32x32x16_{f16,bf16}; lane l holds A[l&31][8*(l>>5)+e],
//           B[8*(l>>5)+e][l&31], e = 0..7 (K = 16 per instruction).
//   f32   : v_mfma_f32_32x32x2_f32; lane l holds A[l&31][l>>5], B[l>>5][l&31].
//   C/D   : col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5), r = 0..15.
// ---------------------------------------------------------------------------
template <typename T> struct Mfma;

template <> struct Mfma<half_t> {
  static constexpr int KSTEP = 16;  // K per instruction
  static constexpr int KPL = 8;     // K elements per lane
  typedef half8 frag;
  __device__ static inline f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

template <> struct Mfma<bf16_t> {
  static constexpr int KSTEP = 16;
  static constexpr int KPL = 8;
  typedef bf16x8 frag;
  __device__ static inline f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

template <> struct Mfma<float> {
  static constexpr int KSTEP = 2;
  static constexpr int KPL = 1;
  typedef float frag;
  __device__ static inline f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
};

// ---------------------------------------------------------------------------
// Scalar conversions
// ---------------------------------------------------------------------------
template <typename T> __device__ __host__ inline float to_f32(T v) { return (float)v; }
template <typename T> __device__ __host__ inline T from_f32(float v) { return (T)v; }

// 4 consecutive elements <-> float4 (one 8-byte (16-bit) or 16-byte (f32) access)
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  typedef f32x4 type;
  __device__ static inline f32x4 load(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  __device__ static inline void store(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
};
template <> struct Vec4<half_t> {
  __device__ static inline f32x4 load(const half_t* p) {
    half4 h = *reinterpret_cast<const half4*>(p);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
  __device__ static inline void store(half_t* p, f32x4 v) {
    half4 h = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
    *reinterpret_cast<half4*>(p) = h;
  }
};
template <> struct Vec4<bf16_t> {
  __device__ static inline f32x4 load(const bf16_t* p) {
    bf16x4 h = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
  __device__ static inline void store(bf16_t* p, f32x4 v) {
    *reinterpret_cast<bf16x4*>(p) = __builtin_convertvector(v, bf16x4);  // 2 x v_cvt_pk_bf16_f32
  }
};

// 16-byte chunk of T (8 x 16-bit or 4 x f32)
template <typename T> struct Chunk16 {
  static constexpr int N = 16 / sizeof(T);
};

__device__ inline float leaky(float x, float slope) { return x >= 0.f ? x : x * slope; }

// Range guard of the split-precision (three-f16) paths (conv_split.hip, the split attention): an
// fp32 operand is held as hi = f16(x) plus a scaled remainder, so |x| >= 65520 (hi = inf) or a
// NaN cannot be represented.  f16x2_nonfinite(w) has bit 15 / 31 set iff the low / high half of
// the f16 pair w has an all-ones exponent (inf or NaN): (e & 0x7c00) + 0x0400 reaches 0x8000 only
// for e = 0x7c00, with no carry out of the half.  A kernel ORs these over its hi halves and, at
// its end, reports a hit to a device word the host reads (range_report).
#ifndef TTS_RANGE_GUARD
#define TTS_RANGE_GUARD 1  // 0: A/B builds without the guard (the word is never set)
#endif
__device__ inline unsigned f16x2_nonfinite(unsigned w) { return TTS_RANGE_GUARD ? (w & 0x7c007c00u) + 0x04000400u : 0u; }
__device__ inline void range_report(int* flag, unsigned acc) {
  if (TTS_RANGE_GUARD && (acc & 0x80008000u) && flag) __hip_atomic_fetch_or(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bf16 pairs.  One 32-bit word holds elements (lo, hi); as f32 they are w << 16 and
// w & 0xffff0000 (exact), and a pair rounds back with one v_cvt_pk_bf16_f32 (RNE).  Element-wise
// (T)float casts instead cost a one-sided cvt per element plus an SDWA or to merge the halves.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ inline f32x2 bf16x2_unpack(unsigned w) {
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ inline unsigned bf16x2_pack(f32x2 v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
// LeakyReLU of a bf16 pair for 0 <= slope <= 1.  max(x, slope*x) is x itself where x >= 0 and
// RNE(slope*x) where x < 0 (the f32 product rounded once more, exactly as the f32 max then
// cast), so the product pair is packed once and each half's sign bit selects: v_pk_mul_f32,
// v_cvt_pk_bf16_f32, v_pk_ashrrev_i16 (sign -> 16-bit mask), v_bfi_b32 -- 6 instructions per pair
// with the unpack, against ~10 for the per-element form (written in C, the bit-select is turned
// into 16-bit compares and cndmasks, so the mask and select are spelled out).
__device__ inline unsigned lrelu_bf16x2(unsigned w, float slope) {
  const unsigned y = bf16x2_pack(bf16x2_unpack(w) * slope);
  unsigned m, r;
  asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(m) : "v"(w));  // 15 for both halves
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(y), "v"(w));
  return r;
}

// 4 / 8 x f32 -> 16-bit T: one v_cvt_pk_{f16,bf16}_f32 per pair
template <typename T>
__device__ inline uint2 pack4(f32x4 v) {
  static_assert(sizeof(T) == 2, "16-bit dtypes only");
  typedef T t4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(uint2, __builtin_convertvector(v, t4));
}
template <typename T>
__device__ inline uint4 pack8(f32x4 a, f32x4 b) {
  const uint2 lo = pack4<T>(a), hi = pack4<T>(b);
  return uint4{lo.x, lo.y, hi.x, hi.y};
}

// LeakyReLU of one 16-byte chunk.  f16 with 0 <= slope <= 1 runs packed:
// max(x, slope*x) as v_pk_mul_f16 + v_pk_max_f16 (8 instructions per chunk instead of ~40
// unpacked converts/compares); slope is then rounded to f16 (0.1 -> 0.09998, within the
// f16 path's tolerance); bf16 in that range runs as pairs (lrelu_bf16x2).  Other dtypes /
// slopes go through f32.
template <typename T>
__device__ inline uint4 lrelu_chunk(uint4 u, float slope) {
  if constexpr (sizeof(T) == 2 && __is_same(T, _Float16)) {
    if (slope >= 0.f && slope <= 1.f) {
      half8 v = *reinterpret_cast<half8*>(&u);
      const half8 s = v * (_Float16)slope;
      v = __builtin_elementwise_max(v, s);
      return *reinterpret_cast<uint4*>(&v);
    }
  }
  if constexpr (__is_same(T, bf16_t)) {
    if (slope >= 0.f && slope <= 1.f)
      return uint4{lrelu_bf16x2(u.x, slope), lrelu_bf16x2(u.y, slope), lrelu_bf16x2(u.z, slope),
                   lrelu_bf16x2(u.w, slope)};
  }
  constexpr int N = 16 / sizeof(T);
  T* e = reinterpret_cast<T*>(&u);
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = (T)leaky((float)e[i], slope);
  return u;
}

// Branch-free LeakyReLU of one 16-byte chunk for 0 <= slope <= 1 (callers validate the slope
// at launch): max(x, slope*x) -- packed f16, bf16 pairs, or f32 per element for f32.  Same
// results as lrelu_chunk in that range, without its runtime slope branch (a uniform branch in
// an epilogue splits the block the scheduler interleaves MFMAs across).
// f16 max of two packed pairs without the IEEE-mode quieting the compiler puts in front of a
// max of loaded values (v_pk_max_f16 x, x, x per operand: 12 instead of 8 instructions per
// chunk); identical results for non-NaN inputs
__device__ inline unsigned pk_max_f16(unsigned a, unsigned b) {
  unsigned r;
  asm("v_pk_max_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <typename T>
__device__ inline uint4 lrelu_unit(uint4 u, float slope) {
  if constexpr (sizeof(T) == 2 && __is_same(T, _Float16)) {
    const half8 v = *reinterpret_cast<half8*>(&u);
    const uint4 m = __builtin_bit_cast(uint4, v * (_Float16)slope);
    return uint4{pk_max_f16(u.x, m.x), pk_max_f16(u.y, m.y), pk_max_f16(u.z, m.z), pk_max_f16(u.w, m.w)};
  } else if constexpr (__is_same(T, bf16_t)) {
    return uint4{lrelu_bf16x2(u.x, slope), lrelu_bf16x2(u.y, slope), lrelu_bf16x2(u.z, slope),
                 lrelu_bf16x2(u.w, slope)};
  } else {
    constexpr int N = 16 / sizeof(T);
    T* e = reinterpret_cast<T*>(&u);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const float x = (float)e[i];
      e[i] = (T)__builtin_fmaxf(x, x * slope);
    }
    return u;
  }
}

// 16-byte store with an explicit cache policy (gfx950 CPol bits: 1 = sc0, 2 = nt, 16 = sc1).
// sc1 stores leave the XCD's L2 (MI355X_MICROARCH.md: "sc1 / sc0 sc1 DROP the line"), so
// outputs the next launch reads from another XCD do not evict this launch's L2-resident
// weights.  base must be wave-uniform; byte_off < 2^31.
template <int POL>
__device__ inline void store16(void* base, int byte_off, uint4 v) {
  if constexpr (POL == 0) {
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(base) + byte_off) = v;
  } else {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, byte_off, 0, POL);
  }
}

// activation codes shared by host and device
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_LRELU = 3, ACT_SILU = 4 };
// compile-time activation tag (epilogues dispatch on the runtime kind once, outside their loops)
template <int A>
struct ActC { static constexpr int value = A; };

__device__ inline float apply_act(float v, int act, float slope) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_TANH: return tanhf(v);
    case ACT_LRELU: return leaky(v, slope);
    case ACT_SILU: return v / (1.f + __expf(-v));
    default: return v;
  }
}

// v_dot2_f32_{f16,bf16}: c + a.lo*b.lo + a.hi*b.hi over packed 16-bit pairs (conv_post)
template <typename T>
struct Dot2;
template <>
struct Dot2<half_t> {
  typedef _Float16 v2 __attribute__((ext_vector_type(2)));
  __device__ static inline float dot(unsigned a, unsigned b, float c) {
    return __builtin_amdgcn_fdot2(*reinterpret_cast<v2*>(&a), *reinterpret_cast<v2*>(&b), c, false);
  }
};
template <>
struct Dot2<bf16_t> {
  typedef __bf16 v2 __attribute__((ext_vector_type(2)));
  __device__ static inline float dot(unsigned a, unsigned b, float c) {
    return __builtin_amdgcn_fdot2_f32_bf16(*reinterpret_cast<v2*>(&a), *reinterpret_cast<v2*>(&b), c, false);
  }
};

}  // namespace tts
