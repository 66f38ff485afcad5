// Row LayerNorm arithmetic shared by the standalone LayerNorm kernels (acoustic_kernels.hip) and
// the GEMM epilogues that apply a post-LN themselves (conv_gemm.hip conv_xres, conv_split.hip
// conv_splitp): one wave per row, fp32 two-pass mean / variance, the same lane layout and wave
// reduction everywhere, so a fused LayerNorm is bit-identical to the separate launch.
//
// Fused form: the blocks that produce one row tile (its M blocks) each store their part with
// write-through (sc1) stores, drain them and add to the tile's counter (Guideline 16 R1, below);
// the last to arrive acquires at agent scope and normalises the tile's rows (cdna_hip_programming.md Guideline 16,
// the counter form of the R1 hand-off).  Counters start at 0 (the workspace is zeroed when it is
// allocated) and the last arriver puts its counter back to 0 for the next launch.
#pragma once
#include "common.h"

// The hand-off's publish is the R1 form of cdna_hip_programming.md Guideline 16: every part is
// stored write-through (sc1, buffer-store aux 16) and drained by its storing wave (vmcnt(0) +
// the block barrier) before the relaxed agent-scope ticket, so the bytes are past every L2 before
// the count can complete ("store payload WRITE-THROUGH (sc1), so no release fence"); the last
// arriver's agent-scope acquire drops its CU's stale lines before its plain loads.  An explicit
// release fence (TTS_LN_RELEASE=1: buffer_wbl2 sc1 + wait per block) writes back the XCD's whole
// L2 and cost 0.3 ms of a 6.1 ms batch-32 forward (profiles/r04b_ab_ln_release.txt); the results
// were bit-identical and run-to-run stable with and without it, the (since removed) in-launch
// split-K reduce included (profiles/r04c_splitk_stability.txt).
#ifndef TTS_LN_RELEASE
#define TTS_LN_RELEASE 0
#endif
#ifndef TTS_LN_FENCE
#define TTS_LN_FENCE 0  // diagnostic builds: __threadfence() in the last arriver instead of the agent acquire
#endif

namespace tts {

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// RB rows at once, one wave per row (independent rows interleave their reductions): v[r][i] are
// the lane's PER values of row r, on[i] whether value i is a channel (< C); g / bb: the lane's
// gains and biases of LN1 (and LN2 when LN2: the second LayerNorm on LN1's output, materialised
// in T).  Every standalone LayerNorm kernel and every fused epilogue normalises through this, so
// their bits agree.
// Every multiply-add below is an explicit fmaf and contraction is off: the compiler vectorises and
// schedules these instances differently (one row vs four interleaved, a standalone kernel vs a GEMM
// epilogue), and an implicit contraction it forms in one and not the other changed the bits.
template <typename T, int RB, int PER, bool LN2>
__device__ inline void ln_batch(float (&v)[RB][PER], const bool (&on)[PER], int C, const float (&g)[2][PER],
                                const float (&bb)[2][PER], float eps) {
#pragma clang fp contract(off)
  const float invC = 1.f / (float)C;
#pragma unroll
  for (int pass = 0; pass < (LN2 ? 2 : 1); ++pass) {
    float mu[RB], rstd[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) sm += v[r][i];
      mu[r] = sm;
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) mu[r] = wave_sum(mu[r]) * invC;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const float d = on[i] ? v[r][i] - mu[r] : 0.f;
        q = fmaf(d, d, q);
      }
      rstd[r] = q;
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) rstd[r] = rsqrtf(fmaf(wave_sum(rstd[r]), invC, eps));
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int i = 0; i < PER; ++i)
        if (on[i]) {
          float y = fmaf((v[r][i] - mu[r]) * rstd[r], g[pass][i], bb[pass][i]);
          // the fp32 result is what gets rounded to T: without this the compiler may fold the
          // multiply-add and the rounding into one v_fma_mix (a single rounding to f16 -- other
          // bits than fp32-then-f16), and does so in some instances only
          asm volatile("" : "+v"(y));
          if (LN2 && pass == 0) y = to_f32(from_f32<T>(y));  // first LN output is materialised in T
          v[r][i] = y;
        }
  }
}

// the lane's gains / biases for ln_batch: channel ch[i] of LN1 and (g2 != null) LN2
template <int PER>
__device__ inline void ln_params(float (&g)[2][PER], float (&bb)[2][PER], const int (&ch)[PER], const bool (&on)[PER],
                                 const float* g1, const float* b1, const float* g2, const float* b2) {
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    g[0][i] = on[i] ? g1[ch[i]] : 0.f;
    bb[0][i] = on[i] ? b1[ch[i]] : 0.f;
    g[1][i] = on[i] && g2 ? g2[ch[i]] : 0.f;
    bb[1][i] = on[i] && g2 ? b2[ch[i]] : 0.f;
  }
}

// the same for a lane owning the contiguous channels c0 .. c0 + 7 (ln_lanes8), 16-byte-aligned
// arrays: two 16-byte loads per array instead of eight 4-byte ones
__device__ inline void ln_load8v(float (&d)[8], bool on, const float* src, int c0) {
  float4 x = float4{0.f, 0.f, 0.f, 0.f}, y = x;
  if (on && src) {
    x = *reinterpret_cast<const float4*>(src + c0);
    y = *reinterpret_cast<const float4*>(src + c0 + 4);
  }
  d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
  d[4] = y.x; d[5] = y.y; d[6] = y.z; d[7] = y.w;
}
__device__ inline void ln_params8v(float (&g)[2][8], float (&bb)[2][8], bool on, int c0, const float* g1,
                                   const float* b1, const float* g2, const float* b2) {
  ln_load8v(g[0], on, g1, c0);
  ln_load8v(bb[0], on, b1, c0);
  ln_load8v(g[1], on, g2, c0);
  ln_load8v(bb[1], on, b2, c0);
}

// LayerNorm + Linear(C -> 1) of RB rows (the variance predictors' last layer, HF:176-181): the LN
// output rounded to T, dotted with w in channel order per lane, wave-summed, + wb -> out[r].
template <typename T, int RB, int PER>
__device__ inline void ln_linear1_batch(float (&v)[RB][PER], const bool (&on)[PER], int C, const float (&g)[PER],
                                        const float (&bb)[PER], const float (&w)[PER], float eps, float wb,
                                        float (&out)[RB]) {
#pragma clang fp contract(off)
  float mu[RB], rstd[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) sm += v[r][i];
    mu[r] = sm;
  }
#pragma unroll
  for (int r = 0; r < RB; ++r) mu[r] = wave_sum(mu[r]) / (float)C;
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const float d = on[i] ? v[r][i] - mu[r] : 0.f;
      q = fmaf(d, d, q);
    }
    rstd[r] = q;
  }
#pragma unroll
  for (int r = 0; r < RB; ++r) rstd[r] = rsqrtf(wave_sum(rstd[r]) / (float)C + eps);
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (on[i]) {
        float y = fmaf((v[r][i] - mu[r]) * rstd[r], g[i], bb[i]);
        asm volatile("" : "+v"(y));  // rounded from fp32 (see ln_batch)
        y = to_f32(from_f32<T>(y));
        dot = fmaf(y, w[i], dot);
      }
    out[r] = dot;
  }
#pragma unroll
  for (int r = 0; r < RB; ++r) out[r] = wave_sum(out[r]) + wb;
}

// lane layouts: 16-bit rows with 16-byte pieces (lane l: channels 8l .. 8l+7), or lane l owning
// channels l + 64 i
__device__ inline void ln_lanes8(int (&ch)[8], bool (&on)[8], int C, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) { ch[i] = 8 * lane + i; on[i] = 8 * lane < C; }
}
template <int PER>
__device__ inline void ln_lanes64(int (&ch)[PER], bool (&on)[PER], int C, int lane) {
#pragma unroll
  for (int i = 0; i < PER; ++i) { ch[i] = lane + 64 * i; on[i] = ch[i] < C; }
}

// 8 x T of a 16-byte piece <-> floats
template <typename T>
__device__ inline void ln_unpack8(uint4 u, float (&v)[8]) {
  const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = to_f32(e[i]);
}
template <typename T>
__device__ inline uint4 ln_pack8(const float (&v)[8]) {
  T o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = from_f32<T>(v[i]);
  return *reinterpret_cast<const uint4*>(o);
}

// Last-arriver hand-off of one row tile produced by `parts` blocks.  Call from every thread after
// the block's last (sc1) store of its part; returns true in the last block, which may then read
// every part with plain loads.  flag: a 4-byte slot of the block's LDS that no wave still reads.
__device__ inline bool ln_tile_last(int* cnt, int parts, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
  __syncthreads();
  if (threadIdx.x == 0) {
    // (TTS_LN_RELEASE builds: an agent-scope release before the ticket, the asm wait after the
    // fence -- Guideline 16 Pitfall 12)
#if TTS_LN_RELEASE
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == parts - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
#if TTS_LN_FENCE
      __threadfence();
#else
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

}  // namespace tts
