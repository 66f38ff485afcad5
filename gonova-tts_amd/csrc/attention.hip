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
//   O^T += Vt . P^T    A = Vt rows (LDS),      B = P^T: the lane's own 8 probabilities
// P^T's k index is permuted (keys 4g..4g+3, 16+4g..16+4g+3 for lane group g) and the Vt
// fragment is read with the same permutation, so no cross-lane move is needed.
#include "acoustic_kernels.h"
#include "common.h"
#include "mrf_tile.h"

namespace tts {

namespace {

constexpr int AT_BQ = 64;   // queries per block
constexpr int AT_BK = 32;   // keys per step
constexpr int AT_RW = AT_BQ + AT_BK;  // R window rows per block (95 used)

template <typename T, int DK>
__global__ __launch_bounds__(256, 2) void rel_attn_kernel(const float* __restrict__ pu, const float* __restrict__ pv,
                                                         const T* __restrict__ qkv, const T* __restrict__ vt,
                                                         const T* __restrict__ ptab, const int* __restrict__ lens,
                                                         int Tp, int D, int H, int Sk, int rmax, float scale,
                                                         T* __restrict__ out, int nqb, int nbatch) {
  using MF = Mfma16<T>;
  typedef typename Mfma<T>::frag Frag;
  constexpr int KS = DK / 32;         // k-steps over dk
  constexpr int DT = DK / 16;         // 16-row tiles of dk (O^T)
  constexpr int KR = DK * 2 + 16;     // K / R row stride in LDS (bytes; odd 16-byte slots)
  constexpr int VR = AT_BK * 2 + 16;  // Vt row stride (80 B)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;                                  // [32 keys][DK]
  char* Vs = Ks + AT_BK * KR;                       // [DK][32 keys]
  char* Rs = Vs + DK * VR;                          // [96 slots][DK]
  float* Gs = reinterpret_cast<float*>(Rs + AT_RW * KR);  // [4 waves][48 slots][16 q]

  // 1-D grid, XCD-grouped: the query blocks of one (utterance, head) -- which all stream the
  // same K / Vt / R rows -- run on one XCD, so those rows come from its L2 after the first
  int bh, qb;
  if (!xcd_tile(nqb, H * nbatch, bh, qb)) return;
  const int b = bh / H, h = bh - b * H;
  const int i0 = qb * AT_BQ;
  const int len = lens[b];
  if (i0 >= len) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane & 15, g = lane >> 4;
  const int i0w = i0 + 16 * w;
  const long long rowD = D;
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
  float* gw = Gs + w * 48 * 16;

  // Staging.  K[j0 .. j0+32) (zero past len) and Vt[:, j0 .. j0+32) per step; the R window
  // (block slot sb <-> m = i0 - j0 - 31 + sb, 96 rows) lives in a 96-row ring indexed by
  // m mod 96: a step shifts the window by 32, so only the 32 rows entering it are loaded,
  // into the slots of the 32 that left.  Loads for step s+1 are issued before step s's
  // MFMAs (registers) and written to LDS after the barrier that ends step s.
  constexpr int KP = AT_BK * (DK / 8) / 256;   // 16-byte pieces per thread: K, Vt, new R rows
  static_assert(AT_BK * (DK / 8) % 256 == 0 && DK * (AT_BK / 8) % 256 == 0, "staging split");
  auto rslot = [](int m) { const int r = m % AT_RW; return r < 0 ? r + AT_RW : r; };
  auto rrow = [&](int m) { return min(max(rmax - 1 - m, 0), 2 * rmax - 1); };
  uint4 pkv[KP], pvt[KP], prr[KP];
  auto stage_load = [&](int j0, bool first) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int p = tid + 256 * i;
      const int r = p / (DK / 8), c = p - r * (DK / 8);
      const int j = j0 + r;
      // addresses clamped into the buffers and the loads consumed unconditionally (a load under
      // a branch or consumed only under a mask makes the waitcnt pass drain vmcnt); keys past
      // len are masked out of the softmax, so their K / Vt only have to be finite
      const uint4 kv = *reinterpret_cast<const uint4*>(qkv + ((long long)b * Tp + min(j, Tp - 1)) * 3 * rowD + D + h * DK + c * 8);
      pkv[i] = j < len ? kv : uint4{0u, 0u, 0u, 0u};
      const int d = p / (AT_BK / 8), cv = p - d * (AT_BK / 8);
      const int jv = j0 + cv * 8;  // Vt is zero past len (transpose_v) and padded to Sk
      const uint4 vv = *reinterpret_cast<const uint4*>(vt + (((long long)b * H + h) * DK + d) * Sk + min(jv, Sk - 8));
      pvt[i] = jv < Sk ? vv : uint4{0u, 0u, 0u, 0u};
      // R rows entering the window: m = i0 - j0 - 31 + [0, 32) (the first step loads all 96 below)
      const int m = i0 - j0 - (AT_BK - 1) + r;
      if (!first) prr[i] = *reinterpret_cast<const uint4*>(ptab + (long long)rrow(m) * rowD + h * DK + c * 8);
    }
  };
  auto stage_write = [&](int j0, bool first) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      const int p = tid + 256 * i;
      const int r = p / (DK / 8), c = p - r * (DK / 8);
      *reinterpret_cast<uint4*>(Ks + r * KR + c * 16) = pkv[i];
      const int d = p / (AT_BK / 8), cv = p - d * (AT_BK / 8);
      *reinterpret_cast<uint4*>(Vs + d * VR + cv * 16) = pvt[i];
      if (!first) {
        const int m = i0 - j0 - (AT_BK - 1) + r;
        *reinterpret_cast<uint4*>(Rs + rslot(m) * KR + c * 16) = prr[i];
      }
    }
  };
  // first step: the whole 96-row R window
  for (int p = tid; p < AT_RW * (DK / 8); p += 256) {
    const int sb = p / (DK / 8), c = p - sb * (DK / 8);
    const int m = i0 - (AT_BK - 1) + sb;
    *reinterpret_cast<uint4*>(Rs + rslot(m) * KR + c * 16) =
        *reinterpret_cast<const uint4*>(ptab + (long long)rrow(m) * rowD + h * DK + c * 8);
  }
  stage_load(0, true);
  stage_write(0, true);
  __syncthreads();

  for (int j0 = 0; j0 < len; j0 += AT_BK) {
    const bool more = j0 + AT_BK < len;
    stage_load(j0 + AT_BK, false);  // in flight during this step's MFMAs (the last step's is unused)
    const int mbw = i0w - j0 - (AT_BK - 1);  // m of this wave's G slot 0
    // S^T tiles (keys 16 kt + 4g + e, query q) and G^T tiles (slots 16 t + 4g + e)
    f32x4 sacc[2] = {f32x4{}, f32x4{}};
    f32x4 gacc[3] = {f32x4{}, f32x4{}, f32x4{}};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const Frag a = *reinterpret_cast<const Frag*>(Ks + (16 * kt + q) * KR + (ks * 32 + 8 * g) * 2);
        sacc[kt] = MF::mma(a, bu[ks], sacc[kt]);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const Frag a = *reinterpret_cast<const Frag*>(Rs + rslot(mbw + 16 * t + q) * KR + (ks * 32 + 8 * g) * 2);
        gacc[t] = MF::mma(a, bv[ks], gacc[t]);
      }
    }
    // G^T -> wave scratch [slot][q]; gather G[q][q - key + 31] for the lane's 8 keys
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) gw[(16 * t + 4 * g + e) * 16 + q] = gacc[t][e];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's scratch writes landed
    __builtin_amdgcn_wave_barrier();
    float sv[8];
    float mloc = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = 16 * kt + 4 * g + e;
        const float bd = gw[(q - kk + AT_BK - 1) * 16 + q];
        float sc = (sacc[kt][e] + bd) * sl2;
        if (j0 + kk >= len) sc = -INFINITY;
        sv[4 * kt + e] = sc;
        mloc = fmaxf(mloc, sc);
      }
    __builtin_amdgcn_wave_barrier();
    // row statistics over the 4 lanes of query q (lanes q, q+16, q+32, q+48)
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = exp2f(m_run - m_new);  // m_run = -inf on the first step: alpha = 0
    float lsum = 0.f;
    T pk[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float pe = exp2f(sv[e] - m_new);
      pk[e] = (T)pe;
      lsum += (float)pk[e];  // normalise with the rounded probabilities P.V uses
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    const Frag bp = *reinterpret_cast<const Frag*>(pk);
    // O^T += Vt . P^T with the permuted key order of bp
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const char* vr = Vs + (16 * t + q) * VR + 8 * g;
      const uint2 lo = *reinterpret_cast<const uint2*>(vr);
      const uint2 hi = *reinterpret_cast<const uint2*>(vr + 32);
      const uint4 av = uint4{lo.x, lo.y, hi.x, hi.y};
      oacc[t] = MF::mma(*reinterpret_cast<const Frag*>(&av), bp, oacc[t] * alpha);
    }
    if (more) {
      __syncthreads();  // every wave is done with this step's K / Vt and the leaving R rows
      stage_write(j0 + AT_BK, false);
      __syncthreads();
    }
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

template <int DK>
size_t rel_attn_lds() {
  return (size_t)AT_BK * (DK * 2 + 16) + (size_t)DK * (AT_BK * 2 + 16) + (size_t)AT_RW * (DK * 2 + 16) +
         (size_t)4 * 48 * 16 * 4;
}

}  // namespace

bool rel_attn_supported(int dt, int D, int H) {
  return (dt == DT_F16 || dt == DT_BF16) && H > 0 && D % H == 0 && D / H == 192;
}

hipError_t launch_rel_attn(int dt, const float* pos_u, const float* pos_v, const void* qkv, const void* vt, const void* ptab,
                           const int* lens, int B, int Tm, int Tp, int D, int H, int Sk, int rmax, float scale,
                           void* out, hipStream_t s) {
  if (!rel_attn_supported(dt, D, H) || Tm > rmax || Sk % 8) return hipErrorInvalidValue;
  const int nqb = (Tm + AT_BQ - 1) / AT_BQ;
  dim3 grid(xcd_grid(nqb, H * B));
  const size_t lds = rel_attn_lds<192>();
  if (dt == DT_F16)
    hipLaunchKernelGGL((rel_attn_kernel<half_t, 192>), grid, dim3(256), lds, s, pos_u, pos_v,
                       (const half_t*)qkv, (const half_t*)vt, (const half_t*)ptab, lens, Tp, D, H, Sk, rmax, scale,
                       (half_t*)out, nqb, B);
  else
    hipLaunchKernelGGL((rel_attn_kernel<bf16_t, 192>), grid, dim3(256), lds, s, pos_u, pos_v,
                       (const bf16_t*)qkv, (const bf16_t*)vt, (const bf16_t*)ptab, lens, Tp, D, H, Sk, rmax, scale,
                       (bf16_t*)out, nqb, B);
  return hipGetLastError();
}

}  // namespace tts
