// Non-GEMM kernels of the FastSpeech2-Conformer acoustic model (oracle/acoustic.py).
// The dense contractions (FFN convs, projections, attention products) run on the
// implicit-GEMM MFMA kernel (conv_gemm.hip); these are the row-wise / integer steps.
//
// Activations: [B][Tm][C] channels-last in the compute dtype T; per-utterance valid
// lengths `lens[b]` give B=1 semantics (rows >= len are never read by valid rows).
#include <cstdint>
#include <cstdlib>

#include "acoustic_kernels.h"
#include "common.h"
#include "ln_rows.h"

namespace tts {

// ---------------------------------------------------------------------------
// token embedding * sqrt(D)   (HF:793-795 embed, HF:763 input_scale)
// ---------------------------------------------------------------------------
template <typename T>
__global__ void embed_kernel(const int* __restrict__ ids, const int* __restrict__ lens, int N, int Tm,
                             const T* __restrict__ E, int V, int D, float scale, T* __restrict__ out) {
  const int b = blockIdx.y;
  const int t = blockIdx.x;
  const int L = min(lens[b], N);
  T* o = out + ((long long)b * Tm + t) * D;
  if (t >= L) {
    for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = from_f32<T>(0.f);
    return;
  }
  int id = ids[(long long)b * N + t];
  id = min(max(id, 0), V - 1);
  const T* e = E + (long long)id * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = from_f32<T>(to_f32(e[c]) * scale);
}

// ---------------------------------------------------------------------------
// LayerNorm over C (one wave per row), optional second LayerNorm applied after
// (ff_layer_norm followed by final_layer_norm, HF:644-647).  Two-pass variance in fp32.
// ---------------------------------------------------------------------------

// lens (optional): rows are [B][stride]; row r of utterance b is skipped when r >= lens[b] (the
// padding past each utterance: no consumer reads it, every kernel masks rows >= len on load)
__device__ inline bool ln_row_valid(int row, const int* lens, int stride) {
  if (!lens) return true;
  const int b = row / stride;
  return row - b * stride < lens[b];
}

template <typename T, int PER>
__global__ __launch_bounds__(256) void layernorm_kernel(const T* __restrict__ in, T* __restrict__ out, int rows,
                                                       int C, const float* __restrict__ g1,
                                                       const float* __restrict__ b1, const float* __restrict__ g2,
                                                       const float* __restrict__ b2, float eps, const int* lens,
                                                       int stride) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows || !ln_row_valid(row, lens, stride)) return;
  const T* x = in + (long long)row * C;
  int ch[PER];
  bool on[PER];
  ln_lanes64<PER>(ch, on, C, lane);  // ln_rows.h
  float g[2][PER], bb[2][PER], v[1][PER];
  ln_params<PER>(g, bb, ch, on, g1, b1, g2, b2);
#pragma unroll
  for (int i = 0; i < PER; ++i) v[0][i] = on[i] ? to_f32(x[ch[i]]) : 0.f;
  if (g2) ln_batch<T, 1, PER, true>(v, on, C, g, bb, eps);
  else ln_batch<T, 1, PER, false>(v, on, C, g, bb, eps);
  T* o = out + (long long)row * C;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (on[i]) o[ch[i]] = from_f32<T>(v[0][i]);
}

// G LayerNorms of C channels side by side in rows of ld elements, in place, one launch (blockIdx.y
// = group g: channels [g*C, (g+1)*C) with its own gain and bias): the variance predictors' first
// LayerNorms after their batched first conv.  Per row segment the arithmetic of layernorm_kernel.
template <typename T, int PER>
__global__ __launch_bounds__(256) void layernorm_groups_kernel(T* __restrict__ x, int rows, int C, int ld,
                                                              LnGroups gp, float eps, const int* lens, int stride) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int grp = blockIdx.y;
  if (row >= rows || !ln_row_valid(row, lens, stride)) return;
  T* xr = x + (long long)row * ld + (long long)grp * C;
  int ch[PER];
  bool on[PER];
  ln_lanes64<PER>(ch, on, C, lane);
  float g[2][PER], bb[2][PER], v[1][PER];
  ln_params<PER>(g, bb, ch, on, gp.g[grp], gp.b[grp], nullptr, nullptr);
#pragma unroll
  for (int i = 0; i < PER; ++i) v[0][i] = on[i] ? to_f32(xr[ch[i]]) : 0.f;
  ln_batch<T, 1, PER, false>(v, on, C, g, bb, eps);
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (on[i]) xr[ch[i]] = from_f32<T>(v[0][i]);
}

// ---------------------------------------------------------------------------
// attention prep: Qu = q + pos_bias_u, Qv = q + pos_bias_v (HF:420-423) from QKV [rows][3D]
// ---------------------------------------------------------------------------
template <typename T>
__global__ void pos_bias_kernel(const T* __restrict__ qkv, int rows, int D, const float* __restrict__ u,
                                const float* __restrict__ v, T* __restrict__ qu, T* __restrict__ qv) {
  const long long n = (long long)rows * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / D;
    const int c = (int)(i - r * D);
    const float q = to_f32(qkv[r * 3 * D + c]);
    qu[i] = from_f32<T>(q + u[c]);
    qv[i] = from_f32<T>(q + v[c]);
  }
}

// Vt[b][h][d][j] = v[b][j][h*dk + d] for j < len[b], 0 for len <= j < Sk
template <typename T>
__global__ void transpose_v_kernel(const T* __restrict__ qkv, const int* __restrict__ lens, int Tm, int D, int H,
                                   int Sk, T* __restrict__ vt) {
  __shared__ float tile[32][33];
  const int dk = D / H;
  const int bh = blockIdx.z;
  const int b = bh / H, h = bh - b * H;
  const int L = min(lens[b], Tm);
  const int j0 = blockIdx.x * 32, d0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int j = j0 + r, d = d0 + tx;
    float val = 0.f;
    if (j < L && d < dk) val = to_f32(qkv[((long long)b * Tm + j) * 3 * D + 2 * D + h * dk + d]);
    tile[r][tx] = val;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int d = d0 + r, j = j0 + tx;
    if (d < dk && j < Sk) vt[(((long long)b * H + h) * dk + d) * Sk + j] = from_f32<T>(tile[tx][r]);
  }
}

// 16-bit Vt for dk % 64 == 0, Sk % 8 == 0: 64 keys x 64 channels per block, 16-byte loads of
// 8 channels of one key and 16-byte stores of 8 keys of one channel through an LDS tile (row
// stride 72 elements: the column reads of a row group hit distinct banks).  The bits are copied
// (the f32 round trip of the generic kernel is exact for 16-bit values); keys >= len are 0.
template <typename T>
__global__ __launch_bounds__(256) void transpose_v16_kernel(const T* __restrict__ qkv, const int* __restrict__ lens,
                                                            int Tm, int D, int H, int Sk, T* __restrict__ vt) {
  constexpr int TS = 72;  // LDS row stride (elements)
  __shared__ __attribute__((aligned(16))) T tile[64 * TS];
  const int dk = D / H;
  const int bh = blockIdx.z;
  const int b = bh / H, h = bh - b * H;
  const int L = min(lens[b], Tm);
  const int j0 = blockIdx.x * 64, d0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + 256 * i;
    const int r = p >> 3, c = p & 7;
    const int j = j0 + r;
    uint4 u = uint4{0u, 0u, 0u, 0u};
    if (j < L) u = *reinterpret_cast<const uint4*>(qkv + ((long long)b * Tm + j) * 3 * D + 2 * D + h * dk + d0 + 8 * c);
    *reinterpret_cast<uint4*>(tile + r * TS + 8 * c) = u;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tid + 256 * i;
    const int d = p >> 3, jc = p & 7;
    const int j = j0 + 8 * jc;
    if (j >= Sk) continue;
    T o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = tile[(8 * jc + e) * TS + d];
    *reinterpret_cast<uint4*>(vt + (((long long)b * H + h) * dk + d0 + d) * Sk + j) = *reinterpret_cast<const uint4*>(o);
  }
}

// ---------------------------------------------------------------------------
// scores = (AC[i][j] + BD[i][(Tm-1) - i + j]) / sqrt(dk), key-masked softmax (HF:430-449,
// shift_relative_position_tensor HF:381-393).  One wave per query row.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void rel_softmax_kernel(const T* __restrict__ ac, const T* __restrict__ bd,
                                                         const int* __restrict__ lens, int H, int Tm, int Sac,
                                                         int Sbd, int Sk, float scale, T* __restrict__ pout) {
  const int bh = blockIdx.y;
  const int b = bh / H;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= Tm) return;
  const int L = max(min(lens[b], Tm), 1);
  const T* acr = ac + ((long long)bh * Tm + i) * Sac;
  const T* bdr = bd + ((long long)bh * Tm + i) * Sbd + (Tm - 1 - i);
  T* pr = pout + ((long long)bh * Tm + i) * Sk;
  float mx = -INFINITY;
  for (int j = lane; j < L; j += 64) {
    const float s = (to_f32(acr[j]) + to_f32(bdr[j])) * scale;
    mx = fmaxf(mx, s);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
  for (int j = lane; j < L; j += 64) sum += __expf((to_f32(acr[j]) + to_f32(bdr[j])) * scale - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  for (int j = lane; j < Sk; j += 64) {
    float pv = 0.f;
    if (j < L) pv = __expf((to_f32(acr[j]) + to_f32(bdr[j])) * scale - mx) * inv;
    pr[j] = from_f32<T>(pv);
  }
}

// ---------------------------------------------------------------------------
// Conformer conv module core (HF:501-535): g = a[:, :D] * sigmoid(a[:, D:]) (GLU),
// depthwise conv k (zero padded per utterance), BatchNorm folded into (w, b), SiLU.
// Block: 64 channels x TR rows; LDS holds the GLU output with the halo in fp32.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void glu_dwconv_kernel(const T* __restrict__ a, const int* __restrict__ lens,
                                                        int Tm, int D, const float* __restrict__ w, int k,
                                                        const float* __restrict__ bias, T* __restrict__ out) {
  constexpr int TR = 128, CB = 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* g = reinterpret_cast<float*>(smem);  // [(TR + k - 1)][CB]
  const int b = blockIdx.z;
  const int t0 = blockIdx.x * TR;
  const int c0 = blockIdx.y * CB;
  const int L = min(lens[b], Tm);
  if (t0 >= L) return;
  const int pad = (k - 1) / 2;
  const int rows = TR + k - 1;
  const T* ab = a + (long long)b * Tm * 2 * D;
  for (int i = threadIdx.x; i < rows * CB; i += 256) {
    const int r = i / CB, c = i - r * CB;
    const int t = t0 - pad + r;
    float val = 0.f;
    if (t >= 0 && t < L && c0 + c < D) {
      const float x = to_f32(ab[(long long)t * 2 * D + c0 + c]);
      const float gt = to_f32(ab[(long long)t * 2 * D + D + c0 + c]);
      val = x * (1.f / (1.f + __expf(-gt)));
    }
    g[i] = val;
  }
  __syncthreads();
  const int c = threadIdx.x & (CB - 1);
  const int rg = threadIdx.x / CB;  // 4 row groups
  if (c0 + c >= D) return;
  const float* wc = w + (long long)(c0 + c) * k;
  const float bc = bias[c0 + c];
  T* ob = out + (long long)b * Tm * D;
  for (int r = rg; r < TR; r += 4) {
    const int t = t0 + r;
    if (t >= L) break;
    float acc = bc;
    for (int j = 0; j < k; ++j) acc = fmaf(wc[j], g[(r + j) * CB + c], acc);
    const float y = acc / (1.f + __expf(-acc));  // SiLU
    ob[(long long)t * D + c0 + c] = from_f32<T>(y);
  }
}

// The same with a compile-time kernel size (the conformer's 7 / 31): 16-byte GLU loads
// (8 x 16-bit or 4 x f32 channels of x and of the gate per load), and a register sliding
// window per thread: one channel x RPT consecutive rows reads RPT + K - 1 LDS values for
// RPT * K FMAs (the generic kernel above reads K LDS values per output).  HBM-bound: reads
// the [rows][2D] GLU input once (+ halo), writes [rows][D] once.
template <typename T, int K>
__global__ __launch_bounds__(256) void glu_dwconv_k_kernel(const T* __restrict__ a, const int* __restrict__ lens,
                                                          int Tm, int D, const float* __restrict__ w,
                                                          const float* __restrict__ bias, T* __restrict__ out) {
  constexpr int TR = 128, CB = 64, RPT = TR / 4, PAD = (K - 1) / 2, ROWS = TR + K - 1;
  constexpr int EPP = 16 / (int)sizeof(T);   // channels per 16-byte piece
  constexpr int PPR = CB / EPP;              // pieces per staged row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* g = reinterpret_cast<float*>(smem);  // [ROWS][CB] GLU output, fp32
  const int b = blockIdx.z;
  const int t0 = blockIdx.x * TR;
  const int c0 = blockIdx.y * CB;
  const int L = min(lens[b], Tm);
  if (t0 >= L) return;
  const T* ab = a + (long long)b * Tm * 2 * D;
  for (int i = threadIdx.x; i < ROWS * PPR; i += 256) {
    const int r = i / PPR, pc = i - r * PPR;
    const int t = t0 - PAD + r;
    const int c = c0 + pc * EPP;
    float v[EPP];
    if (t >= 0 && t < L && c < D) {
      const uint4 xu = *reinterpret_cast<const uint4*>(ab + (long long)t * 2 * D + c);
      const uint4 gu = *reinterpret_cast<const uint4*>(ab + (long long)t * 2 * D + D + c);
      const T* xe = reinterpret_cast<const T*>(&xu);
      const T* ge = reinterpret_cast<const T*>(&gu);
#pragma unroll
      for (int e = 0; e < EPP; ++e) v[e] = to_f32(xe[e]) * (1.f / (1.f + __expf(-to_f32(ge[e]))));
    } else {
#pragma unroll
      for (int e = 0; e < EPP; ++e) v[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < EPP; e += 4)
      *reinterpret_cast<f32x4*>(g + r * CB + pc * EPP + e) = f32x4{v[e], v[e + 1], v[e + 2], v[e + 3]};
  }
  __syncthreads();
  const int c = threadIdx.x & (CB - 1);
  const int r0 = (threadIdx.x / CB) * RPT;
  if (c0 + c >= D || t0 + r0 >= L) return;
  float wk[K];
#pragma unroll
  for (int j = 0; j < K; ++j) wk[j] = w[(long long)(c0 + c) * K + j];
  const float bc = bias[c0 + c];
  float win[RPT + K - 1];
#pragma unroll
  for (int i = 0; i < RPT + K - 1; ++i) win[i] = g[(r0 + i) * CB + c];
  T* ob = out + (long long)b * Tm * D + c0 + c;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    float acc = bc;
#pragma unroll
    for (int j = 0; j < K; ++j) acc = fmaf(wk[j], win[r + j], acc);
    const int t = t0 + r0 + r;
    if (t < L) ob[(long long)t * D] = from_f32<T>(acc / (1.f + __expf(-acc)));  // SiLU
  }
}

// ---------------------------------------------------------------------------
// Speaker-embedding term of the projection after the encoder (HF:1192-1196):
//   c[b][o] = bias[o] + sum_i We[o][i] * e[b][i] / max(||e[b]||, 1e-12)
// (F.normalize), the part of Linear(concat(h, e)) that is constant over an utterance's
// frames; the hidden part runs as a k=1 conv with c broadcast as its residual.  One block
// per utterance: a block reduction for the norm, then one output channel per thread.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void spk_bias_kernel(const float* __restrict__ e, int E,
                                                      const float* __restrict__ We, const float* __restrict__ bias,
                                                      int D, T* __restrict__ out) {
  __shared__ float red[256];
  const int b = blockIdx.x;
  const float* eb = e + (long long)b * E;
  float ss = 0.f;
  for (int i = threadIdx.x; i < E; i += 256) ss = fmaf(eb[i], eb[i], ss);
  red[threadIdx.x] = ss;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const float inv = 1.f / fmaxf(sqrtf(red[0]), 1e-12f);
  for (int o = threadIdx.x; o < D; o += 256) {
    const float* wr = We + (long long)o * E;
    float acc = 0.f;
    for (int i = 0; i < E; ++i) acc = fmaf(wr[i], eb[i], acc);
    out[(long long)b * D + o] = from_f32<T>(bias[o] + acc * inv);
  }
}

// ---------------------------------------------------------------------------
// variance-predictor head: LayerNorm(C) then Linear(C -> 1) (HF:261-271, 318)
// ---------------------------------------------------------------------------
template <typename T, int PER>
__global__ __launch_bounds__(256) void ln_linear1_kernel(const T* __restrict__ in, int rows, int C,
                                                        const float* __restrict__ g, const float* __restrict__ bb,
                                                        float eps, const float* __restrict__ w, float wb,
                                                        float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* x = in + (long long)row * C;
  int ch[PER];
  bool on[PER];
  ln_lanes64<PER>(ch, on, C, lane);  // ln_rows.h
  float gl[PER], bl[PER], wl[PER], v[1][PER], o[1];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    gl[i] = on[i] ? g[ch[i]] : 0.f;
    bl[i] = on[i] ? bb[ch[i]] : 0.f;
    wl[i] = on[i] ? w[ch[i]] : 0.f;
    v[0][i] = on[i] ? to_f32(x[ch[i]]) : 0.f;
  }
  ln_linear1_batch<T, 1, PER>(v, on, C, gl, bl, wl, eps, wb, o);
  if (lane == 0) out[row] = o[0];
}

// ---------------------------------------------------------------------------
// durations (HF:183 clamp(round(exp(x) - 1), 0); length_regulator speed + all-zero rule
// HF:104-109, per utterance), exclusive prefix sums, mel lengths (clamped to Tcap) and the
// frame -> token map.  One block per utterance.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void durations_kernel(const float* __restrict__ logd, const int* __restrict__ lens,
                                                       int N, const int* __restrict__ override_d, float speed,
                                                       int Tcap, int* __restrict__ dur, int* __restrict__ mel_lens,
                                                       int* __restrict__ tokmap) {
  extern __shared__ int sm[];  // cum[N + 1]
  __shared__ int total;
  const int b = blockIdx.x;
  const int L = min(lens[b], N);
  int* cum = sm;
  for (int t = threadIdx.x; t < N; t += blockDim.x) {
    int d = 0;
    if (t < L) {
      if (override_d) {
        d = max(override_d[(long long)b * N + t], 0);
      } else {
        const float x = logd[(long long)b * N + t];
        d = (int)fmaxf(rintf(expf(x) - 1.0f), 0.f);  // rint = round half to even, like torch.round
      }
      if (speed != 1.0f) d = (int)rintf((float)d * speed);
    }
    cum[t + 1] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cum[0] = 0;
    int s = 0;
    for (int t = 1; t <= N; ++t) s += cum[t];
    if (s == 0 && L > 0) {  // all-zero rule: every token gets one frame
      for (int t = 1; t <= N; ++t) cum[t] = (t <= L) ? 1 : 0;
    }
    for (int t = 1; t <= N; ++t) cum[t] += cum[t - 1];  // inclusive -> cumulative
    total = min(cum[N], Tcap);
    mel_lens[b] = total;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < N; t += blockDim.x) dur[(long long)b * N + t] = cum[t + 1] - cum[t];
  const int tot = total;
  for (int f = threadIdx.x; f < Tcap; f += blockDim.x) {
    int tok = -1;
    if (f < tot) {
      int lo = 0, hi = N - 1;  // first t with cum[t+1] > f
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cum[mid + 1] > f) hi = mid; else lo = mid + 1;
      }
      tok = lo;
    }
    tokmap[(long long)b * Tcap + f] = tok;
  }
}

// x[row][c] = (x + (e[row] * we[c] + be[c])) + (p[row] * wp[c] + bp[c])    (HF:1216-1218)
template <typename T>
__global__ void var_embed_add_kernel(T* __restrict__ x, int rows, int D, const float* __restrict__ e,
                                     const float* __restrict__ we, const float* __restrict__ be,
                                     const float* __restrict__ p, const float* __restrict__ wp,
                                     const float* __restrict__ bp) {
  const long long n = (long long)rows * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / D;
    const int c = (int)(i - r * D);
    const float ee = to_f32(from_f32<T>(e[r] * we[c] + be[c]));
    const float pp = to_f32(from_f32<T>(p[r] * wp[c] + bp[c]));
    const float y = to_f32(from_f32<T>(to_f32(x[i]) + ee));
    x[i] = from_f32<T>(y + pp);
  }
}

// length regulator gather (HF:82-126) fused with the decoder's input_scale (HF:763); the encoder
// side may be fp32 (TTS_ENCODER_EXACT) while the decoder runs 16-bit: one rounding, after the scale
template <typename T, typename TI = T>
__global__ void regulate_kernel(const TI* __restrict__ enc, int N, int D, const int* __restrict__ tokmap, int Tcap,
                                int Tout, float scale, T* __restrict__ out) {
  const int b = blockIdx.y;
  const int f = blockIdx.x;
  const int tok = tokmap[(long long)b * Tcap + f];
  T* o = out + ((long long)b * Tout + f) * D;
  if (tok < 0) {
    for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = from_f32<T>(0.f);
    return;
  }
  const TI* s = enc + ((long long)b * N + tok) * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = from_f32<T>(to_f32(s[c]) * scale);
}

// mel [B][Tin][C] (T, row stride Tin >= mel_len) -> float32 [B][Tcap][C], rows >= mel_len zeroed
template <typename T>
__global__ void mel_out_kernel(const T* __restrict__ in, const int* __restrict__ mel_lens, int Tin, int Tcap, int C,
                               float* __restrict__ out) {
  const int b = blockIdx.y;
  const long long n = (long long)Tcap * C;
  const int L = mel_lens[b];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / C);
    out[(long long)b * n + i] = t < L ? to_f32(in[(long long)b * Tin * C + i]) : 0.f;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
#define TTS_DISPATCH(dtype, KERNEL_CALL)                       \
  switch (dtype) {                                             \
    case DT_F32: { typedef float TT; KERNEL_CALL; break; }     \
    case DT_F16: { typedef half_t TT; KERNEL_CALL; break; }    \
    case DT_BF16: { typedef bf16_t TT; KERNEL_CALL; break; }   \
    default: return hipErrorInvalidValue;                      \
  }                                                            \
  return hipGetLastError();

static unsigned grid1(long long n) { long long g = (n + 255) / 256; return (unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096); }

hipError_t launch_embed(int dt, const int* ids, const int* lens, int B, int N, int Tm, const void* E, int V, int D,
                        float scale, void* out, hipStream_t s) {
  TTS_DISPATCH(dt, hipLaunchKernelGGL(embed_kernel<TT>, dim3(Tm, B), dim3(128), 0, s, ids, lens, N, Tm,
                                      (const TT*)E, V, D, scale, (TT*)out));
}

#ifndef TTS_LN8_RB
#define TTS_LN8_RB 1  // rows per wave of layernorm8_kernel (batch-8 decoder post-LNs: 1 110 us, 2 127 us, 4 148 us for 16 launches)
#endif

// 16-bit rows of C <= 512 channels, C % 8 == 0: one 16-byte load / store per lane (lane l
// owns channels 8l .. 8l+7), RB rows per wave normalised together (ln_batch interleaves their
// reductions), same arithmetic as layernorm_kernel.  VEC: the gains / biases are 16-byte
// aligned and load as two 16-byte pieces per lane.  The first version loaded them as eight
// 4-byte loads per lane and array, 32 B apart across the wave (16 cache lines per load
// instruction) for every row: at batch 8 the decoder's post-LNs (6912 rows x 384) took
// 14 us (one LayerNorm) / 23 us (two) per launch for 10.6 MB.
template <typename T, int RB, bool VEC>
__global__ __launch_bounds__(256) void layernorm8_kernel(const T* __restrict__ in, T* __restrict__ out, int rows,
                                                        int C, const float* __restrict__ g1,
                                                        const float* __restrict__ b1, const float* __restrict__ g2,
                                                        const float* __restrict__ b2, float eps, const int* lens,
                                                        int stride) {
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RB;
  const int lane = threadIdx.x & 63;
  if (row0 >= rows) return;
  int ch[8];
  bool on[8];
  ln_lanes8(ch, on, C, lane);  // ln_rows.h
  float g[2][8], bb[2][8], v[RB][8];
  if constexpr (VEC) ln_params8v(g, bb, on[0], ch[0], g1, b1, g2, b2);
  else ln_params<8>(g, bb, ch, on, g1, b1, g2, b2);
  bool ok[RB];
  uint4 u[RB];
#pragma unroll
  for (int k = 0; k < RB; ++k) {
    const int row = row0 + k;
    ok[k] = row < rows && ln_row_valid(row, lens, stride);
    u[k] = uint4{0u, 0u, 0u, 0u};
    if (ok[k] && on[0]) u[k] = *reinterpret_cast<const uint4*>(in + (long long)row * C + ch[0]);
  }
#pragma unroll
  for (int k = 0; k < RB; ++k) ln_unpack8<T>(u[k], v[k]);
  if (g2) ln_batch<T, RB, 8, true>(v, on, C, g, bb, eps);
  else ln_batch<T, RB, 8, false>(v, on, C, g, bb, eps);
#pragma unroll
  for (int k = 0; k < RB; ++k)
    if (ok[k] && on[0]) *reinterpret_cast<uint4*>(out + (long long)(row0 + k) * C + ch[0]) = ln_pack8<T>(v[k]);
}

template <typename T>
static void launch_ln8(const T* in, T* out, int rows, int C, const float* g1, const float* b1, const float* g2,
                       const float* b2, float eps, hipStream_t s, const int* lens, int stride) {
  static const int rb_env = getenv("TTS_LN8_RB") ? atoi(getenv("TTS_LN8_RB")) : 0;  // A/B: rows per wave
  const bool vec = ((reinterpret_cast<uintptr_t>(g1) | reinterpret_cast<uintptr_t>(b1) |
                     reinterpret_cast<uintptr_t>(g2) | reinterpret_cast<uintptr_t>(b2)) & 15) == 0;
  const int rb = rb_env == 1 || rb_env == 2 || rb_env == 4 ? rb_env : TTS_LN8_RB;
  const dim3 grid((rows + 4 * rb - 1) / (4 * rb));
#define TTS_LN8(RB_, VEC_) \
  hipLaunchKernelGGL((layernorm8_kernel<T, RB_, VEC_>), grid, dim3(256), 0, s, in, out, rows, C, g1, b1, g2, b2, eps, lens, stride)
  if (!vec) TTS_LN8(1, false);
  else if (rb == 1) TTS_LN8(1, true);
  else if (rb == 2) TTS_LN8(2, true);
  else TTS_LN8(4, true);
#undef TTS_LN8
}

hipError_t launch_layernorm(int dt, const void* in, void* out, int rows, int C, const float* g1, const float* b1,
                            const float* g2, const float* b2, float eps, hipStream_t s, const int* lens, int stride) {
  if (C > 512 || (lens && stride <= 0)) return hipErrorInvalidValue;
  dim3 grid((rows + 3) / 4);
  if (dt != DT_F32 && C % 8 == 0) {
    if (dt == DT_F16)
      launch_ln8((const half_t*)in, (half_t*)out, rows, C, g1, b1, g2, b2, eps, s, lens, stride);
    else
      launch_ln8((const bf16_t*)in, (bf16_t*)out, rows, C, g1, b1, g2, b2, eps, s, lens, stride);
    return hipGetLastError();
  }
  if (C <= 256) {
    TTS_DISPATCH(dt, hipLaunchKernelGGL((layernorm_kernel<TT, 4>), grid, dim3(256), 0, s, (const TT*)in, (TT*)out,
                                        rows, C, g1, b1, g2, b2, eps, lens, stride));
  }
  TTS_DISPATCH(dt, hipLaunchKernelGGL((layernorm_kernel<TT, 8>), grid, dim3(256), 0, s, (const TT*)in, (TT*)out, rows,
                                      C, g1, b1, g2, b2, eps, lens, stride));
}

hipError_t launch_layernorm_groups(int dt, void* x, int rows, int C, int ld, const LnGroups& gp, int groups, float eps,
                                   hipStream_t s, const int* lens, int stride) {
  if (C > 256 || groups < 1 || groups > LnGroups::MAXG || ld < groups * C || (lens && stride <= 0))
    return hipErrorInvalidValue;
  dim3 grid((rows + 3) / 4, groups);
  TTS_DISPATCH(dt, hipLaunchKernelGGL((layernorm_groups_kernel<TT, 4>), grid, dim3(256), 0, s, (TT*)x, rows, C, ld, gp,
                                      eps, lens, stride));
}

hipError_t launch_pos_bias(int dt, const void* qkv, int rows, int D, const float* u, const float* v, void* qu,
                           void* qv, hipStream_t s) {
  TTS_DISPATCH(dt, hipLaunchKernelGGL(pos_bias_kernel<TT>, dim3(grid1((long long)rows * D)), dim3(256), 0, s,
                                      (const TT*)qkv, rows, D, u, v, (TT*)qu, (TT*)qv));
}

hipError_t launch_transpose_v(int dt, const void* qkv, const int* lens, int B, int Tm, int D, int H, int Sk, void* vt,
                              hipStream_t s) {
  if (dt != DT_F32 && (D / H) % 64 == 0 && Sk % 8 == 0) {
    dim3 g16((Sk + 63) / 64, (D / H) / 64, B * H);
    if (dt == DT_F16)
      hipLaunchKernelGGL(transpose_v16_kernel<half_t>, g16, dim3(256), 0, s, (const half_t*)qkv, lens, Tm, D, H, Sk,
                         (half_t*)vt);
    else
      hipLaunchKernelGGL(transpose_v16_kernel<bf16_t>, g16, dim3(256), 0, s, (const bf16_t*)qkv, lens, Tm, D, H, Sk,
                         (bf16_t*)vt);
    return hipGetLastError();
  }
  dim3 grid((Sk + 31) / 32, (D / H + 31) / 32, B * H);
  TTS_DISPATCH(dt, hipLaunchKernelGGL(transpose_v_kernel<TT>, grid, dim3(256), 0, s, (const TT*)qkv, lens, Tm, D, H,
                                      Sk, (TT*)vt));
}

hipError_t launch_rel_softmax(int dt, const void* ac, const void* bd, const int* lens, int B, int H, int Tm, int Sac,
                              int Sbd, int Sk, float scale, void* p, hipStream_t s) {
  dim3 grid((Tm + 3) / 4, B * H);
  TTS_DISPATCH(dt, hipLaunchKernelGGL(rel_softmax_kernel<TT>, grid, dim3(256), 0, s, (const TT*)ac, (const TT*)bd,
                                      lens, H, Tm, Sac, Sbd, Sk, scale, (TT*)p));
}

hipError_t launch_glu_dwconv(int dt, const void* a, const int* lens, int B, int Tm, int D, const float* w, int k,
                             const float* bias, void* out, hipStream_t s) {
  dim3 grid((Tm + 127) / 128, (D + 63) / 64, B);
  const int epp = dt == DT_F32 ? 4 : 8;
  if ((k == 7 || k == 31) && D % epp == 0) {
    const size_t ldsk = (size_t)(128 + k - 1) * 64 * 4;
    if (k == 7) {  // (TTS_DISPATCH returns)
      TTS_DISPATCH(dt, hipLaunchKernelGGL((glu_dwconv_k_kernel<TT, 7>), grid, dim3(256), ldsk, s, (const TT*)a, lens,
                                          Tm, D, w, bias, (TT*)out));
    }
    TTS_DISPATCH(dt, hipLaunchKernelGGL((glu_dwconv_k_kernel<TT, 31>), grid, dim3(256), ldsk, s, (const TT*)a, lens,
                                        Tm, D, w, bias, (TT*)out));
  }
  const size_t lds = (size_t)(128 + k - 1) * 64 * 4;
  TTS_DISPATCH(dt, hipLaunchKernelGGL(glu_dwconv_kernel<TT>, grid, dim3(256), lds, s, (const TT*)a, lens, Tm, D, w, k,
                                      bias, (TT*)out));
}

hipError_t launch_ln_linear1(int dt, const void* in, int rows, int C, const float* g, const float* b, float eps,
                             const float* w, float wb, float* out, hipStream_t s) {
  if (C > 256) return hipErrorInvalidValue;
  TTS_DISPATCH(dt, hipLaunchKernelGGL((ln_linear1_kernel<TT, 4>), dim3((rows + 3) / 4), dim3(256), 0, s,
                                      (const TT*)in, rows, C, g, b, eps, w, wb, out));
}

hipError_t launch_durations(const float* logd, const int* lens, int B, int N, const int* override_d, float speed,
                            int Tcap, int* dur, int* mel_lens, int* tokmap, hipStream_t s) {
  hipLaunchKernelGGL(durations_kernel, dim3(B), dim3(256), (size_t)(N + 1) * sizeof(int), s, logd, lens, N,
                     override_d, speed, Tcap, dur, mel_lens, tokmap);
  return hipGetLastError();
}

hipError_t launch_var_embed_add(int dt, void* x, int rows, int D, const float* e, const float* we, const float* be,
                                const float* p, const float* wp, const float* bp, hipStream_t s) {
  TTS_DISPATCH(dt, hipLaunchKernelGGL(var_embed_add_kernel<TT>, dim3(grid1((long long)rows * D)), dim3(256), 0, s,
                                      (TT*)x, rows, D, e, we, be, p, wp, bp));
}

hipError_t launch_regulate(int dt_in, int dt, const void* enc, int B, int N, int D, const int* tokmap, int Tcap,
                           int frames, int Tout, float scale, void* out, hipStream_t s) {
  if (frames > Tcap || frames > Tout) return hipErrorInvalidValue;
  if (dt_in == DT_F32 && dt != DT_F32) {
    TTS_DISPATCH(dt, hipLaunchKernelGGL((regulate_kernel<TT, float>), dim3(frames, B), dim3(128), 0, s,
                                        (const float*)enc, N, D, tokmap, Tcap, Tout, scale, (TT*)out));
  }
  if (dt_in != dt) return hipErrorInvalidValue;
  TTS_DISPATCH(dt, hipLaunchKernelGGL(regulate_kernel<TT>, dim3(frames, B), dim3(128), 0, s, (const TT*)enc, N, D,
                                      tokmap, Tcap, Tout, scale, (TT*)out));
}

hipError_t launch_mel_out(int dt, const void* in, const int* mel_lens, int B, int Tin, int Tcap, int C, float* out,
                          hipStream_t s) {
  dim3 grid(grid1((long long)Tcap * C), B);
  TTS_DISPATCH(dt, hipLaunchKernelGGL(mel_out_kernel<TT>, grid, dim3(256), 0, s, (const TT*)in, mel_lens, Tin, Tcap,
                                      C, out));
}

// range word read-out (tts_acoustic_range_flag): copy the word to the caller's device buffer and
// clear it, one launch instead of a copy and a fill
__global__ void range_take_kernel(int* __restrict__ src, int* __restrict__ dst) {
  if (threadIdx.x == 0) {
    dst[0] = src[0];
    src[0] = 0;
  }
}

hipError_t launch_range_take(int* src, int* dst, hipStream_t s) {
  hipLaunchKernelGGL(range_take_kernel, dim3(1), dim3(64), 0, s, src, dst);
  return hipGetLastError();
}

hipError_t launch_spk_bias(int dt, const float* e, int B, int E, const float* We, const float* bias, int D, void* out,
                           hipStream_t s) {
  TTS_DISPATCH(dt, hipLaunchKernelGGL(spk_bias_kernel<TT>, dim3(B), dim3(256), 0, s, e, E, We, bias, D, (TT*)out));
}

}  // namespace tts
