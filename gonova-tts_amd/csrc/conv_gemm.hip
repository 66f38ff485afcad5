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
#include "kernels.h"

#include <cstdlib>

namespace tts {

constexpr int HALO_MAX = 64;  // max (taps-1)*dil supported (HiFi-GAN V1: 50)

template <typename T>
__device__ inline uint4 act16(uint4 u, bool valid, float slope) {
  if (!valid) return uint4{0u, 0u, 0u, 0u};
  if (slope != 1.0f) {
    constexpr int N = 16 / sizeof(T);
    T* e = reinterpret_cast<T*>(&u);
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = from_f32<T>(leaky(to_f32(e[i]), slope));
  }
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
__global__ __launch_bounds__(64 * WM * WN) void conv_gemm_kernel(ConvParams p) {
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
  const int b = blockIdx.z / nh;
  const int hd = blockIdx.z - b * nh;
  const int n0 = blockIdx.x * BN;
  const int ylen = p.y_len ? min(p.y_len[b], p.y_rows) : p.y_rows;
  if (n0 >= ylen) return;
  const int xlen = p.x_len ? min(p.x_len[b], p.x_rows) : p.x_rows;
  const int m_blk = blockIdx.y * BM;

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
  load_chunk(0);
  load_a(a_cur, 0, 0);
  store_chunk(xs0, 0);
  __syncthreads();

  for (int ci = 0; ci < nchunks; ++ci) {
    const T* cur = (ci & 1) ? xs1 : xs0;
    T* nxt = (ci & 1) ? xs0 : xs1;
    const int c0 = ci * CK;
    const bool has_next = ci + 1 < nchunks;
    if (has_next) load_chunk(c0 + CK);
    for (int tap = 0; tap < p.taps; ++tap) {
      int ntap = tap + 1, nc0 = c0;
      if (ntap == p.taps) { ntap = 0; nc0 = c0 + CK; }
      if (nc0 < p.Cin) load_a(a_nxt, nc0, ntap);
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

  // ---------------- epilogue ----------------
  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.syb + (long long)hd * p.syh;
  const T* R1 = p.r1 ? reinterpret_cast<const T*>(p.r1) + (long long)b * p.srb + (long long)hd * p.srh : nullptr;
  const T* R2 = p.r2 ? reinterpret_cast<const T*>(p.r2) + (long long)b * p.srb + (long long)hd * p.srh : nullptr;
  const int tlen = p.up_len ? min(p.up_len[b], (p.y_rows - 1) * p.up_s) : 0;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + n_w0 + nt * 32 + l31;
      if (n >= ylen) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = m_w0 + mt * 32 + 8 * g + 4 * hh;
        if (m >= p.M) continue;
        int row = n, col = m;
        if (p.up_s) {
          const int q = m / p.up_cout;
          row = n * p.up_s + q - p.up_p;
          col = m - q * p.up_cout;
          if (row < 0 || row >= tlen) continue;
        }
        f32x4 v = {acc[mt][nt][4 * g + 0], acc[mt][nt][4 * g + 1], acc[mt][nt][4 * g + 2],
                   acc[mt][nt][4 * g + 3]};
        if (p.bias) {
          const f32x4 bb = *reinterpret_cast<const f32x4*>(p.bias + m);
          v += bb;
        }
        if (p.alpha != 1.0f) v *= p.alpha;
        if (p.act_out) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = apply_act(v[i], p.act_out, p.out_slope);
        }
        if (R1) v += Vec4<T>::load(R1 + (long long)row * p.srr + col);
        if (R2) v += Vec4<T>::load(R2 + (long long)row * p.srr + col);
        if (p.out_scale != 1.0f) v *= p.out_scale;
        Vec4<T>::store(Y + (long long)row * p.syr + col, v);
      }
    }
  }
}

template <typename T, int MT, int NT, int WM, int WN, int CK>
static hipError_t launch_cfg(const ConvParams& p, hipStream_t s) {
  constexpr int BM = 32 * MT * WM;
  constexpr int BN = 32 * NT * WN;
  constexpr int LDSR = CK + 16 / (int)sizeof(T);
  const int R = BN + (p.taps - 1) * p.dil;
  const int nchunks = (p.Cin + CK - 1) / CK;
  const size_t lds = (size_t)R * LDSR * sizeof(T) * (nchunks > 1 ? 2 : 1);
  dim3 grid((p.y_rows + BN - 1) / BN, (p.M + BM - 1) / BM, p.B * p.nh);
  hipLaunchKernelGGL((conv_gemm_kernel<T, MT, NT, WM, WN, CK>), grid, dim3(64 * WM * WN), lds, s, p);
  return hipGetLastError();
}

static int wide_mode() {
  static int m = [] {
    const char* e = getenv("TTS_CONV_WIDE");
    return e ? atoi(e) : 0;
  }();
  return m;
}

template <typename T>
static hipError_t launch_t(const ConvParams& p, hipStream_t s) {
  constexpr int CKW = 64 / (int)sizeof(T);   // 32 x 16-bit / 16 x f32 (64-byte rows)
  constexpr int CKWW = 128 / (int)sizeof(T); // 64 x 16-bit / 32 x f32 (128-byte rows)
  const bool wide = wide_mode() && p.Cin % CKWW == 0 && p.Cin >= 2 * CKWW;
  if (p.M <= 32) {
    if (wide) return launch_cfg<T, 1, 2, 1, 4, CKWW>(p, s);
    return launch_cfg<T, 1, 2, 1, 4, CKW>(p, s);
  }
  if (p.M <= 64) {
    if (wide) return launch_cfg<T, 1, 2, 2, 2, CKWW>(p, s);
    return launch_cfg<T, 1, 2, 2, 2, CKW>(p, s);
  }
  if (wide) return launch_cfg<T, 1, 4, 4, 1, CKWW>(p, s);
  return launch_cfg<T, 1, 4, 4, 1, CKW>(p, s);
}

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
  return 0;
}

hipError_t conv_gemm_launch(int dtype, const ConvParams& p, hipStream_t s) {
  switch (dtype) {
    case DT_F32: return launch_t<float>(p, s);
    case DT_F16: return launch_t<half_t>(p, s);
    case DT_BF16: return launch_t<bf16_t>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace tts
