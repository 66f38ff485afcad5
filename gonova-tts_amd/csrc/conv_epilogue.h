// Per-fragment epilogue of the implicit-GEMM conv kernels (conv_gemm.hip, conv_split.hip).
#pragma once
#include "common.h"
#include "kernels.h"

namespace tts {

// Epilogue shared by conv_gemm_kernel and conv_split_kernel: lane (l31, hh) of a wave holds, for each 32x32 tile
// (mt, nt), rows n = n_base + nt*32 + l31 and channels m_base + mt*32 + 8g + 4hh + [0, 4).
//   y = ((alpha * (acc + bias)) -> act) + r1 + r2, times out_scale; transposed-conv row map.
template <typename T, int MT, int NT, int ACT>
__device__ __forceinline__ void conv_epilogue_act(const ConvParams& p, const f32x16 (&acc)[MT][NT], int b, int hd,
                                                  int n_base, int m_base, int ylen, int l31, int hh) {
  T* Y = reinterpret_cast<T*>(p.y) + (long long)b * p.syb + (long long)hd * p.syh;
  const T* R1 = p.r1 ? reinterpret_cast<const T*>(p.r1) + (long long)b * p.srb + (long long)hd * p.srh : nullptr;
  const T* R2 = p.r2 ? reinterpret_cast<const T*>(p.r2) + (long long)b * p.srb + (long long)hd * p.srh : nullptr;
  const int tlen = p.up_len ? min(p.up_len[b], (p.y_rows - 1) * p.up_s) : 0;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n_base + nt * 32 + l31;
      if (n >= ylen) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = m_base + mt * 32 + 8 * g + 4 * hh;
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
        if constexpr (ACT != ACT_NONE) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = apply_act(v[i], ACT, p.out_slope);
        }
        if (R1) v += Vec4<T>::load(R1 + (long long)row * p.srr + col);
        if (R2) v += Vec4<T>::load(R2 + (long long)row * p.srr + col);
        if (p.out_scale != 1.0f) v *= p.out_scale;
        Vec4<T>::store(Y + (long long)row * p.syr + col, v);
      }
    }
  }
}

// the activation kind dispatched once per tile, outside the element loops
template <typename T, int MT, int NT>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, const f32x16 (&acc)[MT][NT], int b, int hd,
                                              int n_base, int m_base, int ylen, int l31, int hh) {
  switch (p.act_out) {
    case ACT_RELU: conv_epilogue_act<T, MT, NT, ACT_RELU>(p, acc, b, hd, n_base, m_base, ylen, l31, hh); break;
    case ACT_TANH: conv_epilogue_act<T, MT, NT, ACT_TANH>(p, acc, b, hd, n_base, m_base, ylen, l31, hh); break;
    case ACT_LRELU: conv_epilogue_act<T, MT, NT, ACT_LRELU>(p, acc, b, hd, n_base, m_base, ylen, l31, hh); break;
    case ACT_SILU: conv_epilogue_act<T, MT, NT, ACT_SILU>(p, acc, b, hd, n_base, m_base, ylen, l31, hh); break;
    default: conv_epilogue_act<T, MT, NT, ACT_NONE>(p, acc, b, hd, n_base, m_base, ylen, l31, hh); break;
  }
}

}  // namespace tts
