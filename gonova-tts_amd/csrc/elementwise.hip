// Small bandwidth-bound kernels around the vocoder GEMMs.
#include "common.h"
#include "kernels.h"

namespace tts {

// mel f32 [B][T][C] (row stride smr) -> (x - mean) / scale in the compute dtype,
// [B][T][C] contiguous.  HF:1445-1446 (normalize_before).
template <typename T>
__global__ void mel_in_kernel(const float* __restrict__ mel, long long smb, int smr,
                              const float* __restrict__ mean, const float* __restrict__ scale,
                              T* __restrict__ out, int T_, int C) {
  const int b = blockIdx.y;
  const long long n = (long long)T_ * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int t = (int)(i / C);
    const int c = (int)(i - (long long)t * C);
    float v = mel[b * smb + (long long)t * smr + c];
    if (mean) v = (v - mean[c]) / scale[c];
    out[b * n + i] = from_f32<T>(v);
  }
}

hipError_t launch_mel_in(int dtype, const float* mel, long long smb, int smr, const float* mean,
                         const float* scale, void* out, int B, int T_, int C, hipStream_t s) {
  const long long n = (long long)T_ * C;
  dim3 grid((unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024), B);
  switch (dtype) {
    case DT_F32: hipLaunchKernelGGL(mel_in_kernel<float>, grid, dim3(256), 0, s, mel, smb, smr, mean, scale, (float*)out, T_, C); break;
    case DT_F16: hipLaunchKernelGGL(mel_in_kernel<half_t>, grid, dim3(256), 0, s, mel, smb, smr, mean, scale, (half_t*)out, T_, C); break;
    case DT_BF16: hipLaunchKernelGGL(mel_in_kernel<bf16_t>, grid, dim3(256), 0, s, mel, smb, smr, mean, scale, (bf16_t*)out, T_, C); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// out[k*B + b] = in[b] * mult[k] + add[k]  (per-utterance row counts of every stage)
__global__ void lens_kernel(const int* __restrict__ in, int* __restrict__ out, int B, int4 m0, int4 m1,
                            int4 a0, int4 a1, int n) {
  const int b = threadIdx.x + blockIdx.x * blockDim.x;
  if (b >= B) return;
  const int v = in[b];
  const int mult[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
  const int add[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  for (int k = 0; k < n; ++k) out[k * B + b] = v * mult[k] + add[k];
}

hipError_t launch_lens(const int* in, int* out, int B, const int* mult, const int* add, int n,
                       hipStream_t s) {
  if (n > 8) return hipErrorInvalidValue;
  int m[8] = {0}, a[8] = {0};
  for (int i = 0; i < n; ++i) { m[i] = mult[i]; a[i] = add[i]; }
  hipLaunchKernelGGL(lens_kernel, dim3((B + 255) / 256), dim3(256), 0, s, in, out, B,
                     make_int4(m[0], m[1], m[2], m[3]), make_int4(m[4], m[5], m[6], m[7]),
                     make_int4(a[0], a[1], a[2], a[3]), make_int4(a[4], a[5], a[6], a[7]), n);
  return hipGetLastError();
}

// conv_post: wav[b][t] = tanh(bias + sum_{j,c} w[j][c] * lrelu(x[b][t+j-pad][c], slope)),
// zero for t >= x_len[b].  HF:1464-1466.  Bandwidth-bound (reads C x 2 B per sample):
// a block stages (512 + k - 1) rows x C channels of lrelu(x) channel-major in LDS
// (fp32) and each thread produces samples t and t+256 (consecutive lanes read
// consecutive rows: conflict-free); the k x C weights are wave-uniform (scalar loads).
template <typename T, int C>
__global__ __launch_bounds__(256) void conv_post_kernel(const T* __restrict__ x, const int* __restrict__ x_len,
                                                       int T_, const float* __restrict__ w, float bias, int k,
                                                       float slope, float* __restrict__ wav, long long swb) {
  constexpr int TB = 512;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* xs = reinterpret_cast<float*>(smem);  // [C][rows]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * TB;
  const int len = x_len ? min(x_len[b], T_) : T_;
  const int pad = (k - 1) / 2;
  const int rows = TB + k - 1;
  constexpr int EPV = 16 / (int)sizeof(T);
  constexpr int VPR = C / EPV;
  const T* xb = x + (long long)b * T_ * C;
  for (int i = threadIdx.x; i < rows * VPR; i += 256) {
    const int r = i / VPR, cv = i - r * VPR;
    const int t = t0 - pad + r;
    const bool ok = t >= 0 && t < len;
    uint4 u = *reinterpret_cast<const uint4*>(xb + (long long)min(max(t, 0), T_ - 1) * C + cv * EPV);
    const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int q = 0; q < EPV; ++q) xs[(cv * EPV + q) * rows + r] = ok ? leaky(to_f32(e[q]), slope) : 0.f;
  }
  __syncthreads();
  float acc0 = bias, acc1 = bias;
  for (int j = 0; j < k; ++j) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float wv = w[j * C + c];
      const float* xr = xs + c * rows + threadIdx.x + j;
      acc0 = fmaf(wv, xr[0], acc0);
      acc1 = fmaf(wv, xr[256], acc1);
    }
  }
  const int ta = t0 + threadIdx.x, tb = ta + 256;
  if (ta < T_) wav[b * swb + ta] = ta < len ? tanhf(acc0) : 0.f;
  if (tb < T_) wav[b * swb + tb] = tb < len ? tanhf(acc1) : 0.f;
}

// 16-bit conv_post: the fp32 version above is LDS/VALU-bound (scalar converts into a
// channel-major fp32 tile, then 224 ds_read_b32 + 224 FMAs per sample: 1.5 TB/s).  Here
// the tile stays row-major in the compute dtype (lrelu applied packed), 16-byte chunk c of
// row r at c ^ ((r >> 2) & 3) -- 16 consecutive rows per ds_read_b128 lane group hit 16
// distinct slots -- and each sample is 4 x 7 row reads + 112 v_dot2_f32_{f16,bf16}
// against wave-uniform packed weights.  Thread tid produces samples t0+tid, t0+tid+256.
template <typename T>
__global__ __launch_bounds__(256) void conv_post16_kernel(const T* __restrict__ x, const int* __restrict__ x_len,
                                                          int T_, const unsigned* __restrict__ wpk, float bias,
                                                          int k, float slope, float* __restrict__ wav,
                                                          long long swb) {
  constexpr int C = 32, TB = 512, VPR = 4;  // 4 x 16-byte chunks per 64-byte row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * TB;
  const int len = x_len ? min(x_len[b], T_) : T_;
  const int pad = (k - 1) / 2;
  const int rows = TB + k - 1;
  const T* xb = x + (long long)b * T_ * C;
  auto slot = [](int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); };
  for (int i0 = threadIdx.x; i0 < rows * VPR; i0 += 256 * 4) {
    uint4 u[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = min(i0 + q * 256, rows * VPR - 1);
      const int t = t0 - pad + i / VPR;
      u[q] = *reinterpret_cast<const uint4*>(xb + (long long)min(max(t, 0), T_ - 1) * C + (i % VPR) * 8);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = i0 + q * 256;
      if (i < rows * VPR) {
        const int r = i / VPR, t = t0 - pad + r;
        *reinterpret_cast<uint4*>(smem + slot(r, i % VPR)) =
            (t >= 0 && t < len) ? lrelu_chunk<T>(u[q], slope) : uint4{0u, 0u, 0u, 0u};
      }
    }
  }
  __syncthreads();
  float acc0 = bias, acc1 = bias;
  for (int j = 0; j < k; ++j) {
    const unsigned* wj = wpk + j * (C / 2);
#pragma unroll
    for (int c = 0; c < VPR; ++c) {
      const uint4 a = *reinterpret_cast<const uint4*>(smem + slot(threadIdx.x + j, c));
      const uint4 d = *reinterpret_cast<const uint4*>(smem + slot(threadIdx.x + 256 + j, c));
      acc0 = Dot2<T>::dot(a.x, wj[4 * c + 0], acc0);
      acc0 = Dot2<T>::dot(a.y, wj[4 * c + 1], acc0);
      acc0 = Dot2<T>::dot(a.z, wj[4 * c + 2], acc0);
      acc0 = Dot2<T>::dot(a.w, wj[4 * c + 3], acc0);
      acc1 = Dot2<T>::dot(d.x, wj[4 * c + 0], acc1);
      acc1 = Dot2<T>::dot(d.y, wj[4 * c + 1], acc1);
      acc1 = Dot2<T>::dot(d.z, wj[4 * c + 2], acc1);
      acc1 = Dot2<T>::dot(d.w, wj[4 * c + 3], acc1);
    }
  }
  const int ta = t0 + threadIdx.x, tb = ta + 256;
  if (ta < T_) wav[b * swb + ta] = ta < len ? tanhf(acc0) : 0.f;
  if (tb < T_) wav[b * swb + tb] = tb < len ? tanhf(acc1) : 0.f;
}

hipError_t launch_conv_post(int dtype, const void* x, const int* x_len, int B, int T_, int C,
                            const float* w, const void* wpk, float bias, int k, float slope, float* wav,
                            long long swb, hipStream_t s) {
  if (C != 32) return hipErrorInvalidValue;
  if (dtype != DT_F32 && wpk) {
    dim3 grid((T_ + 511) / 512, B);
    const size_t lds = (size_t)(512 + k - 1) * 64;
    if (dtype == DT_F16)
      hipLaunchKernelGGL((conv_post16_kernel<half_t>), grid, dim3(256), lds, s, (const half_t*)x, x_len, T_,
                         (const unsigned*)wpk, bias, k, slope, wav, swb);
    else
      hipLaunchKernelGGL((conv_post16_kernel<bf16_t>), grid, dim3(256), lds, s, (const bf16_t*)x, x_len, T_,
                         (const unsigned*)wpk, bias, k, slope, wav, swb);
    return hipGetLastError();
  }
  dim3 grid((T_ + 511) / 512, B);
  const size_t lds = (size_t)C * (512 + k - 1) * 4;
  switch (dtype) {
    case DT_F32: hipLaunchKernelGGL((conv_post_kernel<float, 32>), grid, dim3(256), lds, s, (const float*)x, x_len, T_, w, bias, k, slope, wav, swb); break;
    case DT_F16: hipLaunchKernelGGL((conv_post_kernel<half_t, 32>), grid, dim3(256), lds, s, (const half_t*)x, x_len, T_, w, bias, k, slope, wav, swb); break;
    case DT_BF16: hipLaunchKernelGGL((conv_post_kernel<bf16_t, 32>), grid, dim3(256), lds, s, (const bf16_t*)x, x_len, T_, w, bias, k, slope, wav, swb); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace tts
