// Rational-rate polyphase resampler for the waveform output:
// 22,050 Hz -> 24,000 Hz (up 160, down 147) for clients that assume the reference's
// hard-coded 24 kHz (synthesizer.py:119, queue_manager.py:40), or any up/down.
//
// Restates scipy.signal.resample_poly(x, up, down) with its default window ('kaiser', 5.0)
// and constant (zero) padding, per utterance:
//   h       = firwin(2*half_len + 1, 1/max(up,down), window=kaiser(5.0)) * up,
//             half_len = 10 * max(up, down)
//   h'      = [zeros(n_pre_pad), h],  n_pre_pad = down - half_len % down
//   y[m]    = sum_k h'[k] * xu[(m + n_pre_remove) * down - k],   n_pre_remove = (half_len + n_pre_pad) / down
//             (xu = x upsampled by zero insertion), m < n_out = ceil(n_in * up / down)
// Polyphase: with t = (m + n_pre_remove) * down only taps k = t mod up + up*q meet a nonzero
// xu, so y[m] = sum_q hp[t mod up][q] * x[t / up - q] -- NQ = ceil(len(h') / up) MACs per
// output (21 at 160/147).  One thread per output sample; coefficients [up][NQ] fp32 are
// read through L1/L2 (13 KB at 160/147), the input window is shared by neighbouring lanes.
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "common.h"

namespace tts {

// modified Bessel function of the first kind, order 0 (power series; converges for the
// Kaiser arguments used here, beta <= 20)
static double bessel_i0(double x) {
  double sum = 1.0, term = 1.0;
  const double q = x * x / 4.0;
  for (int k = 1; k < 200; ++k) {
    term *= q / ((double)k * (double)k);
    sum += term;
    if (term < sum * 1e-17) break;
  }
  return sum;
}

// scipy.signal.resample_poly's default filter (firwin with a symmetric Kaiser(5.0) window,
// DC gain normalised to 1, then scaled by up) after the pre-padding it applies.
// Returns the padded length; h_out (if cap suffices) receives the taps.
int resample_design(int up, int down, std::vector<double>& h, int& n_pre_remove) {
  const int max_rate = up > down ? up : down;
  const double fc = 1.0 / max_rate;
  const int half_len = 10 * max_rate;
  const int n = 2 * half_len + 1;
  const double alpha = 0.5 * (n - 1);
  const double beta = 5.0;
  std::vector<double> f(n);
  double s = 0.0;
  for (int i = 0; i < n; ++i) {
    const double m = i - alpha;
    const double xx = fc * m;
    const double sinc = xx == 0.0 ? 1.0 : std::sin(M_PI * xx) / (M_PI * xx);
    const double r = 2.0 * i / (n - 1) - 1.0;
    const double w = bessel_i0(beta * std::sqrt(std::max(0.0, 1.0 - r * r))) / bessel_i0(beta);
    f[i] = fc * sinc * w;
    s += f[i];
  }
  const int n_pre_pad = down - half_len % down;
  n_pre_remove = (half_len + n_pre_pad) / down;
  h.assign(n_pre_pad + n, 0.0);
  for (int i = 0; i < n; ++i) h[n_pre_pad + i] = f[i] / s * up;
  return (int)h.size();
}

__global__ __launch_bounds__(256) void resample_poly_kernel(const float* __restrict__ x, long long sxb,
                                                            const int* __restrict__ in_lens, int up, int down,
                                                            int nq, int n_pre_remove, const float* __restrict__ hp,
                                                            float* __restrict__ y, long long syb, int y_cap,
                                                            int* __restrict__ out_lens) {
  const int b = blockIdx.y;
  const int n_in = in_lens[b];
  const long long n_out = ((long long)n_in * up + down - 1) / down;
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m == 0 && out_lens) out_lens[b] = (int)min(n_out, (long long)y_cap);
  if (m >= y_cap) return;
  float* yb = y + (long long)b * syb;
  if (m >= n_out) {  // zero tail, like the vocoder's output past each utterance
    yb[m] = 0.f;
    return;
  }
  const long long t = ((long long)m + n_pre_remove) * down;
  const int ph = (int)(t % up);
  const long long base = t / up;
  const float* hr = hp + (long long)ph * nq;
  const float* xb = x + (long long)b * sxb;
  float acc = 0.f;
  for (int q = 0; q < nq; ++q) {
    const long long i = base - q;
    if (i >= 0 && i < n_in) acc = fmaf(hr[q], xb[i], acc);
  }
  yb[m] = acc;
}

hipError_t launch_resample_poly(const float* x, long long sxb, const int* in_lens, int B, int up, int down, int nq,
                                int n_pre_remove, const float* hp, float* y, long long syb, int y_cap,
                                int* out_lens, hipStream_t s) {
  if (B <= 0 || y_cap <= 0) return hipSuccess;
  dim3 grid((y_cap + 255) / 256, B);
  hipLaunchKernelGGL(resample_poly_kernel, grid, dim3(256), 0, s, x, sxb, in_lens, up, down, nq, n_pre_remove, hp,
                     y, syb, y_cap, out_lens);
  return hipGetLastError();
}

}  // namespace tts
