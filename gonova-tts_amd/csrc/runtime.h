// Host-side runtime helpers shared by the vocoder and acoustic runtimes:
// error type, weight packing/upload, and the implicit-GEMM launch wrapper with
// optional live hipEvent profiling.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tts_hip.h"
#include "common.h"
#include "kernels.h"

namespace tts {

struct TtsError : std::runtime_error {
  int code;
  TtsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// On failure the error is also consumed from HIP's per-thread last-error slot, so a caught
// failure (e.g. an out-of-memory reservation) is not reported again by the next launch check
// of another library (PyTorch) on this thread.
#define HIP_CHECK(expr)                                                                       \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      (void)hipGetLastError();                                                                \
      throw ::tts::TtsError(TTS_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    }                                                                                         \
  } while (0)

inline size_t dtype_size(int dt) { return dt == DT_F32 ? 4 : 2; }

// Device memory the library holds (weights, workspaces), per HIP device: every device buffer is
// allocated through dev_malloc and released through dev_free, which keep a registry of live
// buffers (tts_device_bytes, the service's /health "gpu" report; the reference reads only
// torch's allocator there, server.py:456-465, which never sees these buffers).
struct DevRegistry {
  std::mutex mu;
  std::map<uintptr_t, std::pair<int, size_t>> live;  // buffer -> (device, bytes), address-ordered
  std::unordered_map<int, long long> bytes;          // device -> live bytes
};
inline DevRegistry& dev_registry() {
  static DevRegistry r;
  return r;
}
template <typename T>
inline hipError_t dev_malloc(T** p, size_t n) {
  void* q = nullptr;
  const hipError_t e = hipMalloc(&q, n);
  if (e != hipSuccess) return e;
  int dev = 0;
  (void)hipGetDevice(&dev);
  DevRegistry& r = dev_registry();
  std::lock_guard<std::mutex> g(r.mu);
  r.live[reinterpret_cast<uintptr_t>(q)] = {dev, n};
  r.bytes[dev] += (long long)n;
  *p = static_cast<T*>(q);
  return e;
}
inline hipError_t dev_free(void* p) {
  if (!p) return hipSuccess;
  {
    DevRegistry& r = dev_registry();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.live.find(reinterpret_cast<uintptr_t>(p));
    if (it != r.live.end()) {
      r.bytes[it->second.first] -= (long long)it->second.second;
      r.live.erase(it);
    }
  }
  return hipFree(p);
}
// Diagnostic builds (-DTTS_BOUNDS_CHECK=1): whether [p, p + n) lies inside one live library buffer
// (pointers the library did not allocate -- the caller's torch tensors -- are not judged: true)
inline bool dev_range_ok(const void* p, long long n, std::string* why) {
  if (!p || n <= 0) return true;
  DevRegistry& r = dev_registry();
  std::lock_guard<std::mutex> g(r.mu);
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = r.live.upper_bound(a);
  if (it == r.live.begin()) return true;
  --it;
  if (a >= it->first + it->second.second) return true;  // not a library buffer
  if (a + (uintptr_t)n <= it->first + it->second.second) return true;
  if (why)
    *why = "needs " + std::to_string(n) + " bytes at offset " + std::to_string(a - it->first) + " of a " +
           std::to_string(it->second.second) + "-byte buffer";
  return false;
}
inline long long dev_bytes(int dev) {
  DevRegistry& r = dev_registry();
  std::lock_guard<std::mutex> g(r.mu);
  auto it = r.bytes.find(dev);
  return it == r.bytes.end() ? 0 : it->second;
}

inline uint16_t f32_to_bf16_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// host fp32 -> new device buffer in dtype dt
inline void* upload(const std::vector<float>& h, int dt) {
  void* d = nullptr;
  const size_t n = h.size();
  HIP_CHECK(dev_malloc(&d, std::max<size_t>(n, 1) * dtype_size(dt)));
  if (n == 0) return d;
  if (dt == DT_F32) {
    HIP_CHECK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  } else if (dt == DT_F16) {
    std::vector<_Float16> t(n);
    for (size_t i = 0; i < n; ++i) t[i] = (_Float16)h[i];
    HIP_CHECK(hipMemcpy(d, t.data(), n * 2, hipMemcpyHostToDevice));
  } else {
    std::vector<uint16_t> t(n);
    for (size_t i = 0; i < n; ++i) t[i] = f32_to_bf16_bits(h[i]);
    HIP_CHECK(hipMemcpy(d, t.data(), n * 2, hipMemcpyHostToDevice));
  }
  return d;
}

inline float* upload_f32(const std::vector<float>& h) { return (float*)upload(h, DT_F32); }

// A packed implicit-GEMM conv layer: W[M][taps][Cin] in the compute dtype, bias fp32 [M].
struct ConvLayer {
  void* w = nullptr;
  void* wpk = nullptr;    // fragment-packed copy (frag_pack), or null
  void* wpk16 = nullptr;  // 16x16 fragment-packed copy (frag_pack16, MRF convs at C <= 64), or null
  void* wup16 = nullptr;  // transposed conv: [M/16][K/32][64][8] copy (frag_pack_up16), or null
  float* bias = nullptr;
  float wpk_unscale = 1.f;  // split-packed wpk: the power of two its sums are multiplied by
  int M = 0, Cin = 0, taps = 1, dil = 1, pad = 0;
  int up_s = 0, up_cout = 0, up_p = 0;  // transposed-conv output mapping
};

// Fragment-packed weights for conv_xres_kernel: W[M][taps][Cin] (host fp32) ->
//   P[M/32][taps][Cin/16][lane 0..63][8],  lane l holding row 32*mb + (l & 31),
//   channels 16*ks + 8*(l >> 5) + [0, 8)   (the A operand of v_mfma_f32_32x32x16_*),
// so one wave's fragment for (32-row block, tap, k-step) is 1 KiB contiguous.  Rows past
// M are zero.  Only for 16-bit dtypes with Cin % 64 == 0 and M >= 64 (else null).
inline void* frag_pack(const std::vector<float>& w, int M, int taps, int ci, int dt, std::vector<void*>& allocs) {
  if (dt == DT_F32 || ci % 64 || M < 64) return nullptr;
  const int MB = (M + 31) / 32, KS = ci / 16;
  std::vector<float> p((size_t)MB * 32 * taps * ci, 0.f);
  size_t o = 0;
  for (int mb = 0; mb < MB; ++mb)
    for (int t = 0; t < taps; ++t)
      for (int ks = 0; ks < KS; ++ks)
        for (int l = 0; l < 64; ++l) {
          const int m = mb * 32 + (l & 31);
          for (int j = 0; j < 8; ++j, ++o)
            if (m < M) p[o] = w[((size_t)m * taps + t) * ci + ks * 16 + 8 * (l >> 5) + j];
        }
  void* d = upload(p, dt);
  allocs.push_back(d);
  return d;
}

// Split-precision packing for conv_split_kernel (fp32 layers run as three f16 MFMAs):
// frag_pack's fragment order, two f16 planes of the layer scaled by 2^s -- hi = f16(w 2^s), then
// lo = f16(w 2^s - hi) -- with 2^s the power of two that puts max|w| in [2^14, 2^15): hi stays
// finite and lo (~2^-11 of hi) in f16's normal range for every weight above ~2^-19 max|w|.  The
// three products hi*hi + hi*lo + lo*hi then share one fp32 accumulator (no scale between the
// terms) and the GEMM multiplies its sums by *unscale = 2^-s, an exact step.
inline void* frag_pack_split(const std::vector<float>& w, int M, int taps, int ci, std::vector<void*>& allocs,
                             float* unscale) {
  if (ci % 32 || M % 4) return nullptr;
  const int MB = (M + 31) / 32, KS = ci / 16;
  const size_t plane = (size_t)MB * 32 * taps * ci;
  float mx = 0.f;
  for (float v : w) mx = std::max(mx, std::fabs(v));
  int e = 0;
  if (mx > 0.f) (void)std::frexp(mx, &e);  // mx = f * 2^e, f in [0.5, 1)
  const int s = std::max(-24, std::min(60, 15 - e));
  const float sc = std::ldexp(1.f, s);
  *unscale = std::ldexp(1.f, -s);
  std::vector<float> p(2 * plane, 0.f);
  size_t o = 0;
  for (int mb = 0; mb < MB; ++mb)
    for (int t = 0; t < taps; ++t)
      for (int ks = 0; ks < KS; ++ks)
        for (int l = 0; l < 64; ++l) {
          const int m = mb * 32 + (l & 31);
          for (int j = 0; j < 8; ++j, ++o) {
            if (m >= M) continue;
            const float v = w[((size_t)m * taps + t) * ci + ks * 16 + 8 * (l >> 5) + j] * sc;  // exact
            const float hi = (float)(_Float16)v;
            p[o] = hi;
            p[plane + o] = v - hi;
          }
        }
  void* d = upload(p, DT_F16);
  allocs.push_back(d);
  return d;
}

// 16x16 fragment packing for mrf_pair_kernel: nn.Conv1d weight [C][C][k] (host fp32) ->
//   P[C/16][k][C/32][lane 0..63][8],  lane l holding output channel 16*mb + (l & 15),
//   input channels 32*ks + 8*(l >> 4) + [0, 8)  (the A operand of v_mfma_f32_16x16x32_*).
inline void* frag_pack16(const std::vector<float>& w, int C, int k, int dt, std::vector<void*>& allocs) {
  if (dt == DT_F32 || C % 32) return nullptr;
  std::vector<float> p((size_t)C * C * k);
  size_t o = 0;
  for (int mb = 0; mb < C / 16; ++mb)
    for (int t = 0; t < k; ++t)
      for (int ks = 0; ks < C / 32; ++ks)
        for (int l = 0; l < 64; ++l) {
          const int m = mb * 16 + (l & 15);
          for (int j = 0; j < 8; ++j, ++o) p[o] = w[((size_t)m * C + ks * 32 + 8 * (l >> 4) + j) * k + t];
        }
  void* d = upload(p, dt);
  allocs.push_back(d);
  return d;
}

// Packing for upsample_stream_kernel: W'[M][K] (host fp32, K = tap*Cin + ci) ->
//   P[M/16][K/32][lane 0..63][8],  lane l holding row 16*mt + (l & 15), k 32*ks + 8*(l >> 4) + [0, 8)
// (the A operand of v_mfma_f32_16x16x32_*; one 1 KiB LDS fragment per (mt, ks)).
inline void* frag_pack_up16(const std::vector<float>& w, int M, int K, int dt, std::vector<void*>& allocs) {
  if (dt == DT_F32 || M % 16 || K % 32) return nullptr;
  std::vector<float> p((size_t)M * K);
  size_t o = 0;
  for (int mt = 0; mt < M / 16; ++mt)
    for (int ks = 0; ks < K / 32; ++ks)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j, ++o) p[o] = w[(size_t)(mt * 16 + (l & 15)) * K + ks * 32 + 8 * (l >> 4) + j];
  void* d = upload(p, dt);
  allocs.push_back(d);
  return d;
}

// nn.Conv1d weight [Cout][Cin][k] (host fp32) -> ConvLayer; scale[o] (optional) folds a
// per-output-channel factor (BatchNorm) into the weights.
// split: an fp32 layer also gets a split-packed copy (runs as three f16 MFMAs, conv_split.hip).
inline ConvLayer make_conv(const std::vector<float>& w, int co, int ci, int k, const std::vector<float>& bias,
                           int dil, int pad, int dt, std::vector<void*>& allocs,
                           const std::vector<float>* scale = nullptr, bool split = false) {
  if (w.size() != (size_t)co * ci * k) throw TtsError(TTS_ERR_INVALID, "conv weight size mismatch");
  std::vector<float> p((size_t)co * k * ci);
  for (int o = 0; o < co; ++o) {
    const float s = scale ? (*scale)[o] : 1.f;
    for (int c = 0; c < ci; ++c)
      for (int j = 0; j < k; ++j) p[((size_t)o * k + j) * ci + c] = w[((size_t)o * ci + c) * k + j] * s;
  }
  if (dt == DT_F32 && split)  // split packing scales the layer by a power of two (frag_pack_split): any finite weights
    for (float v : p)
      if (!std::isfinite(v)) throw TtsError(TTS_ERR_INVALID, "non-finite weight in a split-precision layer");
  ConvLayer L;
  L.w = upload(p, dt);
  allocs.push_back(L.w);
  L.wpk = (dt == DT_F32 && split) ? frag_pack_split(p, co, k, ci, allocs, &L.wpk_unscale)
                                  : frag_pack(p, co, k, ci, dt, allocs);
  std::vector<float> b = bias;
  if (b.empty()) b.assign(co, 0.f);
  if (b.size() != (size_t)co) throw TtsError(TTS_ERR_INVALID, "conv bias size mismatch");
  L.bias = upload_f32(b);
  allocs.push_back(L.bias);
  L.M = co; L.Cin = ci; L.taps = k; L.dil = dil; L.pad = pad;
  return L;
}

// Live kernel timing (bench.py roofline): hipEvents around every implicit-GEMM launch.
struct Profiler {
  bool on = false;
  struct Rec { hipEvent_t a, b; double flops; int kind; int nk = 1; };  // nk: kernels between a and b
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    return e;
  }
  // sums per ProfKind (arrays of nk entries; kinds >= nk are dropped), then resets
  void read_kinds(int nk, double* ms, double* fl, int* n) {
    for (int k = 0; k < nk; ++k) { ms[k] = 0; fl[k] = 0; n[k] = 0; }
    for (auto& r : recs) {
      HIP_CHECK(hipEventSynchronize(r.b));
      float e = 0.f;
      HIP_CHECK(hipEventElapsedTime(&e, r.a, r.b));
      if (r.kind < nk) { ms[r.kind] += e; fl[r.kind] += r.flops; n[r.kind] += r.nk; }
      pool.push_back(r.a); pool.push_back(r.b);
    }
    recs.clear();
  }
  void read(double* ms, double* fl, int* n) {
    double m[PK_N], f[PK_N];
    int c[PK_N];
    read_kinds(PK_N, m, f, c);
    double tm = 0, tf = 0;
    int tc = 0;
    for (int k = 0; k < PK_N; ++k) { tm += m[k]; tf += f[k]; tc += c[k]; }
    if (ms) *ms = tm;
    if (fl) *fl = tf;
    if (n) *n = tc;
  }
  // one launch (a callable returning hipError_t) bracketed by events when profiling is on
  template <typename F>
  void launch(int kind, double flops, hipStream_t s, F&& f) {
    if (!on) {
      HIP_CHECK(f());
      return;
    }
    Rec r{get(), get(), flops, kind};
    HIP_CHECK(hipEventRecord(r.a, s));
    HIP_CHECK(f());
    HIP_CHECK(hipEventRecord(r.b, s));
    recs.push_back(r);
  }
  ~Profiler() {
    for (auto& r : recs) { hipEventDestroy(r.a); hipEventDestroy(r.b); }
    for (auto e : pool) hipEventDestroy(e);
  }
};

#ifndef TTS_BOUNDS_CHECK
#define TTS_BOUNDS_CHECK 0  // diagnostic builds: every conv launch's operand extents against the buffers
#endif
// the byte extents a conv launch can touch, checked against the library's buffers (diagnostic)
inline void conv_bounds_check(const ConvParams& p, int dt) {
  const long long e = dt == DT_F32 ? 4 : 2;
  const long long F = (long long)p.B * p.x_rows;
  auto need = [&](const char* what, const void* q, long long bytes) {
    std::string why;
    if (!dev_range_ok(q, bytes, &why))
      throw TtsError(TTS_ERR_INVALID, std::string("bounds: ") + what + " " + why + " (M " + std::to_string(p.M) +
                                          ", Cin " + std::to_string(p.Cin) + ", taps " + std::to_string(p.taps) +
                                          ", B " + std::to_string(p.B) + ", rows " + std::to_string(p.x_rows) + "/" +
                                          std::to_string(p.y_rows) + ", rows_pad " + std::to_string(p.rows_pad) + ")");
  };
  if (p.nh == 1 && !p.up_s) {
    need("x", p.x, ((long long)(p.B - 1) * p.sxb + (long long)(p.x_rows - 1) * p.sxr + p.Cin) * e);
    need("y", p.y, ((long long)(p.B - 1) * p.syb + (long long)(p.y_rows - 1) * p.syr + p.M) * e);
    if (p.r1) need("r1", p.r1, ((long long)(p.B - 1) * p.srb + (long long)(p.y_rows - 1) * p.srr + p.M) * e);
    if (p.r2) need("r2", p.r2, ((long long)(p.B - 1) * p.srb + (long long)(p.y_rows - 1) * p.srr + p.M) * e);
    if (p.ln_out) need("ln_out", p.ln_out, ((long long)(p.B - 1) * p.syb + (long long)(p.y_rows - 1) * p.syr + p.M) * e);
  }
  need("bias", p.bias, (long long)p.M * 4);
  if (p.ws) need("ws", p.ws, p.ws_bytes);
  if (p.x_len) need("x_len", p.x_len, (long long)p.B * 4);
  if (p.y_len) need("y_len", p.y_len, (long long)p.B * 4);
  if (p.ln_cnt) need("ln_cnt", p.ln_cnt, (long long)p.ln_cnt_n * 4);
  (void)F;
}

// Launch one implicit-GEMM conv (validates, optionally profiles).
inline void launch_conv_checked(const ConvParams& p, int dt, hipStream_t s, Profiler* prof, double flops) {
  const char* why = nullptr;
  if (conv_gemm_check(p, dt, &why)) throw TtsError(TTS_ERR_INVALID, std::string("conv: ") + why);
  if (TTS_BOUNDS_CHECK) conv_bounds_check(p, dt);
  if (prof && prof->on) {
    Profiler::Rec r{prof->get(), prof->get(), flops, conv_gemm_kind(dt, p)};
    HIP_CHECK(hipEventRecord(r.a, s));
    HIP_CHECK(conv_gemm_launch(dt, p, s));
    HIP_CHECK(hipEventRecord(r.b, s));
    r.nk = conv_last_kernels();
    prof->recs.push_back(r);
  } else {
    HIP_CHECK(conv_gemm_launch(dt, p, s));
  }
}

// Standard conv over activations [B][rows][C]: X [B][x_rows][Cin] -> Y [B][y_rows][M] (+ residual R like Y).
inline void run_layer(const ConvLayer& L, const void* x, int x_rows, const int* lens, void* y, int y_rows, int B,
                      int dt, hipStream_t s, Profiler* prof, float in_slope = 1.f, int act = ACT_NONE,
                      float alpha = 1.f, const void* r1 = nullptr, const void* r2 = nullptr, float out_scale = 1.f,
                      int x_ld = 0, int y_ld = 0, int rows_pad = 0, float* ws = nullptr, long long ws_bytes = 0,
                      const ConvParams* ln = nullptr) {  // ln: LayerNorm fields, range_flag, no_split
  ConvParams p = conv_params_default();
  const int xl = x_ld ? x_ld : L.Cin, yl = y_ld ? y_ld : L.M;
  p.x = x; p.sxb = (long long)x_rows * xl; p.sxr = xl; p.x_len = lens; p.x_rows = x_rows;
  p.w = L.w; p.w_ld = L.taps * L.Cin; p.bias = L.bias; p.wpk = L.wpk; p.w_unscale = L.wpk_unscale;
  p.y = y; p.syb = (long long)y_rows * yl; p.syr = yl;
  p.r1 = r1; p.r2 = r2; p.srb = p.syb; p.srr = yl;
  p.y_len = lens; p.y_rows = y_rows;
  p.M = L.M; p.Cin = L.Cin; p.taps = L.taps; p.dil = L.dil; p.pad = L.pad;
  p.in_slope = in_slope; p.act_out = act; p.alpha = alpha; p.out_scale = out_scale;
  p.B = B;
  p.rows_pad = rows_pad; p.ws = ws; p.ws_bytes = ws_bytes;
  if (ln) {  // the LayerNorm fields of *ln (ln_out, gains, biases, eps)
    p.ln_out = ln->ln_out; p.ln_g1 = ln->ln_g1; p.ln_b1 = ln->ln_b1; p.ln_g2 = ln->ln_g2; p.ln_b2 = ln->ln_b2;
    p.ln_eps = ln->ln_eps;
    p.ln_cnt = ln->ln_cnt; p.ln_cnt_n = ln->ln_cnt_n;
    p.ln_lin_w = ln->ln_lin_w; p.ln_lin_b = ln->ln_lin_b; p.ln_lin_out = ln->ln_lin_out;
    p.range_flag = ln->range_flag; p.no_split = ln->no_split;  // (the split path's guard / fallback)
    p.f32_splitk = ln->f32_splitk;
  }
  launch_conv_checked(p, dt, s, prof, 2.0 * L.M * (double)L.Cin * L.taps * (double)B * y_rows);
}

}  // namespace tts
