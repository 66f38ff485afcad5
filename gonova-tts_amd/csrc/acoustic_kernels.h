// Launchers of the acoustic-model row-wise kernels (acoustic_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tts {

hipError_t launch_embed(int dt, const int* ids, const int* lens, int B, int N, int Tm, const void* E, int V, int D,
                        float scale, void* out, hipStream_t s);
hipError_t launch_layernorm(int dt, const void* in, void* out, int rows, int C, const float* g1, const float* b1,
                            const float* g2, const float* b2, float eps, hipStream_t s, const int* lens = nullptr, int stride = 0);
// groups LayerNorms (C <= 256 channels each, side by side in rows of ld elements) in place, one launch
struct LnGroups {
  static constexpr int MAXG = 4;
  const float* g[MAXG];
  const float* b[MAXG];
};
hipError_t launch_layernorm_groups(int dt, void* x, int rows, int C, int ld, const LnGroups& gp, int groups, float eps,
                                   hipStream_t s, const int* lens = nullptr, int stride = 0);
hipError_t launch_pos_bias(int dt, const void* qkv, int rows, int D, const float* u, const float* v, void* qu,
                           void* qv, hipStream_t s);
hipError_t launch_transpose_v(int dt, const void* qkv, const int* lens, int B, int Tm, int D, int H, int Sk, void* vt,
                              hipStream_t s);
hipError_t launch_rel_softmax(int dt, const void* ac, const void* bd, const int* lens, int B, int H, int Tm, int Sac,
                              int Sbd, int Sk, float scale, void* p, hipStream_t s);
hipError_t launch_glu_dwconv(int dt, const void* a, const int* lens, int B, int Tm, int D, const float* w, int k,
                             const float* bias, void* out, hipStream_t s);
hipError_t launch_ln_linear1(int dt, const void* in, int rows, int C, const float* g, const float* b, float eps,
                             const float* w, float wb, float* out, hipStream_t s);
hipError_t launch_durations(const float* logd, const int* lens, int B, int N, const int* override_d, float speed,
                            int Tcap, int* dur, int* mel_lens, int* tokmap, hipStream_t s);
hipError_t launch_var_embed_add(int dt, void* x, int rows, int D, const float* e, const float* we, const float* be,
                                const float* p, const float* wp, const float* bp, hipStream_t s);
// enc in dt_in (dt or fp32), out in dt: frames <= Tcap rows per utterance (tokmap row stride Tcap)
// written at row stride Tout
hipError_t launch_regulate(int dt_in, int dt, const void* enc, int B, int N, int D, const int* tokmap, int Tcap,
                           int frames, int Tout, float scale, void* out, hipStream_t s);
// in: row stride Tin; out: float32 [B][Tcap][C]
hipError_t launch_mel_out(int dt, const void* in, const int* mel_lens, int B, int Tin, int Tcap, int C, float* out,
                          hipStream_t s);

hipError_t launch_spk_bias(int dt, const float* e, int B, int E, const float* We, const float* bias, int D, void* out,
                           hipStream_t s);

hipError_t launch_range_take(int* src, int* dst, hipStream_t s);
// attention.hip: fused relative-position attention (dk = 192): 16-bit dtypes, fp32 (exact f32
// MFMA) and, with split set, fp32 in split precision (three f16 MFMAs per product)
bool rel_attn_supported(int dt, int D, int H);
// ws: the fp32 form's key-chunk partials (rel_attn_f32_ws_bytes; null or too small: one chunk)
hipError_t launch_rel_attn(int dt, bool split, const float* pos_u, const float* pos_v, const void* qkv,
                           const void* ptab, const int* lens, int B, int Tm, int Tp, int D, int H, int rmax,
                           float scale, void* out, hipStream_t s, int* range_flag = nullptr, float* ws = nullptr,
                           long long ws_bytes = 0);
int rel_attn_f32_kc();  // keys per chunk of the fp32 form (0: no chunks)
long long rel_attn_f32_ws_bytes(int B, int Tm, int Tp, int D, int H);
long long rel_attn_split_ws_bytes(int B, int Tm, int Tp, int D, int H);  // split form's key-chunk partials (0: none)

}  // namespace tts
