// libtts_hip.so — engine runtime and C-ABI (include/tts_hip.h).
//
// The engine owns device weights (packed for the implicit-GEMM kernels) and a
// workspace sized for [max_batch x max_frames]; forwards enqueue kernels on the
// caller's stream and never allocate once reserved.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/tts_hip.h"
#include "acoustic.h"
#include "switches.h"
#include "common.h"
#include "kernels.h"
#include "runtime.h"

using namespace tts;

static thread_local std::string g_last_error;

namespace {

struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
};

}  // namespace

struct VocoderWeights {
  bool loaded = false;
  float* mean = nullptr;
  float* scale = nullptr;
  bool normalize = false;
  ConvLayer conv_pre;
  std::vector<ConvLayer> ups;  // per stage
  std::vector<int> up_rate;
  std::vector<int> stage_ch;
  // mrf[stage][block][pair][0=conv1,1=conv2]
  std::vector<std::vector<std::vector<std::array<ConvLayer, 2>>>> mrf;
  float* post_w = nullptr;  // fp32 [k][C]
  void* post_wh = nullptr;  // [k][C] in the vocoder dtype (16-bit conv_post kernel), or null
  float post_b = 0.f;
  int post_k = 7, post_c = 32;
  int hop = 256;
};

// TTS_MRF_FUSED=0 selects the unfused per-conv path (A/B and parity tests)
static bool mrf_fused_enabled() { return sw(SW_MRF_FUSED) != 0; }
// resblock chain kernel for the HBM-bound resblocks (default on; TTS_MRF_CHAIN=0: pairs only)
static bool mrf_chain_enabled() { return sw(SW_MRF_CHAIN) != 0; }
// conv_post inside the vocoder's last pair launch (default on; TTS_POST_FUSE=0: separate launch)
static bool post_fuse_enabled() { return sw(SW_POST_FUSE) != 0; }
// streaming upsampler for the small stages (default on; TTS_UP_STREAM=0: conv_xres)
static bool up_stream_enabled() { return sw(SW_UP_STREAM) != 0; }

struct tts_engine {
  int device = 0;
  tts_config cfg{};
  std::mutex mu;
  std::map<std::string, HostTensor> host;
  bool finalized = false;
  std::vector<void*> allocs;  // weight allocations

  VocoderWeights voc;
  AcousticModel ac;
  Profiler prof;

  // vocoder workspace
  void* vbuf[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  size_t vbuf_elems = 0;
  void* vmel = nullptr;  // normalized mel in compute dtype
  size_t vmel_elems = 0;
  int* vlens = nullptr;  // [16][max_batch]
  int vlens_batch = 0;
  float* vchunk_wav = nullptr;
  size_t vchunk_elems = 0;
  // fp32 vocoder: split-K partials of the resblock convs with >= VWS_MIN_CIN input channels
  // (ConvParams::f32_splitk; at batch 1 -- C1 -- stage 0 at C = 256 ran on 54 blocks, stage 1 on 213)
#ifndef TTS_VWS_MIN_CIN
#define TTS_VWS_MIN_CIN 128
#endif
#ifndef TTS_VOC_SPLIT_MINC
#define TTS_VOC_SPLIT_MINC 32  // fp32 vocoders: resblock convs with >= this many channels run split-precision
#endif
  static constexpr int VWS_MIN_CIN = TTS_VWS_MIN_CIN;  // (A/B builds: 64 with TTS_F32_SK_MINM=32)
  float* vws = nullptr;
  long long vws_bytes = 0;
  // fp32 vocoder: its wide resblock convs run as split-precision GEMMs (finalize_vocoder), whose
  // operands must stay inside f16's range.  Their range word (vrange) is read back after each
  // forward (one stream sync, fp32 vocoders only); when set, the forward reruns with every layer
  // on the fp32 MFMA path (voc_no_split) -- the vocoder counterpart of the exact encoder's guard.
  bool voc_split = false;
  int* vrange = nullptr;
  int* vrange_h = nullptr;  // pinned
  int voc_no_split = 0;
  long long voc_range_fallbacks = 0;
  // polyphase resampler tables, keyed by the reduced (up, down): [up][nq] fp32 on the device
  struct Resampler { int up, down, nq, n_pre_remove; float* hp; };
  std::vector<Resampler> resamplers;

  // The workspace above is shared by every call on this engine.  Every enqueuing call records
  // order_ev on its own stream when it returns (CallOrder below); a call on a stream other than
  // the previous call's first waits for that event, so two callers on two streams never
  // overwrite each other's scratch.  The engine touches a caller's stream only inside that
  // caller's own call: a C caller may destroy its stream as soon as the call has returned.
  hipStream_t last_stream = nullptr;
  bool has_last = false;
  hipEvent_t order_ev = nullptr;
  void order_after_previous(hipStream_t s) {
    if (!order_ev) HIP_CHECK(hipEventCreateWithFlags(&order_ev, hipEventDisableTiming));
    if (has_last && s != last_stream) HIP_CHECK(hipStreamWaitEvent(s, order_ev, 0));
  }
  // records order_ev on s after the call's work (also when the call failed midway: whatever it
  // enqueued is then ordered before the next caller's)
  void order_record(hipStream_t s) {
    if (order_ev && hipEventRecord(order_ev, s) == hipSuccess) {
      last_stream = s;
      has_last = true;
    } else {
      // nothing recorded: the next call on any other stream must not wait on a stale record
      // older than this call's work, so fall back to a full device-side ordering point
      hipStreamSynchronize(s);
      has_last = false;
    }
  }
  struct CallOrder {
    tts_engine* e;
    hipStream_t s;
    CallOrder(tts_engine* e_, hipStream_t s_) : e(e_), s(s_) { e->order_after_previous(s); }
    ~CallOrder() { e->order_record(s); }
  };

  ~tts_engine() {
    hipSetDevice(device);
    if (order_ev) hipEventDestroy(order_ev);
    for (void* p : allocs) dev_free(p);
    for (void*& p : vbuf) if (p) dev_free(p);
    if (vmel) dev_free(vmel);
    if (vlens) dev_free(vlens);
    if (vchunk_wav) dev_free(vchunk_wav);
    if (vws) dev_free(vws);
    for (auto& r : resamplers) dev_free(r.hp);
    if (vrange_h) hipHostFree(vrange_h);
    ac.free_all();
  }

  void* track(void* p) { allocs.push_back(p); return p; }

  const HostTensor& get(const std::string& n) {
    auto it = host.find(n);
    if (it == host.end()) throw TtsError(TTS_ERR_STATE, "missing weight: " + n);
    return it->second;
  }
  bool has(const std::string& n) const { return host.count(n) != 0; }

  // nn.Conv1d weight [Cout][Cin][k] -> W[Cout][k][Cin]; split: an fp32 layer also gets the
  // split-precision packing (three f16 MFMAs per product, conv_split.hip)
  ConvLayer pack_conv(const std::string& wname, const std::string& bname, int dil, int pad, int dt, bool split = false) {
    const HostTensor& w = get(wname);
    if (w.shape.size() != 3) throw TtsError(TTS_ERR_INVALID, wname + ": expected 3-D conv weight");
    std::vector<float> b;
    if (!bname.empty() && has(bname)) b = get(bname).data;
    return make_conv(w.data, (int)w.shape[0], (int)w.shape[1], (int)w.shape[2], b, dil, pad, dt, allocs, nullptr,
                     split && dt == DT_F32);
  }

  // nn.ConvTranspose1d weight [Cin][Cout][k], stride s, padding p as a polyphase conv:
  //   y[u*s + r - p][co] = b[co] + sum_{t<taps} sum_ci x[u + t - (taps-1)][ci] * W[ci][co][r + (taps-1-t)*s]
  // i.e. M = s*Cout rows (r, co), taps = k/s, conv pad = taps-1 (oracle: conv_transpose1d).
  ConvLayer pack_transposed(const std::string& wname, const std::string& bname, int s, int dt) {
    const HostTensor& w = get(wname);
    const int ci = (int)w.shape[0], co = (int)w.shape[1], k = (int)w.shape[2];
    if (k % s || (k - s) % 2) throw TtsError(TTS_ERR_INVALID, wname + ": need k % s == 0 and even k-s");
    const int taps = k / s;
    const int M = s * co;
    std::vector<float> p((size_t)M * taps * ci);
    for (int r = 0; r < s; ++r)
      for (int o = 0; o < co; ++o)
        for (int t = 0; t < taps; ++t) {
          const int j = r + (taps - 1 - t) * s;
          for (int c = 0; c < ci; ++c)
            p[(((size_t)(r * co + o)) * taps + t) * ci + c] = w.data[((size_t)c * co + o) * k + j];
        }
    ConvLayer L;
    L.w = track(upload(p, dt));
    L.wpk = frag_pack(p, M, taps, ci, dt, allocs);
    if (upsample_stream_supported(dt, ci, M, taps)) L.wup16 = frag_pack_up16(p, M, taps * ci, dt, allocs);
    const auto& bh = get(bname).data;
    std::vector<float> b(M);
    for (int r = 0; r < s; ++r)
      for (int o = 0; o < co; ++o) b[r * co + o] = bh[o];
    L.bias = (float*)track(upload_f32(b));
    L.M = M; L.Cin = ci; L.taps = taps; L.dil = 1; L.pad = taps - 1;
    L.up_s = s; L.up_cout = co; L.up_p = (k - s) / 2;
    return L;
  }

  void finalize_vocoder() {
    if (!has("conv_pre.weight")) return;
    const int dt = cfg.vocoder_dtype;
    VocoderWeights& v = voc;
    v.conv_pre = pack_conv("conv_pre.weight", "conv_pre.bias", 1, 3, dt);
    if (has("mean") && has("scale")) {
      v.mean = (float*)track(upload_f32(get("mean").data));
      v.scale = (float*)track(upload_f32(get("scale").data));
      v.normalize = true;
    }
    int nst = 0;
    while (has("upsampler." + std::to_string(nst) + ".weight")) ++nst;
    int nres = 0;
    while (has("resblocks." + std::to_string(nres) + ".convs1.0.weight")) ++nres;
    if (nst == 0 || nres % nst) throw TtsError(TTS_ERR_INVALID, "inconsistent vocoder weights");
    const int nk = nres / nst;
    v.hop = 1;
    v.ups.clear(); v.up_rate.clear(); v.stage_ch.clear(); v.mrf.assign(nst, {});
    for (int i = 0; i < nst; ++i) {
      const HostTensor& w = get("upsampler." + std::to_string(i) + ".weight");
      const int k = (int)w.shape[2];
      // stride from "__cfg__.upsample_rates" if given, else HiFi-GAN V1's k = 2*stride
      int s = k / 2;
      if (has("__cfg__.upsample_rates")) s = (int)std::lround(get("__cfg__.upsample_rates").data.at(i));
      v.ups.push_back(pack_transposed("upsampler." + std::to_string(i) + ".weight",
                                      "upsampler." + std::to_string(i) + ".bias", s, dt));
      v.up_rate.push_back(s);
      v.hop *= s;
      const int ch = (int)w.shape[1];
      v.stage_ch.push_back(ch);
      v.mrf[i].resize(nk);
      for (int j = 0; j < nk; ++j) {
        const std::string pre = "resblocks." + std::to_string(i * nk + j) + ".";
        const int ks = (int)get(pre + "convs1.0.weight").shape[2];
        int np = 0;
        while (has(pre + "convs1." + std::to_string(np) + ".weight")) ++np;
        v.mrf[i][j].resize(np);
        for (int q = 0; q < np; ++q) {
          int d = q == 0 ? 1 : (q == 1 ? 3 : 5);
          if (has("__cfg__.resblock_dilation_sizes")) {
            const HostTensor& dd = get("__cfg__.resblock_dilation_sizes");  // [nk][np]
            d = (int)std::lround(dd.data.at((size_t)j * dd.shape.at(1) + q));
          }
          // fp32 vocoders: the wide stages' resblock convs (C >= TTS_VOC_SPLIT_MINC) as split-precision
          // GEMMs -- C1's batch-1 fp32 vocoder ran them on the fp32 MFMA at 15-25 TF/s
          const bool split = dt == DT_F32 && ch >= TTS_VOC_SPLIT_MINC && ch % 32 == 0;
          v.mrf[i][j][q][0] = pack_conv(pre + "convs1." + std::to_string(q) + ".weight",
                                        pre + "convs1." + std::to_string(q) + ".bias", d, (ks * d - d) / 2, dt, split);
          v.mrf[i][j][q][1] = pack_conv(pre + "convs2." + std::to_string(q) + ".weight",
                                        pre + "convs2." + std::to_string(q) + ".bias", 1, (ks - 1) / 2, dt, split);
          // pair-kernel copies (C in {32, 64}, 16-bit): 16x16 fragment-packed
          for (int cv = 0; cv < 2; ++cv) {
            const HostTensor& cw = get(pre + (cv ? "convs2." : "convs1.") + std::to_string(q) + ".weight");
            if (mrf_pair_supported(dt, ch, ks) && cw.shape[0] == ch && cw.shape[1] == ch)
              v.mrf[i][j][q][cv].wpk16 = frag_pack16(cw.data, ch, ks, dt, allocs);
          }
        }
      }
    }
    const HostTensor& pw = get("conv_post.weight");  // [1][C][k]
    v.post_c = (int)pw.shape[1];
    v.post_k = (int)pw.shape[2];
    std::vector<float> t((size_t)v.post_k * v.post_c);
    for (int c = 0; c < v.post_c; ++c)
      for (int j = 0; j < v.post_k; ++j) t[(size_t)j * v.post_c + c] = pw.data[(size_t)c * v.post_k + j];
    v.post_w = (float*)track(upload_f32(t));
    v.post_wh = dt == DT_F32 ? nullptr : track(upload(t, dt));
    v.post_b = get("conv_post.bias").data[0];
    voc_split = false;
    for (const auto& st : v.mrf)
      for (const auto& rb : st)
        for (const auto& pr : rb) voc_split = voc_split || (dt == DT_F32 && (pr[0].wpk || pr[1].wpk));
    if (voc_split && !vrange) {
      HIP_CHECK(dev_malloc(&vrange, 16));
      HIP_CHECK(hipMemset(vrange, 0, 16));
      track(vrange);
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&vrange_h), 16, hipHostMallocDefault));
    }
    v.loaded = true;
  }

  void reserve_vocoder(int B, int T) {
    if (!voc.loaded) return;
    size_t per_frame = (size_t)voc.conv_pre.M;  // conv_pre output channels
    size_t cum = 1;
    for (size_t i = 0; i < voc.ups.size(); ++i) {
      cum *= voc.up_rate[i];
      per_frame = std::max(per_frame, cum * voc.stage_ch[i]);
    }
    const size_t need = (size_t)B * T * per_frame;
    const int dt = cfg.vocoder_dtype;
    if (need > vbuf_elems) {
      for (void*& p : vbuf) { if (p) dev_free(p); p = nullptr; }
      vbuf_elems = 0;
      for (void*& p : vbuf) {
        if (dev_malloc(&p, need * dtype_size(dt)) != hipSuccess) {
          (void)hipGetLastError();
          p = nullptr;
          for (void*& q : vbuf) { if (q) dev_free(q); q = nullptr; }  // release the partial set
          throw TtsError(TTS_ERR_HIP, "vocoder workspace: hipMalloc of " + std::to_string(need * dtype_size(dt)) +
                                          " bytes failed");
        }
      }
      vbuf_elems = need;
    }
    const size_t mel_need = (size_t)B * T * voc.conv_pre.Cin;
    if (mel_need > vmel_elems) {
      if (vmel) dev_free(vmel);
      vmel = nullptr; vmel_elems = 0;
      HIP_CHECK(dev_malloc(&vmel, mel_need * dtype_size(dt)));
      vmel_elems = mel_need;
    }
    if (dt == DT_F32) {  // split-K partials of the fp32 resblock convs (run_conv)
      long long wsb = 0;
      size_t cum2 = 1;
      for (size_t i = 0; i < voc.ups.size(); ++i) {
        cum2 *= voc.up_rate[i];
        const int C = voc.stage_ch[i];
        if (C >= VWS_MIN_CIN) wsb = std::max(wsb, f32_splitk_ws_bytes(3, C, C, (long long)B * T * (long long)cum2));
      }
      if (wsb > vws_bytes) {
        if (vws) dev_free(vws);
        vws = nullptr; vws_bytes = 0;
        HIP_CHECK(dev_malloc(&vws, (size_t)wsb));
        vws_bytes = wsb;
      }
    }
    if (B > vlens_batch) {
      if (vlens) dev_free(vlens);
      vlens = nullptr; vlens_batch = 0;
      HIP_CHECK(dev_malloc(&vlens, sizeof(int) * 16 * B));
      vlens_batch = B;
    }
  }

  // streaming window output (tts_vocoder_forward_chunk): [B][T_win * hop] fp32
  void reserve_chunk(int B, int T_win) {
    const size_t need = (size_t)B * T_win * voc.hop;
    if (need <= vchunk_elems) return;
    float* old = vchunk_wav;
    vchunk_wav = nullptr; vchunk_elems = 0;
    if (old) HIP_CHECK(dev_free(old));
    HIP_CHECK(dev_malloc(&vchunk_wav, need * 4));
    vchunk_elems = need;
  }

  void run_conv(const ConvLayer& L, const void* x, long long sxb, int sxr, const int* x_len, int x_rows,
                void* y, long long syb, int syr, const int* y_len, int y_rows, float in_slope,
                const void* r1, const void* r2, long long srb, int srr, float out_scale, int B,
                const int* up_len, int dt, hipStream_t s, int act_out = ACT_NONE, float out_slope = 0.f) {
    ConvParams p = conv_params_default();
    p.act_out = act_out; p.out_slope = out_slope;
    p.x = x; p.sxb = sxb; p.sxr = sxr; p.x_len = x_len; p.x_rows = x_rows;
    p.w = L.w; p.w_ld = L.taps * L.Cin; p.wpk = L.wpk; p.w_unscale = L.wpk_unscale;
    p.range_flag = vrange;     // the split-precision layers' range guard (vocoder_forward)
    p.no_split = voc_no_split;  // its fallback: the same layers on the fp32 MFMA path
    p.bias = L.bias;
    p.y = y; p.syb = syb; p.syr = syr;
    p.r1 = r1; p.r2 = r2; p.srb = srb; p.srr = srr;
    p.y_len = y_len; p.y_rows = y_rows;
    p.M = L.M; p.Cin = L.Cin; p.taps = L.taps; p.dil = L.dil; p.pad = L.pad;
    p.in_slope = in_slope; p.out_scale = out_scale;
    p.up_s = L.up_s; p.up_cout = L.up_cout; p.up_p = L.up_p; p.up_len = up_len;
    p.B = B;
    if (dt == DT_F32 && L.Cin >= VWS_MIN_CIN && !L.up_s && vws) {  // (a layer-shape rule: batch-independent sums)
      p.f32_splitk = 1; p.ws = vws; p.ws_bytes = vws_bytes;
    }
    // algorithmic FLOPs: 2 * Cout * Cin * k per produced row (transposed: per input row, all phases)
    const double fl = 2.0 * L.M * (double)L.Cin * L.taps * (double)B * (L.up_s ? (y_rows - 1) : y_rows);
    launch_conv_checked(p, dt, s, &prof, fl);
  }

  // The forward with the split layers' range guard (fp32 vocoders with split-packed convs): one
  // read of the range word after the forward, and a rerun on the fp32 MFMA path when it is set.
  void vocoder_forward(const float* mel, const int* mel_lens, int B, int T, float* wav, long long swb,
                       hipStream_t s) {
    if (!voc_split || voc_no_split) {
      vocoder_forward_once(mel, mel_lens, B, T, wav, swb, s);
      return;
    }
    HIP_CHECK(hipMemsetAsync(vrange, 0, 4, s));
    vocoder_forward_once(mel, mel_lens, B, T, wav, swb, s);
    HIP_CHECK(hipMemcpyAsync(vrange_h, vrange, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (*vrange_h == 0) return;
    ++voc_range_fallbacks;
    voc_no_split = 1;
    try {
      vocoder_forward_once(mel, mel_lens, B, T, wav, swb, s);
    } catch (...) {
      voc_no_split = 0;
      throw;
    }
    voc_no_split = 0;
  }

  // HiFi-GAN V1 forward (oracle/vocoder.py vocoder_forward; HF:1435-1475).
  void vocoder_forward_once(const float* mel, const int* mel_lens, int B, int T, float* wav, long long swb,
                            hipStream_t s) {
    if (!voc.loaded) throw TtsError(TTS_ERR_STATE, "vocoder weights not loaded/finalized");
    const int dt = cfg.vocoder_dtype;
    reserve_vocoder(B, T);
    const VocoderWeights& v = voc;
    const int nst = (int)v.ups.size();
    // per-stage lengths: L[i] = len * cum_i (frames of stage i), U[i] = L[i] + 1 (polyphase rows)
    int mult[8], add[8], n = 0;
    int cum = 1;
    mult[n] = 1; add[n] = 0; ++n;  // L0
    for (int i = 0; i < nst; ++i) { cum *= v.up_rate[i]; mult[n] = cum; add[n] = 0; ++n; }
    if (n > 8) throw TtsError(TTS_ERR_INVALID, "too many stages");
    HIP_CHECK(launch_lens(mel_lens, vlens, B, mult, add, n, s));
    int mult2[8], add2[8];
    cum = 1;
    for (int i = 0; i < nst; ++i) { mult2[i] = cum; add2[i] = 1; cum *= v.up_rate[i]; }
    HIP_CHECK(launch_lens(mel_lens, vlens + 8 * B, B, mult2, add2, nst, s));
    auto Lp = [&](int i) { return vlens + i * B; };
    auto Up = [&](int i) { return vlens + (8 + i) * B; };

    const int cin0 = v.conv_pre.Cin;
    HIP_CHECK(launch_mel_in(dt, mel, (long long)T * cin0, cin0, v.normalize ? v.mean : nullptr, v.scale,
                            vmel, B, T, cin0, s));
    void* XS = vbuf[0];
    void* T1 = vbuf[1];
    void* HA = vbuf[2];
    void* HB = vbuf[3];
    void* S = vbuf[4];
    // conv_pre: [B][T][80] -> S [B][T][512], stored as lrelu(x, 0.1) -- the activation the first
    // upsampler applies (HF:1455-1458), in the conv's fp32 epilogue: S feeds nothing else
    const int c0 = v.conv_pre.M;
    const float slope = 0.1f;
    run_conv(v.conv_pre, vmel, (long long)T * cin0, cin0, Lp(0), T, S, (long long)T * c0, c0, Lp(0), T, 1.f,
             nullptr, nullptr, 0, 0, 1.f, B, nullptr, dt, s, ACT_LRELU, slope);
    int Tin = T, cin = c0;
    // whether S already holds lrelu(S) for the next upsampler (conv_pre, or a stage whose final MRF
    // sum came from a pair launch that applied it, MrfPairParams::out_act); the upsampler then
    // loads it as is, so the X-resident upsamplers can stage it by LDS-DMA
    bool s_act = true;
    bool post_done = false;  // conv_post ran inside the last pair launch
    for (int i = 0; i < nst; ++i) {
      const int ch = v.stage_ch[i];
      const int Tout = Tin * v.up_rate[i];
      const long long sb = (long long)Tout * ch;
      // lrelu -> ConvTranspose1d (polyphase)
      const ConvLayer& U = v.ups[i];
      if (U.wup16 && up_stream_enabled()) {
        UpsampleParams up{};
        up.x = S; up.sxb = (long long)Tin * cin; up.len = Lp(i); up.up_len = Lp(i + 1);
        up.wpk = U.wup16; up.bias = U.bias; up.y = XS; up.syb = sb;
        up.T = Tin; up.B = B; up.s = U.up_s; up.co = U.up_cout; up.pad = U.up_p; up.slope = s_act ? 1.f : slope;
        const double fl = 2.0 * U.M * (double)U.Cin * U.taps * (double)B * Tin;
        if (prof.on) {
          Profiler::Rec r{prof.get(), prof.get(), fl, PK_UPSAMPLE};
          HIP_CHECK(hipEventRecord(r.a, s));
          HIP_CHECK(upsample_stream_launch(dt, U.Cin, U.M, up, s));
          HIP_CHECK(hipEventRecord(r.b, s));
          prof.recs.push_back(r);
        } else {
          HIP_CHECK(upsample_stream_launch(dt, U.Cin, U.M, up, s));
        }
      } else {
        run_conv(U, S, (long long)Tin * cin, cin, Lp(i), Tin, XS, sb, ch, Up(i), Tin + 1, s_act ? 1.f : slope, nullptr,
                 nullptr, 0, 0, 1.f, B, Lp(i + 1), dt, s);
      }
      s_act = false;  // until this stage's final MRF sum says otherwise
      const int nk = (int)v.mrf[i].size();
      // resblock j as single convs: lrelu(h) -> T1 -> conv2 + h (the last one accumulates into S)
      auto convs_resblock = [&](int j) {
        const auto& blk = v.mrf[i][j];
        const int np = (int)blk.size();
        const void* h = XS;
        for (int q = 0; q < np; ++q) {
          run_conv(blk[q][0], h, sb, ch, Lp(i + 1), Tout, T1, sb, ch, Lp(i + 1), Tout, slope, nullptr, nullptr,
                   0, 0, 1.f, B, nullptr, dt, s);
          const bool last = q == np - 1;
          void* out = last ? S : (q % 2 == 0 ? HA : HB);
          const void* r2 = (last && j > 0) ? S : nullptr;
          const float sc = (last && j == nk - 1) ? 1.0f / (float)nk : 1.f;
          run_conv(blk[q][1], T1, sb, ch, Lp(i + 1), Tout, out, sb, ch, Lp(i + 1), Tout, slope, h, r2, sb, ch,
                   sc, B, nullptr, dt, s);
          h = out;
        }
      };
      auto pair_capable = [&](int j) {
        bool ok = true;
        for (const auto& pr : v.mrf[i][j]) ok = ok && pr[0].wpk16 && pr[1].wpk16;
        return ok;
      };
      bool pair_ok = false;
      if (mrf_fused_enabled())
        for (int j = 0; j < nk; ++j) pair_ok = pair_ok || pair_capable(j);
      if (pair_ok) {
        // 9 pair launches: X -> HA -> HB -> S per resblock; S accumulates over resblocks.  A resblock
        // without a pair kernel (its k) runs as single convs in the same S order.
        for (int j = 0; j < nk; ++j) {
          const auto& blk = v.mrf[i][j];
          const int np = (int)blk.size();
          if (!pair_capable(j)) {
            convs_resblock(j);
            continue;
          }
          int dil[4] = {0, 0, 0, 0};
          for (int q = 0; q < np && q < 4; ++q) dil[q] = blk[q][0].dil;
          if (mrf_chain_enabled() && mrf_chain_supported(dt, ch, blk[0][0].taps, dil, np)) {
            // the whole resblock in one launch (HBM-bound resblocks: k = 3 at C <= 64, k = 7 at C = 32)
            MrfChainParams cp{};
            cp.x = XS; cp.y = S; cp.len = Lp(i + 1);
            for (int q = 0; q < 3; ++q) {
              cp.w1[q] = blk[q][0].wpk16; cp.w2[q] = blk[q][1].wpk16;
              cp.b1[q] = blk[q][0].bias; cp.b2[q] = blk[q][1].bias;
            }
            cp.T = Tout; cp.B = B; cp.slope = slope;
            cp.accum = j > 0 ? 1 : 0;
            cp.scale = j == nk - 1 ? 1.0f / (float)nk : 1.f;
            const double fl = 2.0 * 2.0 * ch * (double)ch * blk[0][0].taps * (double)B * Tout * np;
            if (prof.on) {
              Profiler::Rec r{prof.get(), prof.get(), fl, PK_MRF_CHAIN};
              HIP_CHECK(hipEventRecord(r.a, s));
              HIP_CHECK(mrf_chain_launch(dt, ch, blk[0][0].taps, cp, s));
              HIP_CHECK(hipEventRecord(r.b, s));
              prof.recs.push_back(r);
            } else {
              HIP_CHECK(mrf_chain_launch(dt, ch, blk[0][0].taps, cp, s));
            }
            continue;
          }
          const void* h = XS;
          for (int q = 0; q < np; ++q) {
            const bool last = q == np - 1;
            MrfPairParams pp{};
            pp.x = h;
            pp.y = last ? S : (q % 2 == 0 ? HA : HB);
            pp.len = Lp(i + 1);
            pp.w1 = blk[q][0].wpk16; pp.w2 = blk[q][1].wpk16;
            pp.b1 = blk[q][0].bias; pp.b2 = blk[q][1].bias;
            pp.T = Tout; pp.B = B; pp.k = blk[q][0].taps; pp.d = blk[q][0].dil;
            pp.slope = slope;
            pp.tbuf = T1;  // (free in the pair path: the channel-split form's t rows)
            pp.accum = (last && j > 0) ? 1 : 0;
            pp.scale = (last && j == nk - 1) ? 1.0f / (float)nk : 1.f;
            if (last && j == nk - 1 && i == nst - 1 && v.post_wh && post_fuse_enabled() &&
                mrf_pair_post_supported(dt, ch, v.post_k)) {
              // the final MRF sum goes straight into conv_post; S is not written
              pp.post_wpk = v.post_wh; pp.post_b = v.post_b; pp.post_slope = 0.01f; pp.post_k = v.post_k;
              pp.wav = wav; pp.swb = swb;
              post_done = true;
            }
            const double fl = 2.0 * 2.0 * ch * (double)ch * pp.k * (double)B * Tout;
            // the stage's final MRF sum feeds only the next upsampler: store it activated
            if (last && j == nk - 1 && i + 1 < nst && !pp.post_wpk && mrf_pair_outact_supported(dt, ch, pp.k)) {
              pp.out_act = 1; pp.out_slope = slope;
              s_act = true;
            }
            auto launch = [&] { return mrf_pair_launch(dt, ch, pp, s); };
            if (prof.on) {
              Profiler::Rec r{prof.get(), prof.get(), fl, PK_MRF_PAIR};
              HIP_CHECK(hipEventRecord(r.a, s));
              HIP_CHECK(launch());
              HIP_CHECK(hipEventRecord(r.b, s));
              prof.recs.push_back(r);
            } else {
              HIP_CHECK(launch());
            }
            h = pp.y;
          }
        }
        Tin = Tout;
        cin = ch;
        continue;
      }
      for (int j = 0; j < nk; ++j) convs_resblock(j);
      Tin = Tout;
      cin = ch;
    }
    if (!post_done)
      HIP_CHECK(launch_conv_post(dt, S, Lp(nst), B, Tin, cin, v.post_w, v.post_wh, v.post_b, v.post_k, 0.01f, wav,
                                 swb, s));
  }
};

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
template <typename F>
static int guarded(tts_engine* eng, F&& f) {
  try {
    if (!eng) throw TtsError(TTS_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(eng->mu);
    HIP_CHECK(hipSetDevice(eng->device));
    f();
    return TTS_OK;
  } catch (const TtsError& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "out of host memory";
    return TTS_ERR_NOMEM;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return TTS_ERR_INVALID;
  }
}

extern "C" {

const char* tts_last_error(void) { return g_last_error.c_str(); }

int tts_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int tts_abi_version(void) { return TTS_ABI_VERSION; }

int tts_device_bytes(int hip_device, int64_t* bytes) {
  if (!bytes) return TTS_ERR_INVALID;
  *bytes = (int64_t)tts::dev_bytes(hip_device);
  return 0;
}

int tts_engine_create(int hip_device, const tts_config* cfg, tts_engine** out) {
  return tts_engine_create_sized(hip_device, cfg, cfg ? sizeof(tts_config) : 0, out);
}

int tts_engine_create_sized(int hip_device, const tts_config* cfg, size_t cfg_size, tts_engine** out) {
  try {
    if (!out) throw TtsError(TTS_ERR_INVALID, "null out");
    *out = nullptr;
    // the fields a caller's struct does not reach keep their zero defaults (ABI 1's five-int
    // struct: cfg_size 20 -> encoder_precision EXACT); a larger struct is a newer header
    if (cfg && cfg_size % sizeof(int) != 0) throw TtsError(TTS_ERR_INVALID, "cfg_size is not a whole number of fields");
    if (cfg && cfg_size > sizeof(tts_config))
      throw TtsError(TTS_ERR_INVALID, "tts_config of " + std::to_string(cfg_size) + " bytes is newer than this library (" +
                                          std::to_string(sizeof(tts_config)) + ")");
    tts_config c{};
    if (cfg) std::memcpy(&c, cfg, cfg_size);
    auto okdt = [](int d) { return d == DT_F32 || d == DT_F16 || d == DT_BF16; };
    if (!okdt(c.vocoder_dtype) || !okdt(c.acoustic_dtype)) throw TtsError(TTS_ERR_INVALID, "bad dtype");
    if (c.encoder_precision != TTS_ENCODER_EXACT && c.encoder_precision != TTS_ENCODER_FAST)
      throw TtsError(TTS_ERR_INVALID, "bad encoder_precision");
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    if (hip_device < 0 || hip_device >= n)
      throw TtsError(TTS_ERR_INVALID, "hip device " + std::to_string(hip_device) + " out of range");
    std::unique_ptr<tts_engine> e(new tts_engine());
    e->device = hip_device;
    e->cfg = c;
    HIP_CHECK(hipSetDevice(hip_device));
    *out = e.release();
    return TTS_OK;
  } catch (const TtsError& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return TTS_ERR_INVALID;
  }
}

int tts_engine_set_weight(tts_engine* eng, const char* name, const float* host_data, const int64_t* shape,
                          int ndim) {
  return guarded(eng, [&] {
    if (!name || (!host_data) || ndim < 0 || ndim > 8) throw TtsError(TTS_ERR_INVALID, "bad weight args");
    if (eng->finalized) throw TtsError(TTS_ERR_STATE, "engine already finalized");
    HostTensor t;
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) {
      if (shape[i] < 0) throw TtsError(TTS_ERR_INVALID, "negative dim");
      t.shape.push_back(shape[i]);
      n *= (size_t)shape[i];
    }
    t.data.assign(host_data, host_data + n);
    eng->host[name] = std::move(t);
  });
}

int tts_engine_finalize(tts_engine* eng) {
  return guarded(eng, [&] {
    if (eng->finalized) return;
    eng->finalize_vocoder();
    eng->ac.finalize(
        [&](const std::string& n) -> const std::vector<float>* {
          auto it = eng->host.find(n);
          return it == eng->host.end() ? nullptr : &it->second.data;
        },
        [&](const std::string& n) -> std::vector<int64_t> {
          auto it = eng->host.find(n);
          return it == eng->host.end() ? std::vector<int64_t>{} : it->second.shape;
        },
        eng->cfg.acoustic_dtype, eng->cfg.encoder_precision == TTS_ENCODER_EXACT ? DT_F32 : eng->cfg.acoustic_dtype,
        &eng->prof, eng->cfg.encoder_precision == TTS_ENCODER_EXACT && sw(SW_F32_ENC_SPLIT) != 0);
    if (!eng->voc.loaded && !eng->ac.loaded) throw TtsError(TTS_ERR_STATE, "no known weights were set");
    eng->host.clear();
    eng->finalized = true;
    if (eng->cfg.max_batch > 0 && eng->cfg.max_frames > 0 && eng->voc.loaded) {
      eng->reserve_vocoder(eng->cfg.max_batch, eng->cfg.max_frames);
      eng->reserve_chunk(eng->cfg.max_batch, eng->cfg.max_frames);
    }
    if (eng->ac.loaded && eng->cfg.max_batch > 0 && eng->cfg.max_tokens > 0 && eng->cfg.max_frames > 0)
      eng->ac.reserve(eng->cfg.max_batch, eng->cfg.max_tokens, eng->cfg.max_frames);
  });
}

int tts_engine_reserve(tts_engine* eng, int max_batch, int max_frames, int max_tokens) {
  return guarded(eng, [&] {
    if (!eng->finalized) throw TtsError(TTS_ERR_STATE, "finalize first");
    if (max_batch <= 0 || max_frames <= 0) throw TtsError(TTS_ERR_INVALID, "bad reserve sizes");
    if (eng->voc.loaded) {
      eng->reserve_vocoder(max_batch, max_frames);
      eng->reserve_chunk(max_batch, max_frames);
    }
    if (eng->ac.loaded && max_tokens > 0) eng->ac.reserve(max_batch, max_tokens, max_frames);
  });
}

void tts_engine_destroy(tts_engine* eng) { delete eng; }

int tts_vocoder_forward(tts_engine* eng, const float* d_mel, const int32_t* d_mel_lens, int B, int T,
                        float* d_wav, void* stream) {
  return guarded(eng, [&] {
    if (!eng->finalized) throw TtsError(TTS_ERR_STATE, "finalize first");
    if (!d_mel || !d_mel_lens || !d_wav || B <= 0 || T <= 0) throw TtsError(TTS_ERR_INVALID, "bad vocoder args");
    tts_engine::CallOrder order(eng, (hipStream_t)stream);
    eng->vocoder_forward(d_mel, d_mel_lens, B, T, d_wav, (long long)T * eng->voc.hop, (hipStream_t)stream);
  });
}

int tts_vocoder_forward_chunk(tts_engine* eng, const float* d_mel, const int32_t* d_win_lens, int B, int T_win,
                              int ctx_left, int T_chunk, float* d_wav, void* stream) {
  return guarded(eng, [&] {
    if (!eng->finalized) throw TtsError(TTS_ERR_STATE, "finalize first");
    if (!d_mel || !d_win_lens || !d_wav || B <= 0 || T_win <= 0 || ctx_left < 0 || T_chunk <= 0 ||
        ctx_left + T_chunk > T_win)
      throw TtsError(TTS_ERR_INVALID, "bad chunk args");
    hipStream_t s = (hipStream_t)stream;
    tts_engine::CallOrder order(eng, s);
    const int hop = eng->voc.hop;
    eng->reserve_chunk(B, T_win);
    eng->vocoder_forward(d_mel, d_win_lens, B, T_win, eng->vchunk_wav, (long long)T_win * hop, s);
    HIP_CHECK(hipMemcpy2DAsync(d_wav, (size_t)T_chunk * hop * 4, eng->vchunk_wav + (size_t)ctx_left * hop,
                               (size_t)T_win * hop * 4, (size_t)T_chunk * hop * 4, B, hipMemcpyDeviceToDevice, s));
  });
}

int tts_acoustic_forward_spk(tts_engine* eng, const int32_t* d_tokens, const int32_t* d_tok_lens, int B, int N,
                             const int32_t* d_dur_override, const float* d_spk_emb, int spk_dim, float* d_mel,
                             int32_t* d_mel_lens, int Tcap, int32_t* d_durations, void* stream) {
  return guarded(eng, [&] {
    if (!eng->finalized) throw TtsError(TTS_ERR_STATE, "finalize first");
    if (!eng->ac.loaded) throw TtsError(TTS_ERR_STATE, "acoustic weights not loaded");
    if (!d_tokens || !d_tok_lens || !d_mel || !d_mel_lens || B <= 0 || N <= 0 || Tcap <= 0)
      throw TtsError(TTS_ERR_INVALID, "bad acoustic args");
    if (d_spk_emb && eng->ac.speaker_dim() && spk_dim != eng->ac.speaker_dim())
      throw TtsError(TTS_ERR_INVALID, "speaker embedding size does not match the model's projection");
    tts_engine::CallOrder order(eng, (hipStream_t)stream);
    eng->ac.forward(d_tokens, d_tok_lens, B, N, d_dur_override, d_mel, d_mel_lens, Tcap, d_durations, d_spk_emb,
                    (hipStream_t)stream);
  });
}

int tts_acoustic_forward(tts_engine* eng, const int32_t* d_tokens, const int32_t* d_tok_lens, int B, int N,
                         const int32_t* d_dur_override, float* d_mel, int32_t* d_mel_lens, int Tcap,
                         int32_t* d_durations, void* stream) {
  return tts_acoustic_forward_spk(eng, d_tokens, d_tok_lens, B, N, d_dur_override, nullptr, 0, d_mel, d_mel_lens,
                                  Tcap, d_durations, stream);
}

int tts_acoustic_speaker_dim(tts_engine* eng, int* dim) {
  return guarded(eng, [&] {
    if (!dim) throw TtsError(TTS_ERR_INVALID, "null dim");
    *dim = eng->ac.loaded ? eng->ac.speaker_dim() : 0;
  });
}

int tts_acoustic_range_flag(tts_engine* eng, int32_t* dst, void* stream) {
  return guarded(eng, [&] {
    if (!eng->finalized || !eng->ac.loaded) throw TtsError(TTS_ERR_STATE, "acoustic weights not loaded");
    if (!dst) throw TtsError(TTS_ERR_INVALID, "null dst");
    tts_engine::CallOrder order(eng, (hipStream_t)stream);
    eng->ac.range_flag_to(dst, (hipStream_t)stream);
  });
}

int tts_acoustic_set_precision(tts_engine* eng, int precision) {
  return guarded(eng, [&] {
    if (!eng->finalized || !eng->ac.loaded) throw TtsError(TTS_ERR_STATE, "acoustic weights not loaded");
    if (precision != TTS_ENCODER_EXACT && precision != TTS_ENCODER_F32)
      throw TtsError(TTS_ERR_INVALID, "precision must be TTS_ENCODER_EXACT or TTS_ENCODER_F32");
    if (!eng->ac.split_encoder())
      throw TtsError(TTS_ERR_INVALID, "only a model created with TTS_ENCODER_EXACT switches encoder precision");
    eng->ac.set_encoder_f32(precision == TTS_ENCODER_F32);
  });
}

int tts_engine_profile(tts_engine* eng, int enable) {
  return guarded(eng, [&] { eng->prof.on = enable != 0; });
}

int tts_engine_profile_read(tts_engine* eng, double* gemm_ms, double* gemm_flops, int* n_launches) {
  return guarded(eng, [&] { eng->prof.read(gemm_ms, gemm_flops, n_launches); });
}

int tts_set_switch(const char* name, int value) {
  if (tts::sw_set(name, value)) {
    g_last_error = std::string("unknown switch: ") + (name ? name : "(null)");
    return TTS_ERR_INVALID;
  }
  return TTS_OK;
}

int tts_get_switch(const char* name, int* value) {
  if (!value || tts::sw_get(name, value)) {
    g_last_error = std::string("unknown switch: ") + (name ? name : "(null)");
    return TTS_ERR_INVALID;
  }
  return TTS_OK;
}

int tts_engine_profile_read_kinds(tts_engine* eng, int nkinds, double* ms, double* flops, int* n_launches) {
  return guarded(eng, [&] {
    if (nkinds < 1 || !ms || !flops || !n_launches) throw TtsError(TTS_ERR_INVALID, "profile_read_kinds: bad arguments");
    eng->prof.read_kinds(nkinds, ms, flops, n_launches);
  });
}

int tts_resample_filter(int up, int down, double* h, int cap, int* n_pre_remove) {
  try {
    if (up <= 0 || down <= 0) throw TtsError(TTS_ERR_INVALID, "resample: up/down must be positive");
    const int g = std::gcd(up, down);
    std::vector<double> hv;
    int npr = 0;
    const int n = resample_design(up / g, down / g, hv, npr);
    if (n_pre_remove) *n_pre_remove = npr;
    if (h && cap >= n) std::copy(hv.begin(), hv.end(), h);
    return n;
  } catch (const TtsError& e) {
    g_last_error = e.what();
    return e.code;
  }
}

int tts_resample_poly(tts_engine* eng, const float* d_in, int64_t in_stride, const int32_t* d_in_lens, int B,
                      int up, int down, float* d_out, int64_t out_stride, int out_cap, int32_t* d_out_lens,
                      void* stream) {
  return guarded(eng, [&] {
    if (!d_in || !d_in_lens || !d_out || B <= 0 || up <= 0 || down <= 0 || out_cap <= 0 || out_stride < out_cap)
      throw TtsError(TTS_ERR_INVALID, "bad resample args");
    const int g = std::gcd(up, down);
    up /= g; down /= g;
    tts_engine::Resampler* rs = nullptr;
    for (auto& r : eng->resamplers)
      if (r.up == up && r.down == down) rs = &r;
    if (!rs) {
      std::vector<double> h;
      int npr = 0;
      const int n = resample_design(up, down, h, npr);
      const int nq = (n + up - 1) / up;
      std::vector<float> hp((size_t)up * nq, 0.f);
      for (int k = 0; k < n; ++k) hp[(size_t)(k % up) * nq + k / up] = (float)h[k];
      float* d = upload_f32(hp);
      eng->resamplers.push_back({up, down, nq, npr, d});
      rs = &eng->resamplers.back();
    }
    tts_engine::CallOrder order(eng, (hipStream_t)stream);
    HIP_CHECK(launch_resample_poly(d_in, in_stride, d_in_lens, B, up, down, rs->nq, rs->n_pre_remove, rs->hp, d_out,
                                   out_stride, out_cap, d_out_lens, (hipStream_t)stream));
  });
}

int tts_op_conv1d(int dtype, const tts_conv_desc* d, void* stream) {
  try {
    if (!d) throw TtsError(TTS_ERR_INVALID, "null desc");
    if (dtype != DT_F32 && dtype != DT_F16 && dtype != DT_BF16) throw TtsError(TTS_ERR_INVALID, "bad dtype");
    ConvParams p = conv_params_default();
    p.x = d->x; p.sxb = d->sxb; p.sxr = d->sxr; p.x_len = d->x_len; p.x_rows = d->x_rows;
    p.w = d->w; p.swb = d->swb; p.w_ld = d->w_ld; p.bias = d->bias;
    p.y = d->y; p.syb = d->syb; p.syr = d->syr;
    p.r1 = d->r1; p.r2 = d->r2; p.srb = d->srb; p.srr = d->srr;
    p.y_len = d->y_len; p.y_rows = d->y_rows;
    p.M = d->M; p.Cin = d->Cin; p.taps = d->taps; p.dil = d->dil; p.pad = d->pad;
    p.in_slope = d->in_slope; p.act_out = d->act_out; p.out_slope = d->out_slope;
    p.alpha = d->alpha; p.out_scale = d->out_scale;
    p.up_s = d->up_s; p.up_cout = d->up_cout; p.up_p = d->up_p; p.up_len = d->up_len;
    p.B = d->B;
    launch_conv_checked(p, dtype, (hipStream_t)stream, nullptr, 0.0);
    return TTS_OK;
  } catch (const TtsError& e) {
    g_last_error = e.what();
    return e.code;
  }
}

}  // extern "C"
