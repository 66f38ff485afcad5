// FastSpeech2-Conformer acoustic model runtime: tokens -> mel frames on the GPU.
//
// Mirrors oracle/acoustic.py (HF:1099-1288) with B=1-per-utterance semantics on a
// padded batch: every conv masks rows outside [0, len[b]), attention masks keys
// j >= len[b], durations / the all-zero rule are per utterance.
//
// Dense work runs on the implicit-GEMM MFMA kernel:
//   FFN convs (k=3, 384->1536->384), Q|K|V and output projections (k=1),
//   Q.K^T, Q.P^T (relative-position term) and P.V as head-batched GEMMs,
//   conv-module pointwise convs, predictor convs, postnet convs (BatchNorm folded).
// The relative-position projections linear_pos(pos_emb) depend only on the
// relative offset, so they are computed once per layer at load time into a table
// indexed by (RMAX-1 - rel) and every forward reads a window of it.
#include "acoustic.h"

#include <array>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "acoustic_kernels.h"
#include "runtime.h"
#include "switches.h"

#ifndef TTS_DEC_TRIM_RATIO
#define TTS_DEC_TRIM_RATIO 8  // frames per token above which a predicted-duration forward trims the decoder extent
#endif

namespace tts {

namespace {

// TTS_REL_ATTN=0: the unfused attention path (four launches) for A/B and parity tests
bool rel_attn_enabled() { return sw(SW_REL_ATTN) != 0; }

inline int rup(int x, int m) { return (x + m - 1) / m * m; }

struct LNParam {
  float* g = nullptr;
  float* b = nullptr;
};

struct ConformerLayer {
  int dt = DT_F32;  // activation dtype of this layer
  bool split_attn = false;  // fp32 layer of a split encoder side: the split-precision attention
  ConvLayer ffm1, ffm2, ff1, ff2, qkv, out, pw1, pw2, pos;
  float* pos_u = nullptr;
  float* pos_v = nullptr;
  void* ptab = nullptr;  // [2*RMAX][D] linear_pos(rel table) in dt
  float* dw_w = nullptr;  // [D][k] BatchNorm-folded
  float* dw_b = nullptr;
  int dw_k = 0;
  LNParam ln_mac, ln_att, ln_conv, ln_ff, ln_final;
};

struct Predictor {
  int dt = DT_F32;
  std::vector<ConvLayer> convs;
  std::vector<LNParam> lns;
  float* lin_w = nullptr;
  float lin_b = 0.f;
};

}  // namespace

#ifndef TTS_F32_DEC_SPLIT_MAXK
#define TTS_F32_DEC_SPLIT_MAXK 1536  // fp32 decoder layers split-packed up to this K = taps * Cin
#endif

struct AcousticModel::Impl {
  int dt = DT_F32;   // decoder / postnet activations
  int dte = DT_F32;  // encoder, speaker projection, variance adaptor (fp32 + split GEMMs when dt is 16-bit)
  int bdt = DT_F32;  // dtype of the layers being built (finalize)
  bool f32_split_enc = false;  // fp32 model: encoder side on split-precision GEMMs (finalize)
  bool f32_split_dec = false;  // ... and the decoder / postnet GEMMs of short K (finalize)
  bool f32_dec_packed = false; // ... and the decoder's FFN down-projections on the packed split-K form
  bool force_no_split = false; // run(): this launch on the fp32 path (a packed-only layer without pad rows)
  bool enc_side = false;       // the layers being built are the encoder side's (finalize)
  // fp32 layers of a 16-bit model (and the encoder side of an fp32 model with f32_split_enc) get
  // split-packed weights (three f16 MFMAs, conv_split.hip)
  bool split_now() const { return bdt == DT_F32 && (dt != DT_F32 || (f32_split_enc && enc_side)); }
  // the same for one layer of K = taps * Cin: an fp32 model's decoder-side layers split too
  // (f32_split_dec) when K is at most TTS_F32_DEC_SPLIT_MAXK -- they run the per-utterance split
  // kernel, which has no split-K, so the 4,608-deep FFN down-projections stay on the fp32
  // split-K GEMM (C1's batch-1 decoder: 42 blocks walking K = 4,608 would be slower)
  bool split_for(int taps, int cin) const {
    return split_now() || (bdt == DT_F32 && dt == DT_F32 && f32_split_dec && !enc_side &&
                           ((long long)taps * cin <= TTS_F32_DEC_SPLIT_MAXK || f32_dec_packed));
  }
  // the fp32 decoder's deep-K layers (the FFN down-projections, K = 4,608) run split only on the
  // packed form, whose split-K needs the rows past each utterance as pad rows (the per-utterance
  // split kernel has no split-K): with f32_dec_packed the decoder's row stride keeps at least one
  // (dec_pad), so every batch takes the same path -- a stride without them would make the path,
  // and an utterance's bits, depend on the batch's longest utterance
  // (2: the postnet's k = 5 convs need two, and with them every split decoder-side GEMM runs packed)
  int dec_pad() const { return f32_dec_packed ? 2 : 0; }
  bool dec_deep(const ConvLayer& L) const {
    return dt == DT_F32 && f32_dec_packed && L.wpk && (long long)L.taps * L.Cin > TTS_F32_DEC_SPLIT_MAXK;
  }
  void run_deep_ln(const ConvLayer& L, const void* x, int x_rows, const int* lens, void* y, int y_rows, int B, int d,
                   hipStream_t s, float alpha, const void* r1, void* out, const LNParam& a, const LNParam* b2, int rpad) {
    const int keep = cur_rpad;
    const bool packed = rpad >= std::max(1, L.pad);
    if (packed) cur_rpad = rpad; else force_no_split = true;
    run_ln(L, x, x_rows, lens, y, y_rows, B, d, s, alpha, r1, out, a, b2);
    cur_rpad = keep;
    force_no_split = false;
  }
  bool split_enc() const { return dte == DT_F32 && (dt != DT_F32 || f32_split_enc); }
  size_t esz() const { return std::max(dtype_size(dt), dtype_size(dte)); }
  // encoder row stride: at least ENC_PAD masked rows after every utterance, so the split-precision
  // GEMMs run packed 128-row tiles across utterances (ConvParams::rows_pad; k <= 5 convs)
  static constexpr int ENC_PAD = 2;
  static int enc_rows(int N) { return rup(N + ENC_PAD, 32); }
  int cur_rpad = 0;            // rows_pad of the convs being launched (encoder side; an fp32 split decoder)
  float* split_ws = nullptr;   // split-K partial sums of the packed split GEMMs
  long long split_ws_bytes = 0;
  float* attn_ws = nullptr;    // fp32 attention key-chunk partials (fp32 models)
  long long attn_ws_bytes = 0;
  // Range guard of the exact encoder (tts_hip.h, TTS_ENCODER_EXACT): the split GEMMs and the
  // split attention OR 1 into this device word when a staged fp32 operand is outside f16's range;
  // the host reads and clears it (tts_acoustic_range_flag) and reruns with enc_f32 set, which
  // sends the same fp32 layers through the exact fp32 MFMA kernels (no split form).
  int* range_flag = nullptr;
  bool enc_f32 = false;
  void run(const ConvLayer& L, const void* x, int x_rows, const int* lens, void* y, int y_rows, int B, int d,
           hipStream_t s, Profiler* pr, float in_slope = 1.f, int act = ACT_NONE, float alpha = 1.f,
           const void* r1 = nullptr, const ConvParams* ln = nullptr) {
    ConvParams ex = ln ? *ln : conv_params_default();
    ex.range_flag = range_flag;
    ex.no_split = enc_f32 || force_no_split ? 1 : 0;
    ex.f32_splitk = dt == DT_F32 ? 1 : 0;  // fp32 model: split-K over split_ws (sized in reserve_fresh)
    run_layer(L, x, x_rows, lens, y, y_rows, B, d, s, pr, in_slope, act, alpha, r1, nullptr, 1.f, 0, 0, cur_rpad,
              split_ws, split_ws_bytes, &ex);
  }
  // the LayerNorm fields (ConvParams) of a post-LN -- LN2?(LN1(y)) -> out -- with the row-tile
  // counters that let the 16-bit X-resident and one-slice split GEMMs apply it in their own launch
  // (ln_rows.h); the split-K fp32 GEMMs apply it in their reduce, and any other path runs it as a
  // separate launch inside conv_gemm_launch (TTS_LN_FUSE=0: no counters)
  ConvParams ln_params(void* out, const LNParam& a, const LNParam* b2) const {
    ConvParams ln = conv_params_default();
    ln.ln_out = out; ln.ln_g1 = a.g; ln.ln_b1 = a.b; ln.ln_g2 = b2 ? b2->g : nullptr; ln.ln_b2 = b2 ? b2->b : nullptr;
    ln.ln_eps = eps;
    if (sw(SW_LN_FUSE) != 0) { ln.ln_cnt = ln_cnt; ln.ln_cnt_n = ln_cnt_n; }
    return ln;
  }
  // a residual GEMM followed by the block's post-LN: out = LN2?(LN1(y))
  void run_ln(const ConvLayer& L, const void* x, int x_rows, const int* lens, void* y, int y_rows, int B, int d,
              hipStream_t s, float alpha, const void* r1, void* out, const LNParam& a, const LNParam* b2) {
    const ConvParams ln = ln_params(out, a, b2);
    run(L, x, x_rows, lens, y, y_rows, B, d, s, prof, 1.f, ACT_NONE, alpha, r1, &ln);
  }
  Profiler* prof = nullptr;
  int D = 384, H = 2, V = 78, NMEL = 80, FFN = 1536, PRED = 256;
  float eps = 1e-5f;
  void* embed = nullptr;
  std::vector<ConformerLayer> enc, dec;
  Predictor pitch, energy, duration;
  // the predictors' first convs batched along M (pitch | energy | duration, and pitch | energy for
  // given durations) and their first LayerNorms as one grouped launch (predict_batched)
  ConvLayer vp0_all, vp0_pe;
  LnGroups vp_ln{};
  bool vp_batched = false;
  float *pe_w = nullptr, *pe_b = nullptr, *ee_w = nullptr, *ee_b = nullptr;
  ConvLayer feat_out;
  std::vector<ConvLayer> postnet;
  // speaker-embedding projection (HF:1051-1053, 1192-1196): hidden part as a k=1 conv,
  // embedding part (fp32 [D][E]) + bias folded per utterance by spk_bias_kernel
  int E = 0;
  ConvLayer proj_h;
  float *proj_we = nullptr, *proj_b = nullptr;
  void* SPK = nullptr;  // [B][D] per-utterance term, compute dtype
  std::vector<void*> allocs;
  int rmax = 0;
  float* pe_host_table_dummy = nullptr;

  // workspace
  int cap_B = 0, cap_N = 0, cap_T = 0;
  std::vector<void*> ws;
  void *X = nullptr, *Y = nullptr, *O = nullptr, *G = nullptr, *Qu = nullptr, *Qv = nullptr;
  void *H1 = nullptr, *QKV = nullptr, *A = nullptr, *Vt = nullptr, *AC = nullptr, *BD = nullptr, *P = nullptr;
  void *ENC = nullptr, *PB1 = nullptr, *PB2 = nullptr, *BEF = nullptr, *PN1 = nullptr, *PN2 = nullptr, *MELT = nullptr;
  void* VP = nullptr;
  float *f_pitch = nullptr, *f_energy = nullptr, *f_logd = nullptr;
  int *i_dur = nullptr, *i_tokmap = nullptr;
  int* ln_cnt = nullptr;  // row-tile counters of the fused post-LNs (zeroed once; ln_rows.h)
  int ln_cnt_n = 0;
  int* h_lens = nullptr;  // pinned host copy of the frame counts (the decoder-extent read)
  int h_lens_n = 0;

  ~Impl() {
    for (void* p : allocs) dev_free(p);
    for (void* p : ws) dev_free(p);
    for (void* p : score_ws) dev_free(p);
    if (h_lens) hipHostFree(h_lens);
  }

  void* track(void* p) { allocs.push_back(p); return p; }
  float* upf(const std::vector<float>& v) { return (float*)track(upload_f32(v)); }

  // ---------------------------------------------------------------- weights
  const std::vector<float>& need(const GetData& get, const std::string& n) {
    const std::vector<float>* p = get(n);
    if (!p) throw TtsError(TTS_ERR_STATE, "missing acoustic weight: " + n);
    return *p;
  }

  ConvLayer conv(const GetData& get, const GetShape& shape, const std::string& w, const std::string& b, int pad,
                 const std::vector<float>* scale = nullptr, const std::vector<float>* bias_override = nullptr) {
    try {
      return conv_unnamed(get, shape, w, b, pad, scale, bias_override);
    } catch (const TtsError& e) {
      throw TtsError(e.code, w + ": " + e.what());
    }
  }
  ConvLayer conv_unnamed(const GetData& get, const GetShape& shape, const std::string& w, const std::string& b, int pad,
                         const std::vector<float>* scale, const std::vector<float>* bias_override) {
    const auto s = shape(w);
    std::vector<float> bias;
    if (bias_override) bias = *bias_override;
    else if (!b.empty() && get(b)) bias = *get(b);
    if (s.size() == 3)
      return make_conv(need(get, w), (int)s[0], (int)s[1], (int)s[2], bias, 1, pad, bdt, allocs, scale,
                       split_for((int)s[2], (int)s[1]));
    if (s.size() == 2)
      return make_conv(need(get, w), (int)s[0], (int)s[1], 1, bias, 1, 0, bdt, allocs, scale, split_for(1, (int)s[1]));
    throw TtsError(TTS_ERR_INVALID, "bad weight rank: " + w);
  }

  LNParam ln(const GetData& get, const std::string& p) {
    LNParam l;
    l.g = upf(need(get, p + ".weight"));
    l.b = upf(need(get, p + ".bias"));
    return l;
  }

  ConformerLayer layer(const GetData& get, const GetShape& shape, const std::string& p) {
    ConformerLayer L;
    L.dt = bdt;
    const int kf = (int)shape(p + "feed_forward.conv1.weight").at(2);
    L.ffm1 = conv(get, shape, p + "feed_forward_macaron.conv1.weight", p + "feed_forward_macaron.conv1.bias", (kf - 1) / 2);
    L.ffm2 = conv(get, shape, p + "feed_forward_macaron.conv2.weight", p + "feed_forward_macaron.conv2.bias", (kf - 1) / 2);
    L.ff1 = conv(get, shape, p + "feed_forward.conv1.weight", p + "feed_forward.conv1.bias", (kf - 1) / 2);
    L.ff2 = conv(get, shape, p + "feed_forward.conv2.weight", p + "feed_forward.conv2.bias", (kf - 1) / 2);
    // fused Q|K|V projection [3D][D]
    const std::string a = p + "self_attn.";
    std::vector<float> wq, bq;
    for (const char* n : {"linear_q", "linear_k", "linear_v"}) {
      const auto& w = need(get, a + n + ".weight");
      const auto& b = need(get, a + n + ".bias");
      wq.insert(wq.end(), w.begin(), w.end());
      bq.insert(bq.end(), b.begin(), b.end());
    }
    L.qkv = make_conv(wq, 3 * D, D, 1, bq, 1, 0, bdt, allocs, nullptr, split_for(1, D));
    L.split_attn = split_now();
    L.out = conv(get, shape, a + "linear_out.weight", a + "linear_out.bias", 0);
    L.pos = make_conv(need(get, a + "linear_pos.weight"), D, D, 1, {}, 1, 0, bdt, allocs, nullptr, split_now());
    L.pos_u = upf(need(get, a + "pos_bias_u"));
    L.pos_v = upf(need(get, a + "pos_bias_v"));
    const std::string c = p + "conv_module.";
    L.pw1 = conv(get, shape, c + "pointwise_conv1.weight", c + "pointwise_conv1.bias", 0);
    L.pw2 = conv(get, shape, c + "pointwise_conv2.weight", c + "pointwise_conv2.bias", 0);
    // depthwise conv with BatchNorm folded: w' = w*s, b' = (b - rm)*s + beta, s = g / sqrt(rv + eps)
    const auto& dw = need(get, c + "depthwise_conv.weight");  // [D][1][k]
    const int k = (int)shape(c + "depthwise_conv.weight").at(2);
    const auto& dwb = need(get, c + "depthwise_conv.bias");
    const auto& g = need(get, c + "norm.weight");
    const auto& be = need(get, c + "norm.bias");
    const auto& rm = need(get, c + "norm.running_mean");
    const auto& rv = need(get, c + "norm.running_var");
    std::vector<float> wf((size_t)D * k), bf(D);
    for (int ch = 0; ch < D; ++ch) {
      const float s = g[ch] / std::sqrt(rv[ch] + eps);
      for (int j = 0; j < k; ++j) wf[(size_t)ch * k + j] = dw[(size_t)ch * k + j] * s;
      bf[ch] = (dwb[ch] - rm[ch]) * s + be[ch];
    }
    L.dw_w = upf(wf);
    L.dw_b = upf(bf);
    L.dw_k = k;
    L.ln_mac = ln(get, p + "ff_macaron_layer_norm");
    L.ln_att = ln(get, p + "self_attn_layer_norm");
    L.ln_conv = ln(get, p + "conv_layer_norm");
    L.ln_ff = ln(get, p + "ff_layer_norm");
    L.ln_final = ln(get, p + "final_layer_norm");
    return L;
  }

  Predictor predictor(const GetData& get, const GetShape& shape, const std::string& p) {
    Predictor P;
    P.dt = bdt;
    for (int i = 0;; ++i) {
      const std::string q = p + "conv_layers." + std::to_string(i) + ".";
      if (!get(q + "conv.weight")) break;
      const int k = (int)shape(q + "conv.weight").at(2);
      P.convs.push_back(conv(get, shape, q + "conv.weight", q + "conv.bias", (k - 1) / 2));
      P.lns.push_back(ln(get, q + "layer_norm"));
    }
    if (P.convs.empty()) throw TtsError(TTS_ERR_STATE, "predictor without layers: " + p);
    P.lin_w = upf(need(get, p + "linear.weight"));
    P.lin_b = need(get, p + "linear.bias").at(0);
    return P;
  }

  // The three variance predictors read the same encoder output (HF:1198-1210): their first convs
  // run as one GEMM whose M blocks are the three layers' and their first LayerNorms as one grouped
  // launch; each predictor's second conv reads its slice of the batched rows.  Two launches
  // instead of six at the start of the variance adaptor, where the 80-block grids of batch 8 left
  // two thirds of the CUs idle.  The layers' kernel widths differ (HF: pitch 5, energy and
  // duration 3): the narrower ones are zero-padded to the widest tap for tap, centred, so each
  // output channel's products arrive in the layer's own order with exact zeros (+0 products)
  // around them -- the same sums, bit for bit (tests/test_acoustic_gpu.py).  fp32 encoder
  // activations only (the exact encoder and fp32 models); the fast 16-bit encoder keeps the
  // per-predictor launches.
  void batch_predictors(const GetData& get, const GetShape& shape) {
    vp_batched = false;
    if (bdt != DT_F32 || sw(SW_VP_BATCH) == 0) return;
    Predictor* ps[3] = {&pitch, &energy, &duration};
    const ConvLayer& c0 = pitch.convs.at(0);
    int kmax = 1;
    for (Predictor* q : ps) {
      const ConvLayer& c = q->convs.at(0);
      if (q->convs.size() < 2 || c.M != c0.M || c.Cin != c0.Cin || c.pad != (c.taps - 1) / 2 || c.taps % 2 == 0 ||
          c.dil != 1 || c.M > 256)
        return;
      kmax = std::max(kmax, c.taps);
    }
    const char* names[3] = {"pitch_predictor.", "energy_predictor.", "duration_predictor."};
    const int M = c0.M, Ci = c0.Cin;
    std::vector<float> w, b;  // [3 M][Cin][kmax] (PyTorch Conv1d layout), taps centred
    for (int i = 0; i < 3; ++i) {
      const std::string q = std::string(names[i]) + "conv_layers.0.";
      const auto& wi = need(get, q + "conv.weight");
      const int k = (int)shape(q + "conv.weight").at(2), off = (kmax - k) / 2;
      if (wi.size() != (size_t)M * Ci * k) return;
      std::vector<float> wp((size_t)M * Ci * kmax, 0.f);
      for (size_t oc = 0; oc < (size_t)M * Ci; ++oc)
        for (int t = 0; t < k; ++t) wp[oc * kmax + off + t] = wi[oc * k + t];
      w.insert(w.end(), wp.begin(), wp.end());
      if (get(q + "conv.bias")) {
        const auto& bi = *get(q + "conv.bias");
        b.insert(b.end(), bi.begin(), bi.end());
      } else {
        b.insert(b.end(), (size_t)M, 0.f);
      }
      vp_ln.g[i] = ps[i]->lns.at(0).g;
      vp_ln.b[i] = ps[i]->lns.at(0).b;
      if (i == 1)
        vp0_pe = make_conv(w, 2 * M, Ci, kmax, b, 1, (kmax - 1) / 2, bdt, allocs, nullptr, split_now());
    }
    vp0_all = make_conv(w, 3 * M, Ci, kmax, b, 1, (kmax - 1) / 2, bdt, allocs, nullptr, split_now());
    vp_batched = true;
  }

  // relative-position table through linear_pos, rows q <-> rel = rmax-1-q (HF:723-752, 419)
  void build_ptabs(int new_rmax, hipStream_t s) {
    const int rows = 2 * new_rmax;
    std::vector<float> pe((size_t)rows * D, 0.f);
    for (int q = 0; q < 2 * new_rmax - 1; ++q) {
      const float rel = (float)(new_rmax - 1 - q);
      for (int i = 0; i < D / 2; ++i) {
        const float div = std::exp((float)(2 * i) * (float)(-(std::log(10000.0) / D)));
        const double ang = (double)(rel * div);
        pe[(size_t)q * D + 2 * i] = (float)std::sin(ang);
        pe[(size_t)q * D + 2 * i + 1] = (float)std::cos(ang);
      }
    }
    void* ped[3] = {nullptr, nullptr, nullptr};  // the table in each layer dtype used
    for (auto* stack : {&enc, &dec})
      for (auto& L : *stack) {
        if (L.ptab) {
          dev_free(L.ptab);
          for (auto& a : allocs) if (a == L.ptab) a = nullptr;
        }
        if (!ped[L.dt]) ped[L.dt] = upload(pe, L.dt);
        void* t = nullptr;
        HIP_CHECK(dev_malloc(&t, (size_t)rows * D * dtype_size(L.dt)));
        L.ptab = track(t);
        run_layer(L.pos, ped[L.dt], rows, nullptr, L.ptab, rows, 1, L.dt, s, nullptr);
      }
    HIP_CHECK(hipStreamSynchronize(s));
    for (void* p : ped) if (p) dev_free(p);
    rmax = new_rmax;
  }

  // ---------------------------------------------------------------- workspace
  void* alloc_ws(size_t elems, size_t esz) {
    void* p = nullptr;
    HIP_CHECK(dev_malloc(&p, std::max<size_t>(elems, 1) * esz));
    HIP_CHECK(hipMemset(p, 0, std::max<size_t>(elems, 1) * esz));
    ws.push_back(p);
    return p;
  }

  // Drop the workspace: caps to 0 and every pointer to null BEFORE freeing, so a failed
  // re-reservation (HIP_CHECK throws midway) can never leave a cap describing freed memory.
  void drop_ws() {
    cap_B = cap_N = cap_T = 0;
    X = Y = O = G = Qu = Qv = H1 = QKV = A = Vt = ENC = SPK = PB1 = PB2 = BEF = PN1 = PN2 = MELT = VP = nullptr;
    f_pitch = f_energy = f_logd = nullptr;
    i_dur = i_tokmap = nullptr;
    ln_cnt = nullptr;
    ln_cnt_n = 0;
    split_ws = nullptr;
    split_ws_bytes = 0;
    attn_ws = nullptr;
    attn_ws_bytes = 0;
    std::vector<void*> old;
    old.swap(ws);
    for (void* p : old) dev_free(p);
    drop_scores();
  }

  // The unfused attention path's score buffers (AC / BD / P: B*H*Tm*(Sac+Sbd+Sk) elements,
  // quadratic in the frame cap) exist only while that path runs (fp32, TTS_REL_ATTN=0).
  int cap_sB = 0, cap_sTm = 0;
  std::vector<void*> score_ws;
  void drop_scores() {
    cap_sB = cap_sTm = 0;
    AC = BD = P = nullptr;
    std::vector<void*> old;
    old.swap(score_ws);
    for (void* p : old) dev_free(p);
  }
  void reserve_scores(int B, int Tm) {
    if (B <= cap_sB && Tm <= cap_sTm) return;
    B = std::max(B, cap_sB); Tm = std::max(Tm, cap_sTm);
    drop_scores();
    const size_t e = esz();
    const int Sk = rup(Tm, 16), Sac = rup(Tm, 16), Sbd = rup(2 * Tm, 16);
    auto al = [&](size_t n) { void* p = alloc_ws(n, e); ws.pop_back(); score_ws.push_back(p); return p; };
    AC = al((size_t)B * H * Tm * Sac);
    BD = al((size_t)B * H * Tm * Sbd);
    P = al((size_t)B * H * Tm * Sk);
    cap_sB = B; cap_sTm = Tm;
  }

  void reserve(int B, int N, int T) {
    if (B <= cap_B && N <= cap_N && T <= cap_T) return;
    B = std::max(B, cap_B); N = std::max(N, cap_N); T = std::max(T, cap_T);
    drop_ws();
    try {
      reserve_fresh(B, N, T);
    } catch (...) {
      drop_ws();  // release what was allocated before the failure; caps stay 0
      throw;
    }
  }

  void reserve_fresh(int B, int N, int T) {
    const size_t ee = dtype_size(dte), ed = dtype_size(dt);  // encoder-side / decoder-side element sizes
    const int Tm = std::max(N, T);
    const int Tp = std::max(rup(Tm + dec_pad(), 32), enc_rows(N));
    const int dk = D / H;
    const size_t rows = (size_t)B * Tp;
    const size_t nrows = (size_t)B * enc_rows(N);
    // buffers both stacks use: the encoder's nrows in dte, the decoder's rows in dt (an fp32
    // exact encoder of a 16-bit model needs 4-byte elements only for its own B*Np rows)
    auto both = [&](size_t C) { return alloc_ws(std::max(nrows * C * ee, rows * C * ed), 1); };
    X = both(D); Y = both(D); O = both(D); G = both(D);
    Qu = both(D); Qv = both(D);
    H1 = both(FFN); QKV = both(3 * D); A = both(2 * D);
    Vt = alloc_ws(std::max((size_t)B * H * dk * rup(N, 16) * ee, (size_t)B * H * dk * rup(Tm, 16) * ed), 1);
    ENC = alloc_ws(nrows * D, ee);
    SPK = alloc_ws((size_t)B * D, ee);
    PB1 = alloc_ws(nrows * PRED, std::max<size_t>(ee, 2)); PB2 = alloc_ws(nrows * PRED, ee);  // PB1 also holds f32 logd [B][N]
    VP = alloc_ws(nrows * 3 * 256, 4);  // the batched first predictor convs (fp32, <= 256 channels each)
    const size_t trows = (size_t)B * rup(T + dec_pad(), 32);
    BEF = alloc_ws(trows * NMEL, ed); MELT = alloc_ws(trows * NMEL, ed);
    PN1 = alloc_ws(trows * PRED, ed); PN2 = alloc_ws(trows * PRED, ed);
    f_pitch = (float*)alloc_ws(nrows, 4); f_energy = (float*)alloc_ws(nrows, 4); f_logd = (float*)alloc_ws(nrows, 4);
    i_dur = (int*)alloc_ws((size_t)B * N, 4);
    i_tokmap = (int*)alloc_ws((size_t)B * T, 4);
    // one counter per row tile of the fused post-LN launches: >= 64-row tiles per utterance (conv_xres)
    // or over the packed encoder rows (conv_splitp)
    ln_cnt_n = (int)std::max((size_t)B * (std::max(Tp, enc_rows(N)) / 32 + 2), nrows / 32 + 2);
    ln_cnt = (int*)alloc_ws((size_t)ln_cnt_n, 4);
    // split-K partials of the encoder's packed split GEMMs (fp32 encoder of a 16-bit model)
    long long wsb = 0;
    if (split_enc()) {
      const int F = B * enc_rows(N);
      for (auto& L : enc)
        for (const ConvLayer* c : {&L.ffm1, &L.ffm2, &L.ff1, &L.ff2, &L.qkv, &L.out, &L.pw1, &L.pw2})
          wsb = std::max(wsb, conv_split_ws_bytes(c->taps, c->Cin, c->M, F));
      for (const Predictor* pr : {&pitch, &energy, &duration})
        for (const ConvLayer& c : pr->convs) wsb = std::max(wsb, conv_split_ws_bytes(c.taps, c.Cin, c.M, F));
    }
    if (dt == DT_F32) {  // fp32 model: the split-K partials of its fp32 conv_gemm launches (every
                         // layer: a split encoder's fallback runs its layers on them too)
      const long long F = (long long)B * Tp;  // >= every stack's B * rows
      auto add = [&](const ConvLayer& c) { wsb = std::max(wsb, f32_splitk_ws_bytes(c.taps, c.Cin, c.M, F)); };
      for (const auto* st : {&enc, &dec})
        for (auto& L : *st)
          for (const ConvLayer* c : {&L.ffm1, &L.ffm2, &L.ff1, &L.ff2, &L.qkv, &L.out, &L.pw1, &L.pw2, &L.pos}) add(*c);
      for (const Predictor* pr : {&pitch, &energy, &duration})
        for (const ConvLayer& c : pr->convs) add(c);
      add(vp0_all); add(vp0_pe); add(feat_out);
      for (const ConvLayer& c : postnet) add(c);
    }
    split_ws = wsb ? (float*)alloc_ws((size_t)wsb, 1) : nullptr;
    split_ws_bytes = wsb;
    // fp32 models: the key-chunk partials of the fp32 attention (attention.hip), both stacks
    attn_ws_bytes = dt == DT_F32 ? rel_attn_f32_ws_bytes(B, Tm, Tp, D, H) : 0;
    // the split-precision attention of an fp32 encoder side (key chunks in TTS_ATTN_SPLIT_KC builds)
    if (dte == DT_F32) attn_ws_bytes = std::max(attn_ws_bytes, rel_attn_split_ws_bytes(B, N, enc_rows(N), D, H));
    attn_ws = attn_ws_bytes ? (float*)alloc_ws((size_t)attn_ws_bytes, 1) : nullptr;
    cap_B = B; cap_N = N; cap_T = T;
  }

  // ---------------------------------------------------------------- forward
  // a non-GEMM launch (profiled as PK_AC_ELEM when the bench's live timing is on)
  template <typename F>
  void elem(hipStream_t s, F&& f) { prof_launch(PK_AC_ELEM, 0.0, s, f); }
  template <typename F>
  void prof_launch(int kind, double flops, hipStream_t s, F&& f) {
    if (prof) prof->launch(kind, flops, s, f);
    else HIP_CHECK(f());
  }
  // one head-batched attention GEMM: Y[b,h][n][m] = sum_c X[b,h][n][c] * W[b,h][m][c]
  void attn_gemm(int d, const void* x, long long sxb, long long sxh, int sxr, const int* lens, int x_rows, const void* w,
                 long long swb, long long swh, int w_ld, int M, int K, void* y, long long syb, long long syh,
                 int syr, int B, hipStream_t s) {
    ConvParams p = conv_params_default();
    p.x = x; p.sxb = sxb; p.sxh = sxh; p.sxr = sxr; p.x_len = lens; p.x_rows = x_rows;
    p.w = w; p.swb = swb; p.swh = swh; p.w_ld = w_ld;
    p.y = y; p.syb = syb; p.syh = syh; p.syr = syr;
    p.y_len = lens; p.y_rows = x_rows;
    p.M = M; p.Cin = K; p.taps = 1; p.dil = 1; p.pad = 0;
    p.B = B; p.nh = H;
    launch_conv_checked(p, d, s, prof, 2.0 * M * (double)K * x_rows * B * H);
  }

  // Tm: longest utterance (attention extent); Tp: row stride of Xb and the workspace
  void stack(std::vector<ConformerLayer>& layers, void* Xb, const int* lens, int B, int Tm, int Tp, hipStream_t s) {
    const int dk = D / H;
    const int rows = B * Tp;
    const int Sk = rup(Tm, 16), Sac = rup(Tm, 16), Sbd = rup(2 * Tm, 16);
    const int Mk = rup(Tm, 4), Mbd = rup(2 * Tm - 1, 4);
    const float scale = 1.0f / std::sqrt((float)dk);
    for (auto& L : layers) {
      const int dt = L.dt;
      // macaron FFN: x = LN(x + 0.5 * ffn(x))
      run(L.ffm1, Xb, Tp, lens, H1, Tp, B, dt, s, prof, 1.f, ACT_RELU);
      if (!L.split_attn && dec_deep(L.ffm2)) run_deep_ln(L.ffm2, H1, Tp, lens, Y, Tp, B, dt, s, 0.5f, Xb, Xb, L.ln_mac, nullptr, Tp - Tm);
      else run_ln(L.ffm2, H1, Tp, lens, Y, Tp, B, dt, s, 0.5f, Xb, Xb, L.ln_mac, nullptr);
      // relative-position MHSA: x = LN(x + mhsa(x))
      run(L.qkv, Xb, Tp, lens, QKV, Tp, B, dt, s, prof);
      const bool fused_attn = rel_attn_enabled() && rel_attn_supported(dt, D, H);
      if (!fused_attn) elem(s, [&] { return launch_pos_bias(dt, QKV, rows, D, L.pos_u, L.pos_v, Qu, Qv, s); });
      if (fused_attn) {
        // fused flash-style relative-position attention (attention.hip); Qu / Qv formed in it,
        // V read from the QKV rows (transposed in LDS: no Vt launch)
        // fp32 layers of a 16-bit model (the exact-duration encoder) in split precision, like their GEMMs
        // (the decoder of an fp32 model keeps the fp32 attention: key chunks, attention.hip)
        const bool split = dt == DT_F32 && L.split_attn && !enc_f32;
        if (TTS_BOUNDS_CHECK) {  // (diagnostic builds: runtime.h)
          const long long e = dtype_size(dt);
          std::string why;
          if (!dev_range_ok(QKV, (long long)B * Tp * 3 * D * e, &why) || !dev_range_ok(O, (long long)B * Tp * D * e, &why) ||
              !dev_range_ok(L.ptab, 2LL * rmax * D * e, &why))
            throw TtsError(TTS_ERR_INVALID, "bounds: attention " + why);
        }
        prof_launch(PK_ATTN, 6.0 * D * (double)B * Tm * Tm, s, [&] { return launch_rel_attn(dt, split, L.pos_u, L.pos_v, QKV, L.ptab, lens, B, Tm, Tp, D, H, rmax, scale,
                                  O, s, range_flag, attn_ws, attn_ws_bytes); });
        run_ln(L.out, O, Tp, lens, Y, Tp, B, dt, s, 1.f, Xb, Xb, L.ln_att, nullptr);
        conv_module_and_ffn(L, Xb, lens, B, Tp, rows, s, Tp - Tm);
        continue;
      }
      elem(s, [&] { return launch_transpose_v(dt, QKV, lens, B, Tp, D, H, Sk, Vt, s); });
      const size_t e = dtype_size(dt);
      // AC[b,h][i][j] = Qu[b][i][h] . K[b][j][h]
      attn_gemm(dt, Qu, (long long)Tp * D, dk, D, lens, Tm, (const char*)QKV + (size_t)D * e, (long long)Tp * 3 * D, dk,
                3 * D, Mk, dk, AC, (long long)H * Tm * Sac, (long long)Tm * Sac, Sac, B, s);
      // BD[b,h][i][q] = Qv[b][i][h] . Ptab[rmax - Tm + q][h]   (q <-> rel = Tm-1-q)
      attn_gemm(dt, Qv, (long long)Tp * D, dk, D, lens, Tm, (const char*)L.ptab + (size_t)(rmax - Tm) * D * e, 0, dk, D,
                Mbd, dk, BD, (long long)H * Tm * Sbd, (long long)Tm * Sbd, Sbd, B, s);
      elem(s, [&] { return launch_rel_softmax(dt, AC, BD, lens, B, H, Tm, Sac, Sbd, Sk, scale, P, s); });
      // O[b][i][h*dk + d] = sum_j P[b,h][i][j] * Vt[b,h][d][j]
      attn_gemm(dt, P, (long long)H * Tm * Sk, (long long)Tm * Sk, Sk, lens, Tm, Vt, (long long)H * dk * Sk,
                (long long)dk * Sk, Sk, dk, Sk, O, (long long)Tp * D, dk, D, B, s);
      run_ln(L.out, O, Tp, lens, Y, Tp, B, dt, s, 1.f, Xb, Xb, L.ln_att, nullptr);
      conv_module_and_ffn(L, Xb, lens, B, Tp, rows, s, Tp - Tm);
    }
  }

  void conv_module_and_ffn(ConformerLayer& L, void* Xb, const int* lens, int B, int Tp, int rows, hipStream_t s,
                           int rpad) {
    const int dt = L.dt;
    // conv module: x = LN(x + pw2(silu(bn(dw(glu(pw1(x)))))))
    run(L.pw1, Xb, Tp, lens, A, Tp, B, dt, s, prof);
    elem(s, [&] { return launch_glu_dwconv(dt, A, lens, B, Tp, D, L.dw_w, L.dw_k, L.dw_b, G, s); });
    run_ln(L.pw2, G, Tp, lens, Y, Tp, B, dt, s, 1.f, Xb, Xb, L.ln_conv, nullptr);
    // FFN: x = final_LN(LN(x + 0.5 * ffn(x)))
    run(L.ff1, Xb, Tp, lens, H1, Tp, B, dt, s, prof, 1.f, ACT_RELU);
    if (!L.split_attn && dec_deep(L.ff2)) run_deep_ln(L.ff2, H1, Tp, lens, Y, Tp, B, dt, s, 0.5f, Xb, Xb, L.ln_ff, &L.ln_final, rpad);
    else run_ln(L.ff2, H1, Tp, lens, Y, Tp, B, dt, s, 0.5f, Xb, Xb, L.ln_ff, &L.ln_final);
  }

  // The three predictors run in sequence on one stream: pitch and energy on two side streams
  // (they read the same encoder output, HF:1198-1210) shortened the predictor span in kernel
  // traces (batch 8: 270 -> 149 us) but cost 0.1-0.3 ms end to end in the C3 / C5 measurements
  // (fork / join across hardware queues), so they stay sequential.
  void predict(Predictor& Pr, const void* x, const int* lens, int B, int Np, float* out, hipStream_t s) {
    const int dt = Pr.dt;
    const void* h = x;
    void* bufs[2] = {PB1, PB2};
    const int n = (int)Pr.convs.size();
    for (int i = 0; i < n; ++i) {
      void* o = bufs[i & 1];
      // conv + ReLU, then its LayerNorm in place (the last layer: LayerNorm + Linear(C -> 1) -> out)
      ConvParams ln = ln_params(i + 1 < n ? o : nullptr, Pr.lns[i], nullptr);
      if (i + 1 == n) { ln.ln_lin_w = Pr.lin_w; ln.ln_lin_b = Pr.lin_b; ln.ln_lin_out = out; }
      run(Pr.convs[i], h, Np, lens, o, Np, B, dt, s, prof, 1.f, ACT_RELU, 1.f, nullptr, &ln);
      h = o;
    }
  }

  // the three (with_dur) or two predictors with the batched first conv and grouped first LayerNorm
  // (batch_predictors); each second conv reads its predictor's slice of VP (row stride G * PRED)
  void predict_batched(const void* x, const int* lens, int B, int Np, bool with_dur, hipStream_t s) {
    const int G = with_dur ? 3 : 2;
    const int C = pitch.convs[0].M;
    run(with_dur ? vp0_all : vp0_pe, x, Np, lens, VP, Np, B, DT_F32, s, prof, 1.f, ACT_RELU);
    elem(s, [&] { return launch_layernorm_groups(DT_F32, VP, B * Np, C, G * C, vp_ln, G, eps, s, lens, Np); });
    Predictor* ps[3] = {&pitch, &energy, &duration};
    float* outs[3] = {f_pitch, f_energy, f_logd};
    for (int g = 0; g < G; ++g) {
      Predictor& Pr = *ps[g];
      const void* h = reinterpret_cast<const float*>(VP) + (size_t)g * C;
      int ld = G * C;
      void* bufs[2] = {PB1, PB2};
      const int n = (int)Pr.convs.size();
      for (int i = 1; i < n; ++i) {
        void* o = bufs[i & 1];
        ConvParams ln = ln_params(i + 1 < n ? o : nullptr, Pr.lns[i], nullptr);
        if (i + 1 == n) { ln.ln_lin_w = Pr.lin_w; ln.ln_lin_b = Pr.lin_b; ln.ln_lin_out = outs[g]; }
        ConvParams ex = ln;
        ex.range_flag = range_flag;
        ex.no_split = enc_f32 ? 1 : 0;
        ex.f32_splitk = dt == DT_F32 ? 1 : 0;
        run_layer(Pr.convs[i], h, Np, lens, o, Np, B, DT_F32, s, prof, 1.f, ACT_RELU, 1.f, nullptr, nullptr, 1.f, ld, 0,
                  cur_rpad, split_ws, split_ws_bytes, &ex);
        h = o;
        ld = 0;
      }
    }
  }

  void forward(const int* tokens, const int* tok_lens, int B, int N, const int* dur_override, float* mel,
               int* mel_lens, int Tcap, int* durations, const float* spk, hipStream_t s) {
    reserve(B, N, Tcap);
    const int Tm = std::max(N, Tcap);
    {  // the unfused attention's score buffers, for the stacks that run it (fp32 / TTS_REL_ATTN=0)
      const bool fused = rel_attn_enabled();
      const int need = std::max(fused && rel_attn_supported(dte, D, H) ? 0 : N,
                                fused && rel_attn_supported(dt, D, H) ? 0 : Tcap);
      if (need) reserve_scores(B, need);
    }
    if (Tm > rmax) build_ptabs(rup(Tm, 256), s);
    const float xscale = std::sqrt((float)D);
    const int Np = enc_rows(N);
    // encoder
    elem(s, [&] { return launch_embed(dte, tokens, tok_lens, B, N, Np, embed, V, D, xscale, ENC, s); });
    cur_rpad = Np - N;  // encoder side: packed-row split GEMMs
    stack(enc, ENC, tok_lens, B, N, Np, s);
    if (spk && E) {  // speaker embedding (HF:1192-1196); without one HF skips the projection
      elem(s, [&] { return launch_spk_bias(dte, spk, B, E, proj_we, proj_b, D, SPK, s); });
      ConvParams p = conv_params_default();
      p.x = ENC; p.sxb = (long long)Np * D; p.sxr = D; p.x_len = tok_lens; p.x_rows = Np;
      p.w = proj_h.w; p.w_ld = D; p.bias = nullptr; p.wpk = proj_h.wpk; p.w_unscale = proj_h.wpk_unscale;
      p.y = Y; p.syb = (long long)Np * D; p.syr = D;
      p.r1 = SPK; p.srb = D; p.srr = 0;  // the utterance's term broadcast over its frames
      p.y_len = tok_lens; p.y_rows = Np;
      p.M = D; p.Cin = D; p.B = B;
      p.rows_pad = cur_rpad; p.ws = split_ws; p.ws_bytes = split_ws_bytes;
      p.range_flag = range_flag; p.no_split = enc_f32 ? 1 : 0;
      launch_conv_checked(p, dte, s, prof, 2.0 * D * (double)D * B * Np);
      HIP_CHECK(hipMemcpyAsync(ENC, Y, (size_t)B * Np * D * dtype_size(dte), hipMemcpyDeviceToDevice, s));
    }
    // variance adaptor (HF:1198-1218)
    // HF inference always regulates with the predicted durations (HF:1211-1219); given durations
    // are this engine's override (the oracle's `durations=`), under which the prediction is
    // never read, so the duration predictor does not run
    if (vp_batched && sw(SW_VP_BATCH) != 0) {
      predict_batched(ENC, tok_lens, B, Np, !dur_override, s);
    } else {
      predict(pitch, ENC, tok_lens, B, Np, f_pitch, s);
      predict(energy, ENC, tok_lens, B, Np, f_energy, s);
      if (!dur_override) predict(duration, ENC, tok_lens, B, Np, f_logd, s);
    }
    cur_rpad = 0;
    // logd is laid out [B][Np]; durations kernel reads [B][N] rows -> compact view via stride Np
    int* dur = durations ? durations : i_dur;
    elem(s, [&] { return launch_durations_strided(s, B, N, Np, tok_lens, dur_override, Tcap, dur, mel_lens); });
    elem(s, [&] { return launch_var_embed_add(dte, ENC, B * Np, D, f_energy, ee_w, ee_b, f_pitch, pe_w, pe_b, s); });
    // Decoder extent.  With predicted durations the caller's Tcap is a frame budget (model.py: 12
    // frames per token, retried exactly if exceeded), typically twice the frames the durations
    // give; the decoder then runs at the longest utterance's frame count, read back here (one
    // stream sync, after the variance adaptor is enqueued).  Run at Tcap, every grid doubled with
    // blocks that exit at once: the tile-height and LayerNorm-placement rules saw twice the rows,
    // and a launch whose blocks all fit at once (attention) put two real blocks on some CUs and
    // none on others -- batch-8 acoustic pass 2,061 us at 6 N vs 2,155 us at 12 N
    // (profiles/r05q_tcap_trace.txt).  The read costs ~20-40 us of idle device, so it is made
    // only for a loose budget (Tcap > TTS_DEC_TRIM_RATIO frames per token; a caller passing the
    // frames it expects gets no sync).  A row's result does not depend on the extent
    // (tests/test_acoustic_gpu.py).  TTS_DEC_TRIM=0: never; 1: whatever the budget (tests).
    int Td = Tcap;
    const int trim = sw(SW_DEC_TRIM);
    // a stream being captured into a HIP graph cannot be synchronized: the decoder then runs at
    // Tcap, which the capture records (the same output)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_CHECK(hipStreamIsCapturing(s, &cap));
    if (!dur_override && B > 0 && cap == hipStreamCaptureStatusNone &&
        (trim == 1 || (trim < 0 && Tcap > TTS_DEC_TRIM_RATIO * N))) {
      if (h_lens_n < B) {  // pinned: the copy is a DMA on the stream, not a staged blocking copy
        if (h_lens) HIP_CHECK(hipHostFree(h_lens));
        h_lens = nullptr;
        h_lens_n = 0;
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_lens), (size_t)B * sizeof(int), hipHostMallocDefault));
        h_lens_n = B;
      }
      HIP_CHECK(hipMemcpyAsync(h_lens, mel_lens, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      int mx = 1;
      for (int i = 0; i < B; ++i) mx = std::max(mx, h_lens[i]);
      Td = std::min(Tcap, mx);
    }
    const int Tpd = rup(Td + dec_pad(), 32);  // decoder row stride (dec_pad: at least one pad row)
    // regulate writes the Td frames of each utterance at row stride Tpd (frames past an
    // utterance's length are zero rows)
    void* Xd = X;
    elem(s, [&] { return launch_regulate(dte, dt, ENC, B, Np, D, i_tokmap, Tcap, Td, Tpd, xscale, X, s); });
    // an fp32 model with f32_dec_packed: every split decoder-side GEMM on the packed form (its
    // split-K and fused post-LN), over the pad rows dec_pad keeps after each utterance
    cur_rpad = dec_pad() ? Tpd - Td : 0;
    stack(dec, Xd, mel_lens, B, Td, Tpd, s);
    // postnet (HF:238-244), BatchNorm folded
    run(feat_out, Xd, Tpd, mel_lens, BEF, Tpd, B, dt, s, prof);
    const void* h = BEF;
    void* bufs[2] = {PN1, PN2};
    const int n = (int)postnet.size();
    for (int i = 0; i < n; ++i) {
      const bool last = i == n - 1;
      void* o = last ? MELT : bufs[i & 1];
      run(postnet[i], h, Tpd, mel_lens, o, Tpd, B, dt, s, prof, 1.f, last ? ACT_NONE : ACT_TANH, 1.f,
                last ? BEF : nullptr);
      h = o;
    }
    cur_rpad = 0;
    // MELT rows have stride Tpd; output [B][Tcap][80] float32 (rows past mel_len zero)
    elem(s, [&] { return launch_mel_out(dt, MELT, mel_lens, B, Tpd, Tcap, NMEL, mel, s); });
  }

  hipError_t launch_durations_strided(hipStream_t s, int B, int N, int Np, const int* tok_lens, const int* ovr,
                                      int Tcap, int* dur, int* mel_lens) {
    // compact f_logd [B][Np] -> [B][N] in place is unsafe; copy into PB1 (float view) first
    float* logd = f_logd;
    if (Np != N && !ovr) {  // (with given durations the kernel does not read logd)
      HIP_CHECK(hipMemcpy2DAsync(PB1, (size_t)N * 4, f_logd, (size_t)Np * 4, (size_t)N * 4, B,
                                 hipMemcpyDeviceToDevice, s));
      logd = (float*)PB1;
    }
    return launch_durations(logd, tok_lens, B, N, ovr, 1.0f, Tcap, dur, mel_lens, i_tokmap, s);
  }
};

void AcousticModel::finalize(const GetData& get, const GetShape& shape, int dtype, int enc_dtype, Profiler* prof,
                             bool f32_split_enc) {
  if (!get("encoder.embed.weight")) {
    loaded = false;
    return;
  }
  std::unique_ptr<Impl> m(new Impl());
  m->dt = dtype;
  m->dte = enc_dtype == DT_F32 ? DT_F32 : dtype;
  m->bdt = m->dte;
  m->f32_split_enc = dtype == DT_F32 && f32_split_enc;
  m->f32_split_dec = m->f32_split_enc && sw(SW_F32_DEC_SPLIT) != 0;
  m->f32_dec_packed = m->f32_split_dec && sw(SW_F32_DEC_PACKED) != 0;
  m->enc_side = true;
  m->prof = prof;
  const auto es = shape("encoder.embed.weight");
  m->V = (int)es.at(0);
  m->D = (int)es.at(1);
  m->H = (int)shape("encoder.conformer_layers.0.self_attn.pos_bias_u").at(0);
  m->FFN = (int)shape("encoder.conformer_layers.0.feed_forward.conv1.weight").at(0);
  m->PRED = (int)shape("duration_predictor.conv_layers.0.conv.weight").at(0);
  m->NMEL = (int)shape("speech_decoder_postnet.feat_out.weight").at(0);
  if (m->D % 64 || m->D > 512 || (m->D / m->H) % 16) throw TtsError(TTS_ERR_INVALID, "unsupported hidden size");
  // encoder side (bdt = dte): embedding, encoder layers, speaker projection, variance predictors
  m->embed = m->track(upload(*get("encoder.embed.weight"), m->dte));
  for (int i = 0; get("encoder.conformer_layers." + std::to_string(i) + ".self_attn.pos_bias_u"); ++i)
    m->enc.push_back(m->layer(get, shape, "encoder.conformer_layers." + std::to_string(i) + "."));
  m->pitch = m->predictor(get, shape, "pitch_predictor.");
  m->energy = m->predictor(get, shape, "energy_predictor.");
  m->duration = m->predictor(get, shape, "duration_predictor.");
  m->batch_predictors(get, shape);
  if (get("projection.weight")) {
    const auto ps = shape("projection.weight");  // [D][D + E]
    const int din = (int)ps.at(1);
    if ((int)ps.at(0) != m->D || din <= m->D) throw TtsError(TTS_ERR_INVALID, "bad projection.weight shape");
    m->E = din - m->D;
    const auto& pw = m->need(get, "projection.weight");
    std::vector<float> wh((size_t)m->D * m->D), we((size_t)m->D * m->E);
    for (int o = 0; o < m->D; ++o) {
      for (int i = 0; i < m->D; ++i) wh[(size_t)o * m->D + i] = pw[(size_t)o * din + i];
      for (int i = 0; i < m->E; ++i) we[(size_t)o * m->E + i] = pw[(size_t)o * din + m->D + i];
    }
    m->proj_h = make_conv(wh, m->D, m->D, 1, {}, 1, 0, m->dte, m->allocs, nullptr, m->split_now());
    m->proj_we = m->upf(we);
    m->proj_b = m->upf(m->need(get, "projection.bias"));
  }
  m->pe_w = m->upf(m->need(get, "pitch_embed.conv.weight"));
  m->pe_b = m->upf(m->need(get, "pitch_embed.conv.bias"));
  m->ee_w = m->upf(m->need(get, "energy_embed.conv.weight"));
  m->ee_b = m->upf(m->need(get, "energy_embed.conv.bias"));
  // decoder side (bdt = dt): decoder layers, postnet
  m->bdt = dtype;
  m->enc_side = false;
  for (int i = 0; get("decoder.conformer_layers." + std::to_string(i) + ".self_attn.pos_bias_u"); ++i)
    m->dec.push_back(m->layer(get, shape, "decoder.conformer_layers." + std::to_string(i) + "."));
  m->feat_out = m->conv(get, shape, "speech_decoder_postnet.feat_out.weight", "speech_decoder_postnet.feat_out.bias", 0);
  for (int i = 0;; ++i) {
    const std::string p = "speech_decoder_postnet.layers." + std::to_string(i) + ".";
    if (!get(p + "conv.weight")) break;
    const auto s = shape(p + "conv.weight");
    const int co = (int)s.at(0), k = (int)s.at(2);
    const auto& g = m->need(get, p + "batch_norm.weight");
    const auto& be = m->need(get, p + "batch_norm.bias");
    const auto& rm = m->need(get, p + "batch_norm.running_mean");
    const auto& rv = m->need(get, p + "batch_norm.running_var");
    std::vector<float> sc(co), bb(co);
    for (int o = 0; o < co; ++o) {
      sc[o] = g[o] / std::sqrt(rv[o] + m->eps);
      bb[o] = be[o] - rm[o] * sc[o];  // conv has no bias
    }
    m->postnet.push_back(m->conv(get, shape, p + "conv.weight", "", (k - 1) / 2, &sc, &bb));
  }
  m->build_ptabs(1024, nullptr);
  {
    void* f = nullptr;
    HIP_CHECK(dev_malloc(&f, 16));
    HIP_CHECK(hipMemset(f, 0, 16));
    m->range_flag = (int*)m->track(f);
  }
  impl = m.release();
  loaded = true;
}

void AcousticModel::reserve(int B, int N, int T) {
  if (impl) impl->reserve(B, N, T);
}

void AcousticModel::forward(const int32_t* tokens, const int32_t* tok_lens, int B, int N, const int32_t* dur_override,
                            float* mel, int32_t* mel_lens, int Tcap, int32_t* durations, const float* spk,
                            hipStream_t s) {
  if (!impl) throw TtsError(TTS_ERR_STATE, "acoustic model not loaded");
  impl->forward(tokens, tok_lens, B, N, dur_override, mel, mel_lens, Tcap, durations, spk, s);
}

int AcousticModel::speaker_dim() const { return impl ? impl->E : 0; }

bool AcousticModel::split_encoder() const { return impl && impl->split_enc(); }

void AcousticModel::set_encoder_f32(bool on) {
  if (!impl) throw TtsError(TTS_ERR_STATE, "acoustic model not loaded");
  impl->enc_f32 = on;
}

bool AcousticModel::encoder_f32() const { return impl && impl->enc_f32; }

void AcousticModel::range_flag_to(int32_t* dst, hipStream_t s) {
  if (!impl) throw TtsError(TTS_ERR_STATE, "acoustic model not loaded");
  // device (or managed) destination: one small kernel copies and clears the word; host memory:
  // an async copy and a fill
  hipPointerAttribute_t at{};
  const bool dev = hipPointerGetAttributes(&at, dst) == hipSuccess &&
                   (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged);
  if (!dev) (void)hipGetLastError();  // (a plain host pointer reports an error: cleared)
  if (dev) {
    HIP_CHECK(launch_range_take(impl->range_flag, dst, s));
  } else {
    HIP_CHECK(hipMemcpyAsync(dst, impl->range_flag, 4, hipMemcpyDefault, s));
    HIP_CHECK(hipMemsetAsync(impl->range_flag, 0, 4, s));
  }
}

void AcousticModel::free_all() {
  delete impl;
  impl = nullptr;
  loaded = false;
}

}  // namespace tts
