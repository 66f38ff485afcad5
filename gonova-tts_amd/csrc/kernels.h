// Host-side declarations of the HIP kernel launchers (internal to libtts_hip.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace tts {

// Implicit-GEMM conv (conv_gemm.hip).  All strides are in elements of the compute dtype.
struct ConvParams {
  const void* x; long long sxb; int sxr; const int* x_len; int x_rows;
  const void* w; long long swb; int w_ld;
  const float* bias;
  void* y; long long syb; int syr;
  const void* r1; const void* r2; long long srb; int srr;
  const int* y_len; int y_rows;
  int M, Cin, taps, dil, pad;
  float in_slope;          // leaky-relu slope applied to X on load; 1 = identity
  int act_out; float out_slope;
  float alpha, out_scale;  // y = ((alpha*(acc+bias)) -> act) + r1 + r2, then * out_scale
  int up_s, up_cout, up_p; const int* up_len;  // transposed-conv output mapping (up_s = 0: off)
  int B;
  // optional head batching: grid z = B * nh, z -> (b = z / nh, h = z % nh); every pointer is
  // offset by b * s?b + h * s?h (lengths are indexed by b)
  int nh; long long sxh, swh, syh, srh;
  // optional fragment-packed copy of w (frag_pack in runtime.h): enables the X-resident
  // kernel, whose weight loads are then contiguous 1 KiB wave reads
  const void* wpk;
  // split-packed weights (frag_pack_split) are stored scaled by a power of two; the split GEMMs
  // multiply their sums by w_unscale (exact).  1 for every other packing.
  float w_unscale;
  // Packed-row hint (split-precision fp32 GEMMs, conv_split.hip): rows_pad > 0 promises that every
  // utterance is followed by at least rows_pad masked rows (x_rows - len[b] >= rows_pad, X / Y /
  // residuals contiguous [B][x_rows][C]), so row tiles may run across utterance boundaries; the
  // optional split-K workspace ws (ws_bytes) holds fp32 partial sums.
  int rows_pad;
  float* ws;
  long long ws_bytes;
  // optional LayerNorm of the result (post-LN residual blocks, HF:551-645): ln_out[row] =
  // LN2?(LN1(y[row])) with y's strides.  The split-K fp32 path applies it in its reduce
  // (split_reduce_ln_kernel: y is never written); with ln_cnt (below) the conv_xres and one-slice
  // conv_splitp launches apply it in their epilogue; every other path writes y and then runs
  // launch_layernorm(y -> ln_out) over the rows inside each utterance's length (y_len).
  void* ln_out;
  const float *ln_g1, *ln_b1, *ln_g2, *ln_b2;
  float ln_eps;
  // Row-tile counters (ln_cnt_n ints, zero; ln_rows.h): with them the X-resident (16-bit) and
  // packed split-precision (fp32, one K slice) kernels apply the LayerNorm in the launch itself
  // (the last-arriving M block of each row tile normalises its rows; rows past an utterance's
  // length are left alone).  ln_lin_out: LN(y) . ln_lin_w + ln_lin_b per row instead of ln_out
  // (the variance predictors' LayerNorm + Linear(C -> 1)).
  int* ln_cnt;
  int ln_cnt_n;
  const float* ln_lin_w;
  float ln_lin_b;
  float* ln_lin_out;
  // Range guard of the split-precision fp32 GEMMs (conv_split.hip): a staged operand outside f16's
  // range (|x| >= 65520 or NaN) ORs 1 into *range_flag (nullable).  no_split: run an fp32 conv on
  // the exact fp32 MFMA path (conv_gemm_kernel<float>) even where the split form is eligible --
  // the fallback of the exact encoder when its range guard tripped (tts_acoustic_set_precision).
  int* range_flag;
  int no_split;
  // conv_xres block order (launcher-set): 0 = the 3-D grid as dispatched (row tile fastest);
  // 1 = a 1-D grid padded to a multiple of 8, block L -> work item (L % 8) * per + L / 8 (each XCD
  // a contiguous range of items), items ordered M block fastest, so the M blocks of a row tile run
  // on one XCD together and share its X tile through that L2
  int xres_order;
  // Split-K of the fp32 conv_gemm_kernel, at every batch size (it was built for C1's batch-1 FFN
  // convs, which ran on 3-12 blocks; measured at batch 8 / 32 and kept, capped at 16 slices:
  // profiles/r06c/).  f32_splitk (caller): the launch may split its K
  // (Cin chunks) into f32_kslices(taps, Cin) slices -- a count from the layer shape only, so a row's
  // summation order does not depend on the batch -- writing fp32 partials to ws[S][B][y_rows][M],
  // which split_reduce_launch sums in slice order and finishes with conv_epilogue's arithmetic.
  // kslices: set by the launcher for the kernel (0 / 1: no split).
  int f32_splitk;
  int kslices;
};

inline ConvParams conv_params_default() {
  ConvParams p{};
  p.in_slope = 1.f; p.alpha = 1.f; p.out_scale = 1.f; p.out_slope = 0.f;
  p.taps = 1; p.dil = 1; p.nh = 1;
  p.w_unscale = 1.f;
  return p;
}

int conv_gemm_check(const ConvParams& p, int dtype, const char** why);
hipError_t conv_gemm_launch(int dtype, const ConvParams& p, hipStream_t s);
// kernels the calling thread's last conv_gemm_launch enqueued (the GEMM, a split-K reduce, a LayerNorm)
int conv_last_kernels();

// kernel family a launch runs as (live profiling buckets; tts_engine_profile_read_kinds)
enum ProfKind : int { PK_CONV_GEMM = 0, PK_CONV_XRES = 1, PK_RETIRED = 2 /* mrf_fused, removed */, PK_MRF_PAIR = 3, PK_MRF_CHAIN = 4, PK_UPSAMPLE = 5,
                      PK_CONV_SPLIT = 6, PK_ATTN = 7 /* fused relative-position attention */,
                      PK_AC_ELEM = 8 /* the acoustic model's non-GEMM launches: LN, GLU/depthwise, transposes, adaptor */,
                      PK_N = 9 };
int conv_gemm_kind(int dtype, const ConvParams& p);


// fp32 conv as three f16 MFMAs (conv_split.hip): an fp32 layer whose ConvParams::wpk is a
// split-packed copy (frag_pack_split) runs here when eligible (Cin % 64 == 0, no head batching)
bool conv_split_eligible(const ConvParams& p);
// *ln_done: whether the launch applied p.ln_out's LayerNorm itself (the split-K reduce)
hipError_t conv_split_launch(const ConvParams& p, hipStream_t s, bool* ln_done = nullptr);
int conv_split_last_kernels();  // kernels the calling thread's last conv_split_launch enqueued
// split-K workspace bytes a packed-row launch of this shape over `rows` flat rows can use (0: none)
long long conv_split_ws_bytes(int taps, int Cin, int M, int rows);
// fp32 split-K (ConvParams::f32_splitk): slices of a layer, the partials' bytes over `rows` (B * y_rows)
// output rows, and the reduce (p.x_rows = the partials' rows per utterance; LayerNorm fused when
// p asks for one the reduce can apply: *ln_done)
int f32_kslices(int taps, int Cin);
long long f32_splitk_ws_bytes(int taps, int Cin, int M, long long rows);
hipError_t split_reduce_launch(const ConvParams& p, int S, hipStream_t s, bool* ln_done);

// Fused ResBlock pair (mrf_pair.hip): t = lrelu(conv_{k,d}(lrelu(h)) + b1);
// h' = conv_{k,1}(t) + b2 + h;  y = ((accum ? y : 0) + h') * scale.
struct MrfPairParams {
  const void* x;      // [B][T][C] pair input h, compute dtype
  void* y;            // [B][T][C] h' (accum = 0) or the MRF sum S (accum = 1); never aliases x
  const int* len;     // per-utterance valid rows
  const void* w1;     // conv1 / conv2 weights, 16x16 fragment-packed (frag_pack16)
  const void* w2;
  const float* b1;    // fp32 [C]
  const float* b2;
  int T, B, k, d;
  float slope, scale;
  int accum;
  // conv_post fused into the last pair of the vocoder (post_wpk != null; C = 32): the final
  // MRF sum never leaves the block, wav[b][t] = tanh(post_b + conv_post(lrelu(S, post_slope)))
  // is written instead of y (zero for len <= t < T).  Bit-identical to launch_conv_post.
  const void* post_wpk;  // [post_k][C/2] packed 16-bit pairs (the 16-bit conv_post layout)
  float post_b, post_slope;
  int post_k;
  float* wav;
  long long swb;
  // out_act: the stored rows are LeakyReLU(out_slope) of h' / S (rounded to T first) -- the
  // activation the next upsampler would apply on load, so a stage's last pair hands it lrelu(S)
  int out_act;
  float out_slope;
  // optional [B][T][C] scratch (compute dtype): with it, launches whose full-height grid is small
  // (the streamed vocoder's first chunk) run the channel-split form (mrf_pair.hip), bit-identical
  void* tbuf;
};
bool mrf_pair_supported(int dtype, int C, int k);
bool mrf_pair_outact_supported(int dtype, int C, int k);  // the launch can carry out_act

// Streaming ConvTranspose1d with two taps (k = 2s) for the small upsamplers (upsample.hip):
// x [B][T][Cin] (len[b] valid rows) -> y [B][T*s][Co], rows s*u + r - pad for u = 0 .. len,
// r < s, clipped to [0, up_len[b]); weights packed as [M/16][2*Cin/32][64][8] (M = s*Co,
// K = tap*Cin + ci), LeakyReLU(slope) on the input.
struct UpsampleParams {
  const void* x;
  long long sxb, syb;
  const int* len;
  const int* up_len;
  const void* wpk;
  const float* bias;  // fp32 [M]
  void* y;
  int T, B, s, co, pad;
  float slope;
};
bool upsample_stream_supported(int dtype, int Cin, int M, int taps);
hipError_t upsample_stream_launch(int dtype, int Cin, int M, const UpsampleParams& p, hipStream_t s);
// the pair launch can carry conv_post (C, k and post_k it was compiled for)
bool mrf_pair_post_supported(int dtype, int C, int post_k);
hipError_t mrf_pair_launch(int dtype, int C, const MrfPairParams& p, hipStream_t s);

// Fused resblock (mrf_chain.hip): the three pairs of one resblock (dilations 1, 3, 5) in one
// launch; y = ((accum ? y : 0) + resblock(x)) * scale.  Bit-identical to three pair launches.
struct MrfChainParams {
  const void* x;          // [B][T][C] resblock input, compute dtype
  void* y;                // [B][T][C] MRF sum S; never aliases x
  const int* len;
  const void* w1[3];      // per pair: conv1 / conv2 weights, frag_pack16
  const void* w2[3];
  const float* b1[3];
  const float* b2[3];
  int T, B;
  float slope, scale;
  int accum;
};
bool mrf_chain_supported(int dtype, int C, int k, const int* dil, int npair);
hipError_t mrf_chain_launch(int dtype, int C, int k, const MrfChainParams& p, hipStream_t s);

// resample.hip: scipy.signal.resample_poly's default filter (padded taps, n_pre_remove)
int resample_design(int up, int down, std::vector<double>& h, int& n_pre_remove);
hipError_t launch_resample_poly(const float* x, long long sxb, const int* in_lens, int B, int up, int down, int nq,
                                int n_pre_remove, const float* hp, float* y, long long syb, int y_cap,
                                int* out_lens, hipStream_t s);

// elementwise.hip
hipError_t launch_mel_in(int dtype, const float* mel, long long smb, int smr, const float* mean,
                         const float* scale, void* out, int B, int T, int C, hipStream_t s);
hipError_t launch_lens(const int* in, int* out, int B, const int* mult, const int* add, int n,
                       hipStream_t s);
// wpk (optional, 16-bit dtypes): the same weights [k][C] in the compute dtype -> dot2 kernel
hipError_t launch_conv_post(int dtype, const void* x, const int* x_len, int B, int T, int C,
                            const float* w /*[k][C]*/, const void* wpk, float bias, int k, float in_slope,
                            float* wav, long long swb, hipStream_t s);

}  // namespace tts
