/*
 * tts_hip.h — C-ABI of libtts_hip.so, the MI355X (gfx950) batched TTS engine.
 *
 * The reference has no C-ABI: its only model boundary is duck-typed Python
 * (SURVEY.md §8b).  Each entry point below replaces one step of that boundary:
 *
 *   tts_engine_create / tts_engine_set_weight / tts_engine_finalize
 *       replace `ChatterboxTTS.from_pretrained(device=self.device)`
 *       (/root/reference/services/tts/core/synthesizer.py:185; device string from
 *       synthesizer.py:130, "cuda:0" from server.py:400-405).  The Python host maps
 *       "cuda:N" to HIP device N and feeds weights by HF state_dict name.
 *   tts_acoustic_forward + tts_vocoder_forward
 *       replace `self.model.generate(text, audio_prompt_path=..., exaggeration=...,
 *       cfg_weight=0.5, temperature=0.8)` (synthesizer.py:344-350) for a whole
 *       batch of sentences at once (tokens -> mel -> waveform).
 *   tts_vocoder_forward_chunk
 *       sub-sentence streaming the reference lacks (synthesizer.py:320-321 yields
 *       one chunk per sentence); exact receptive-field context.
 *   tts_last_error
 *       replaces Python exception text: the host raises RuntimeError(tts_last_error())
 *       so the reference's exception path (synthesizer.py:323-325, 291-294) holds.
 *
 * Conventions
 *   - Every device buffer passed in is caller-owned (PyTorch-ROCm tensors passed by
 *     data_ptr()).  The engine owns its weights and workspace.
 *   - Work is enqueued asynchronously on `stream` (a hipStream_t; NULL = default).
 *   - Return 0 on success, a negative TTS_ERR_* on failure; no C++ exception crosses
 *     the ABI.  Every entry sets the HIP device and takes a per-engine mutex, so any
 *     host thread may call (the reference calls from a ThreadPoolExecutor,
 *     synthesizer.py:312).  The engine's workspace is shared by all calls: a forward
 *     enqueued on a stream other than the previous call's is made to wait (event edge)
 *     for everything the previous call's stream had enqueued, so calls from different
 *     threads / streams run one after another on the device, never interleaved.
 *   - Activations are channels-last: mel [B][T][80] float32 (HF spectrogram layout),
 *     waveform [B][T*256] float32 at 22,050 Hz.  Compute dtype per stage is chosen
 *     at create time; accumulation is always fp32.
 */
#ifndef TTS_HIP_H
#define TTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TTS_OK 0
#define TTS_ERR_INVALID (-1)
#define TTS_ERR_HIP (-2)
#define TTS_ERR_STATE (-3)
#define TTS_ERR_NOMEM (-4)

enum { TTS_DTYPE_F32 = 0, TTS_DTYPE_F16 = 1, TTS_DTYPE_BF16 = 2 };

typedef struct tts_engine tts_engine;

/* ABI history (INTEGRATION.md "Changelog"):
 *   1  tts_config of five ints (no encoder_precision)
 *   2  tts_config gains encoder_precision (sixth int)
 *   3  tts_engine_create_sized / tts_abi_version / tts_get_switch; stream ordering records
 *      on the caller's stream at the end of each call (a caller may destroy its stream after
 *      the call returns)
 *   4  range guard of the exact encoder: tts_acoustic_range_flag / tts_acoustic_set_precision,
 *      TTS_ENCODER_F32
 *   5  tts_device_bytes (the library's device memory per HIP device); additive */
#define TTS_ABI_VERSION 5
int tts_abi_version(void);

/* Engine configuration.  Fields are only ever appended; a caller built against an older
 * header passes its struct's size to tts_engine_create_sized and the fields past it keep
 * their zero defaults. */
typedef struct tts_config {
  int vocoder_dtype;   /* TTS_DTYPE_*: compute/storage dtype of vocoder activations */
  int acoustic_dtype;  /* TTS_DTYPE_*: compute/storage dtype of acoustic activations */
  int max_batch;       /* workspace reservation hints (0 = grow on demand) */
  int max_frames;
  int max_tokens;
  int encoder_precision; /* TTS_ENCODER_*: precision of the acoustic encoder + variance predictors */
} tts_config;

/* Acoustic encoder precision.  EXACT (the default, 0): with a 16-bit acoustic_dtype the encoder,
 * speaker projection and variance predictors keep fp32 activations and run their GEMMs as three
 * f16 MFMAs (~2^-21 relative per product), so the predicted integer durations
 * clamp(round(exp(x) - 1), 0) (HF:181-183) match an fp32 evaluation; the decoder and postnet run in
 * acoustic_dtype.  FAST (1): the whole acoustic model runs in acoustic_dtype (durations can
 * round differently near .5).  With acoustic_dtype = F32, EXACT runs the encoder side on the same
 * split-precision GEMMs and attention, and the decoder / postnet GEMMs on the split-precision
 * GEMMs too (round 6; the decoder attention stays on the fp32 kernel; its row stride keeps two
 * pad rows per utterance), and
 * FAST keeps every layer on fp32 MFMA (switch TTS_F32_ENC_SPLIT=0 at finalize: the same). */
enum { TTS_ENCODER_EXACT = 0, TTS_ENCODER_FAST = 1, TTS_ENCODER_F32 = 2 };
/* Range limit of EXACT: its split GEMMs and attention hold every fp32 operand as two f16 halves,
 * so activations must stay below 65504 in magnitude (f16 max); weights are stored at a
 * power-of-two scale per layer (round 6), so any finite weights are taken.  Activations are
 * checked on the device (ABI 4): every split GEMM and the split attention test the f16 high half
 * of each operand they stage and, when one is inf or NaN (|x| >= 65520, or a NaN input), set the
 * engine's range word.  The forward itself stays asynchronous; the caller reads the word with
 * tts_acoustic_range_flag after its next sync and, when it is set, reruns the acoustic forward
 * with TTS_ENCODER_F32 (the same fp32 layers on the exact fp32 MFMA kernels, ~3x slower on the
 * encoder side, no range limit).  TTS_ENCODER_F32 is a run-time setting only
 * (tts_acoustic_set_precision), not a tts_config value. */

/* fp32 vocoders (vocoder_dtype = TTS_DTYPE_F32): the resblock convs of every stage (channel counts
 * divisible by 32, >= 32) run as split-precision GEMMs (three f16 MFMAs per product, ~2^-21 relative, like the exact
 * encoder).  tts_vocoder_forward / _chunk then read the layers' range word once at the end of the
 * call (one sync of `stream`) and, if an activation left f16's range, rerun the forward with every
 * layer on the fp32 MFMA path; 16-bit vocoders are unaffected and stay asynchronous. */

/* Number of HIP devices visible to this process. */
int tts_device_count(void);

/* Device memory this library holds on HIP device `hip_device` (every engine's weights and
 * workspaces, in bytes) -> *bytes.  The reference's /health reports torch's allocator
 * (server.py:456-465: memory_allocated / memory_reserved), which never sees these buffers;
 * the service adds this figure to its "gpu" report.  Needs no GPU work (a host-side count). */
int tts_device_bytes(int hip_device, int64_t* bytes);

/* Engine lifetime (replaces ChatterboxTTS.from_pretrained, synthesizer.py:185).
 * tts_engine_create reads a whole tts_config of THIS header; tts_engine_create_sized reads
 * cfg_size bytes of it (sizeof(tts_config) of the caller's header; smaller = an older layout,
 * the missing fields zero; larger than this library's struct = TTS_ERR_INVALID). */
int tts_engine_create(int hip_device, const tts_config* cfg, tts_engine** out);
int tts_engine_create_sized(int hip_device, const tts_config* cfg, size_t cfg_size, tts_engine** out);
/* Host fp32 tensor in HF state_dict naming (e.g. "resblocks.3.convs1.2.weight"). */
int tts_engine_set_weight(tts_engine* eng, const char* name, const float* host_data,
                          const int64_t* shape, int ndim);
/* Fold / pack / upload every weight set so far; must precede any forward. */
int tts_engine_finalize(tts_engine* eng);
/* Pre-size the workspace (so later calls allocate nothing and can be graph-captured). */
int tts_engine_reserve(tts_engine* eng, int max_batch, int max_frames, int max_tokens);
void tts_engine_destroy(tts_engine* eng);

/* Vocoder (replaces the waveform half of model.generate, synthesizer.py:344).
 *   d_mel      [B][T][80] float32, utterance b valid for d_mel_lens[b] <= T frames
 *   d_wav      [B][T*256] float32; samples >= 256*d_mel_lens[b] are written as 0.   */
int tts_vocoder_forward(tts_engine* eng, const float* d_mel, const int32_t* d_mel_lens, int B,
                        int T, float* d_wav, void* stream);

/* Streaming vocoder chunk with exact context: computes the waveform of frames
 * [ctx_left, ctx_left + T_chunk) of each d_mel[b] window [ctx_left + T_chunk + ctx_right][80]
 * (zero context at utterance edges is expressed by the caller passing shorter windows via
 * d_win_lens).  d_wav [B][T_chunk*256]. */
int tts_vocoder_forward_chunk(tts_engine* eng, const float* d_mel, const int32_t* d_win_lens,
                              int B, int T_win, int ctx_left, int T_chunk, float* d_wav,
                              void* stream);

/* Acoustic model (replaces the text->spectrogram half of model.generate).
 *   d_tokens      [B][N] int32 token ids (padding ignored past d_tok_lens[b])
 *   d_dur_override optional [B][N] int32 frame counts (NULL = predicted durations; when given,
 *                  the duration predictor is not run and d_durations returns these counts)
 *   d_mel         [B][Tcap][80] float32 output, d_mel_lens [B] int32 output
 *   d_durations   optional [B][N] int32 output of the durations actually used
 * Frames past Tcap are dropped (d_mel_lens is clamped to Tcap).  With predicted durations and a
 * loose budget (Tcap > 8 N) the call reads the frame counts back once after the variance adaptor
 * (the calling thread waits for the encoder on `stream`) and runs the decoder at the longest
 * utterance's count instead of Tcap; the output is the same (TTS_DEC_TRIM=0: never, 1: at any
 * budget).  Otherwise, and with d_dur_override, the call stays fully asynchronous. */
int tts_acoustic_forward(tts_engine* eng, const int32_t* d_tokens, const int32_t* d_tok_lens,
                         int B, int N, const int32_t* d_dur_override, float* d_mel,
                         int32_t* d_mel_lens, int Tcap, int32_t* d_durations, void* stream);

/* The same with per-utterance speaker embeddings (HF:1192-1196):
 * d_spk_emb [B][spk_dim] fp32 on the device, spk_dim == tts_acoustic_speaker_dim(); each is
 * L2-normalised, concatenated to every encoder frame and projected back to the hidden size.
 * NULL (or a model without a speaker projection) = tts_acoustic_forward. */
int tts_acoustic_forward_spk(tts_engine* eng, const int32_t* d_tokens, const int32_t* d_tok_lens,
                             int B, int N, const int32_t* d_dur_override, const float* d_spk_emb,
                             int spk_dim, float* d_mel, int32_t* d_mel_lens, int Tcap,
                             int32_t* d_durations, void* stream);
/* Speaker-embedding size E of the loaded acoustic model (0: single speaker). */
int tts_acoustic_speaker_dim(tts_engine* eng, int* dim);

/* Range guard (ABI 4, TTS_ENCODER_EXACT above): enqueue on `stream` a copy of the engine's
 * range word into *dst (device or host-pinned int32; 1 = some split-precision operand of an
 * acoustic forward enqueued before this call was outside f16's range, 0 = none), then clear the
 * word.  Read *dst after synchronising the stream. */
int tts_acoustic_range_flag(tts_engine* eng, int32_t* dst, void* stream);
/* Encoder precision of later acoustic forwards of a 16-bit model created with EXACT:
 * TTS_ENCODER_EXACT (split-precision, the default) or TTS_ENCODER_F32 (exact fp32 MFMA: the
 * range guard's fallback).  Other models: TTS_ERR_INVALID. */
int tts_acoustic_set_precision(tts_engine* eng, int precision);

/* Live kernel timing for bench.py: with profiling on, every implicit-GEMM launch is
 * bracketed by hipEvents on its own stream; _read() waits for them and returns the summed
 * kernel time (ms), the algorithmic FLOPs of those launches and their count, then resets. */
int tts_engine_profile(tts_engine* eng, int enable);
int tts_engine_profile_read(tts_engine* eng, double* gemm_ms, double* gemm_flops, int* n_launches);
/* The same, split by kernel family into arrays of nkinds entries:
 * 0 = conv_gemm_kernel, 1 = conv_xres_kernel, 2 = (retired: round 1's whole-stage kernel), 3 = mrf_pair_kernel,
 * 4 = mrf_chain_kernel, 5 = upsample_stream_kernel, 6 = conv_split_kernel, 7 = the fused relative-position
 * attention (FLOPs 6*D*B*Tm^2: scores, relative-position scores and P.V at the padded extent), 8 = the
 * acoustic model's other launches (LayerNorm, GLU/depthwise, transposes, variance adaptor; no FLOPs). */
int tts_engine_profile_read_kinds(tts_engine* eng, int nkinds, double* ms, double* flops, int* n_launches);

/* Process-wide switch selecting an alternative kernel path (A/B runs, the parity tests'
 * reference paths): TTS_REL_ATTN, TTS_MRF_FUSED, TTS_MRF_CHAIN, TTS_POST_FUSE, TTS_UP_STREAM,
 * TTS_XRES_NARROW, TTS_XRES_NT, TTS_PAIR_DIV, TTS_ATTN_KSPLIT, TTS_SPLIT_WHOLE, TTS_XRES_DMA,
 * TTS_LN_FUSE, TTS_SPLIT_NT1, TTS_XRES_ORDER, TTS_PAIR_SPLIT, TTS_VP_BATCH, TTS_DEC_TRIM,
 * TTS_ATTN_F32_KC, TTS_F32_ENC_SPLIT, TTS_F32_DEC_SPLIT, TTS_F32_DEC_PACKED.  Each starts from its environment variable, read once; value -1 restores the built-in default.
 * Applies to launches enqueued after the call (use from one thread while no forward runs). */
int tts_set_switch(const char* name, int value);
/* Current value of a switch (-1 = not set), so a caller can restore what it changed. */
int tts_get_switch(const char* name, int* value);

/* Rational-rate resampling of waveforms (22,050 -> 24,000 Hz for
 * clients that assume the reference's hard-coded 24 kHz, synthesizer.py:119 /
 * queue_manager.py:40).  Restates scipy.signal.resample_poly(x, up, down) with its default
 * Kaiser(5.0) FIR and zero padding, per utterance: d_in [B][in_stride] fp32 with d_in_lens[b]
 * valid samples -> d_out [B][out_stride], d_out_lens[b] = min(ceil(len*up/down), out_cap);
 * samples past each length (up to out_cap) are written as 0.  up/down are reduced by their gcd. */
int tts_resample_poly(tts_engine* eng, const float* d_in, int64_t in_stride, const int32_t* d_in_lens, int B,
                      int up, int down, float* d_out, int64_t out_stride, int out_cap, int32_t* d_out_lens,
                      void* stream);
/* Host only: the padded filter taps tts_resample_poly uses (float64, scaled by up); returns the
 * tap count (h filled only when cap >= it), *n_pre_remove = leading outputs scipy discards. */
int tts_resample_filter(int up, int down, double* h, int cap, int* n_pre_remove);

/* Thread-local message describing the last failure on this thread. */
const char* tts_last_error(void);

/* ---- op-level entry used by the parity tests (one implicit-GEMM conv launch) ---- */
typedef struct tts_conv_desc {
  const void* x; int64_t sxb; int32_t sxr; const int32_t* x_len; int32_t x_rows;
  const void* w; int64_t swb; int32_t w_ld;
  const float* bias;
  void* y; int64_t syb; int32_t syr;
  const void* r1; const void* r2; int64_t srb; int32_t srr;
  const int32_t* y_len; int32_t y_rows;
  int32_t M, Cin, taps, dil, pad;
  float in_slope; int32_t act_out; float out_slope; float alpha; float out_scale;
  int32_t up_s, up_cout, up_p; const int32_t* up_len;
  int32_t B;
} tts_conv_desc;

int tts_op_conv1d(int dtype, const tts_conv_desc* desc, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TTS_HIP_H */
