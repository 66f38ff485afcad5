// FastSpeech2-Conformer acoustic model runtime (acoustic.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

namespace tts {

struct Profiler;

struct AcousticModel {
  bool loaded = false;
  typedef std::function<const std::vector<float>*(const std::string&)> GetData;
  typedef std::function<std::vector<int64_t>(const std::string&)> GetShape;
  // dtype: decoder / postnet activations; enc_dtype: encoder, speaker projection and variance
  // predictors (DT_F32 with a 16-bit dtype = split-precision GEMMs, TTS_ENCODER_EXACT);
  // f32_split_enc: an fp32 model's encoder side on the same split-precision GEMMs and attention
  // (TTS_ENCODER_EXACT with acoustic_dtype F32; its decoder and postnet stay on fp32 MFMA)
  void finalize(const GetData& get, const GetShape& shape, int dtype, int enc_dtype, Profiler* prof,
                bool f32_split_enc = false);
  void reserve(int B, int N, int T);
  // spk: optional [B][speaker_dim()] fp32 speaker embeddings (ignored when the model has none)
  void forward(const int32_t* tokens, const int32_t* tok_lens, int B, int N, const int32_t* dur_override,
               float* mel, int32_t* mel_lens, int Tcap, int32_t* durations, const float* spk, hipStream_t s);
  int speaker_dim() const;
  // encoder side on split-precision GEMMs and attention (a 16-bit model's exact encoder, or an
  // fp32 model's with f32_split_enc)
  bool split_encoder() const;
  // run that encoder on the exact fp32 MFMA kernels instead (the range guard's fallback)
  void set_encoder_f32(bool on);
  bool encoder_f32() const;
  // enqueue on s: copy the range-guard word (1 = a split operand was outside f16's range since the
  // last call) to dst (device or host-pinned), then clear it
  void range_flag_to(int32_t* dst, hipStream_t s);
  void free_all();
  struct Impl;
  Impl* impl = nullptr;
};

}  // namespace tts
