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
  // predictors (DT_F32 with a 16-bit dtype = split-precision GEMMs, TTS_ENCODER_EXACT)
  void finalize(const GetData& get, const GetShape& shape, int dtype, int enc_dtype, Profiler* prof);
  void reserve(int B, int N, int T);
  // spk: optional [B][speaker_dim()] fp32 speaker embeddings (ignored when the model has none)
  void forward(const int32_t* tokens, const int32_t* tok_lens, int B, int N, const int32_t* dur_override,
               float* mel, int32_t* mel_lens, int Tcap, int32_t* durations, const float* spk, hipStream_t s);
  int speaker_dim() const;
  void free_all();
  struct Impl;
  Impl* impl = nullptr;
};

}  // namespace tts
