// Runtime switches selecting alternative kernel paths (A/B runs and the parity tests' reference
// paths).  Each is read from its TTS_* environment variable once, on first use, and can be set
// at run time through tts_set_switch (include/tts_hip.h); nothing on the forward path calls
// getenv.  -1 = not set: the path's built-in default.
#pragma once

namespace tts {

enum Sw : int {
  SW_REL_ATTN,     // TTS_REL_ATTN=0: unfused four-launch attention (16-bit)
  SW_MRF_FUSED,    // TTS_MRF_FUSED=0: the per-conv MRF path
  SW_MRF_CHAIN,    // TTS_MRF_CHAIN=0/1: resblock chain kernel off / on
  SW_POST_FUSE,    // TTS_POST_FUSE=0: conv_post as its own launch
  SW_UP_STREAM,    // TTS_UP_STREAM=0: stages 2-3 upsamplers on conv_xres
  SW_XRES_NARROW,  // TTS_XRES_NARROW=0/1: force conv_xres narrow tiles off / on
  SW_XRES_NT,      // TTS_XRES_NT=2/4: force conv_xres tile height
  SW_PAIR_DIV,     // TTS_PAIR_DIV=1: full-height pair tiles; any other value: short tiles
  SW_ATTN_KSPLIT,  // TTS_ATTN_KSPLIT=1: 16-bit attention with two key groups per block (8 waves)
  SW_SPLIT_WHOLE,  // TTS_SPLIT_WHOLE=0: small split-precision GEMMs stage one channel group at a time
  SW_XRES_DMA,     // TTS_XRES_DMA=0: FFN convs / upsamplers register-staged with round-2 channel groups; 2: register-staged, same bits
  SW_LN_FUSE,      // TTS_LN_FUSE=0: acoustic post-LNs as their own launches; 7: in every eligible GEMM launch (2-6: bisection)
  SW_SPLIT_NT1,    // TTS_SPLIT_NT1=0: split GEMMs always on 64-row tiles; 1: 32-row tiles wherever eligible (default: small grids)
  SW_XRES_ORDER,   // TTS_XRES_ORDER=1: multi-tap DMA conv_xres launches on an XCD-ordered grid (M block fastest); 2: every conv_xres launch
  SW_PAIR_SPLIT,   // TTS_PAIR_SPLIT=0/1: the channel-split pair form never / wherever possible (default: small C >= 128 grids)
  SW_VP_BATCH,     // TTS_VP_BATCH=0: the variance predictors' first convs / LayerNorms as separate launches (fp32 encoder)
  SW_DEC_TRIM,     // TTS_DEC_TRIM=0/1: with predicted durations the decoder never / always runs at the longest utterance's frames (default: budgets over 8 frames per token)
  SW_ATTN_F32_KC,  // TTS_ATTN_F32_KC=n: fp32 attention key chunk of n keys (multiple of 32; 0: one chunk; default 64)
  SW_F32_ENC_SPLIT,  // TTS_F32_ENC_SPLIT=0: an fp32 model's encoder side on fp32 MFMA even with TTS_ENCODER_EXACT (read at finalize)
  SW_F32_DEC_SPLIT,  // TTS_F32_DEC_SPLIT=0: an fp32 model's decoder / postnet all on fp32 MFMA (read at finalize; needs the encoder split)
  SW_F32_DEC_PACKED,  // TTS_F32_DEC_PACKED=0: the fp32 decoder's FFN down-projections on fp32 MFMA, not the packed split-K form (finalize)
  SW_N
};

int sw(Sw s);                              // current value, -1 = not set
int sw_set(const char* name, int value);   // 0, or -1 for an unknown name
int sw_get(const char* name, int* value);  // 0 (value = current setting, -1 = not set), or -1 for an unknown name

}  // namespace tts
