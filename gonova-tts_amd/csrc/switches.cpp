// Runtime switches (switches.h): environment read once, then tts_set_switch.
#include "switches.h"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace tts {

namespace {
// (same order as the Sw enum)
const char* const kNames[SW_N] = {"TTS_REL_ATTN", "TTS_MRF_FUSED", "TTS_MRF_CHAIN", "TTS_POST_FUSE",
                                  "TTS_UP_STREAM", "TTS_XRES_NARROW", "TTS_XRES_NT", "TTS_PAIR_DIV",
                                  "TTS_ATTN_KSPLIT", "TTS_SPLIT_WHOLE", "TTS_XRES_DMA", "TTS_LN_FUSE",
                                  "TTS_SPLIT_NT1", "TTS_XRES_ORDER",
                                  "TTS_PAIR_SPLIT", "TTS_VP_BATCH", "TTS_DEC_TRIM", "TTS_ATTN_F32_KC",
                                  "TTS_F32_ENC_SPLIT", "TTS_F32_DEC_SPLIT",
                                  "TTS_F32_DEC_PACKED"};
std::atomic<int> g_val[SW_N];
std::once_flag g_once;

void init() {
  for (int i = 0; i < SW_N; ++i) {
    const char* e = getenv(kNames[i]);
    g_val[i].store(e ? atoi(e) : -1, std::memory_order_relaxed);
  }
}
}  // namespace

int sw(Sw s) {
  std::call_once(g_once, init);
  return g_val[s].load(std::memory_order_relaxed);
}

int sw_set(const char* name, int value) {
  std::call_once(g_once, init);
  if (!name) return -1;
  for (int i = 0; i < SW_N; ++i)
    if (!strcmp(name, kNames[i])) {
      g_val[i].store(value < 0 ? -1 : value, std::memory_order_relaxed);
      return 0;
    }
  return -1;
}

int sw_get(const char* name, int* value) {
  std::call_once(g_once, init);
  if (!name || !value) return -1;
  for (int i = 0; i < SW_N; ++i)
    if (!strcmp(name, kNames[i])) {
      *value = g_val[i].load(std::memory_order_relaxed);
      return 0;
    }
  return -1;
}

}  // namespace tts
