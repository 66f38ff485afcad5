// FastSpeech2-Conformer acoustic model runtime — placeholder until the HIP path lands.
#include "acoustic.h"

#include <stdexcept>

namespace tts {

struct AcousticModel::Impl {};

void AcousticModel::finalize(const GetData& get, const GetShape&, int) {
  loaded = false;
  (void)get;
}
void AcousticModel::reserve(int, int, int) {}
void AcousticModel::forward(const int32_t*, const int32_t*, int, int, const int32_t*, float*, int32_t*, int,
                            int32_t*, hipStream_t) {
  throw std::runtime_error("acoustic model not implemented");
}
void AcousticModel::free_all() {}

}  // namespace tts
