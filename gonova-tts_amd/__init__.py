"""gonova_tts_amd — MI355X-native batched TTS synthesis engine.

Drop-in for the model behind the reference's `services/tts` synthesis call site
(`services/tts/core/synthesizer.py:167,185,344-350`): a FastSpeech2-Conformer
acoustic model and a HiFi-GAN V1 vocoder whose hot ops are hand-written HIP
kernels for gfx950 behind a C-ABI (`include/tts_hip.h`, `libtts_hip.so`).

Import as ``gonova_tts_amd`` (see the repo-root shim ``gonova_tts_amd.py``).
"""
from .config import AcousticConfig, VocoderConfig, SAMPLE_RATE, HOP_LENGTH  # noqa: F401

__version__ = "0.1.0"
