"""Model configurations for the batched TTS engine.

The hot path replaces the reference's model call site
(`services/tts/core/synthesizer.py:344-350`, `self.model.generate(...)`) with a
non-autoregressive acoustic model (FastSpeech2 with Conformer blocks and a
duration / pitch / energy variance adaptor) followed by a HiFi-GAN V1 vocoder
at 22.05 kHz (north star, BASELINE.json).  The field names mirror the public
`FastSpeech2ConformerConfig` / `FastSpeech2ConformerHifiGanConfig` of
transformers 5.15.0 (the pinned in-container description of that architecture,
SURVEY.md §8c) so that a checkpoint in that naming can be loaded unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field, asdict
from typing import Optional, List, Tuple

SAMPLE_RATE = 22050
HOP_LENGTH = 256  # prod(upsample_rates): one mel frame -> 256 samples


@dataclass
class AcousticConfig:
    hidden_size: int = 384
    vocab_size: int = 78
    num_mel_bins: int = 80
    encoder_layers: int = 4
    decoder_layers: int = 4
    num_attention_heads: int = 2
    linear_units: int = 1536
    positionwise_conv_kernel_size: int = 3
    encoder_kernel_size: int = 7     # conformer depthwise conv, encoder
    decoder_kernel_size: int = 31    # conformer depthwise conv, decoder
    duration_predictor_layers: int = 2
    duration_predictor_channels: int = 256
    duration_predictor_kernel_size: int = 3
    pitch_predictor_layers: int = 5
    pitch_predictor_channels: int = 256
    pitch_predictor_kernel_size: int = 5
    energy_predictor_layers: int = 2
    energy_predictor_channels: int = 256
    energy_predictor_kernel_size: int = 3
    postnet_layers: int = 5
    postnet_units: int = 256
    postnet_kernel: int = 5
    layer_norm_eps: float = 1e-5
    batch_norm_eps: float = 1e-5
    speaking_speed: float = 1.0
    # HF FastSpeech2ConformerConfig.speaker_embed_dim (HF:1051-1053, 1192-1196): when set, an
    # external speaker embedding is L2-normalised, concatenated to every encoder frame and
    # projected back to hidden_size (Linear(hidden + E -> hidden)); None = single speaker
    speaker_embed_dim: Optional[int] = None

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    def to_dict(self):
        return asdict(self)


@dataclass
class VocoderConfig:
    model_in_dim: int = 80
    upsample_initial_channel: int = 512
    upsample_rates: Tuple[int, ...] = (8, 8, 2, 2)
    upsample_kernel_sizes: Tuple[int, ...] = (16, 16, 4, 4)
    resblock_kernel_sizes: Tuple[int, ...] = (3, 7, 11)
    resblock_dilation_sizes: Tuple[Tuple[int, ...], ...] = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    leaky_relu_slope: float = 0.1
    normalize_before: bool = True

    @property
    def hop(self) -> int:
        h = 1
        for r in self.upsample_rates:
            h *= r
        return h

    def stage_channels(self, i: int) -> int:
        return self.upsample_initial_channel // (2 ** (i + 1))

    def to_dict(self):
        return asdict(self)


def vocoder_flops_per_sample(cfg: VocoderConfig = VocoderConfig()) -> float:
    """Algorithmic multiply-add FLOPs (2/MAC) per output sample of the vocoder.

    Counts conv_pre, the transposed-conv upsamplers (k/s taps per output), every MRF
    conv and conv_post; matches the survey's 2,398,848 FLOP/sample.
    """
    hop = cfg.hop
    c0 = cfg.upsample_initial_channel
    f = 0.0
    # conv_pre at mel rate
    f += 2.0 * cfg.model_in_dim * c0 * 7 / hop
    rate = 1.0 / hop  # frames per sample
    cin = c0
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        cout = cfg.stage_channels(i)
        rate *= u
        f += 2.0 * cin * cout * (k / u) * rate  # each output touches k/u taps
        for ks, dils in zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes):
            f += len(dils) * 2 * (2.0 * cout * cout * ks) * rate
        cin = cout
    f += 2.0 * cin * 1 * 7
    return f
