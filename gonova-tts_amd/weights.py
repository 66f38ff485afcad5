"""Weight specification and deterministic seeded weights.

No pretrained checkpoint is reachable offline (the reference's model weights are
fetched by name from the HF Hub at `services/tts/core/synthesizer.py:185`), so
the engine runs on weights re-created from a seed.  Every tensor is drawn from
its own `numpy.random.Generator(PCG64)` seeded by (seed, crc32(name)), so the
same weights come out on any box regardless of iteration order.

Tensor names and shapes follow the transformers 5.15.0 state_dict of
`FastSpeech2ConformerModel` / `FastSpeech2ConformerHifiGan` so a
real checkpoint in that naming loads unchanged.

Initialisation is fan-in scaled (SURVEY.md §7 "Degenerate random init"): conv
std 0.5/sqrt(C_in*k), transposed conv std 1/sqrt(C_in*k/stride); HF's default
init makes the waveform ~1e-5 which is useless for tolerances.
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np

from .config import AcousticConfig, VocoderConfig

# init kinds: (kind, scale)
#   "normal"  : N(0, scale^2)
#   "ones_n"  : 1 + N(0, scale^2)
#   "zeros"   : 0
#   "const"   : scale
#   "uniform" : U(lo, hi) with scale=(lo, hi)
#   "embed"   : N(0, scale^2) with row 0 zeroed (padding_idx=0)


def _vocoder_spec(cfg: VocoderConfig):
    spec = OrderedDict()
    c0 = cfg.upsample_initial_channel
    spec["mean"] = ((cfg.model_in_dim,), ("zeros", 0.0))
    spec["scale"] = ((cfg.model_in_dim,), ("const", 1.0))
    spec["conv_pre.weight"] = ((c0, cfg.model_in_dim, 7), ("normal", 0.5 / math.sqrt(cfg.model_in_dim * 7)))
    spec["conv_pre.bias"] = ((c0,), ("normal", 0.02))
    cin = c0
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        cout = cfg.stage_channels(i)
        spec[f"upsampler.{i}.weight"] = ((cin, cout, k), ("normal", 1.0 / math.sqrt(cin * k / u)))
        spec[f"upsampler.{i}.bias"] = ((cout,), ("normal", 0.02))
        cin = cout
    nk = len(cfg.resblock_kernel_sizes)
    for i in range(len(cfg.upsample_rates)):
        ch = cfg.stage_channels(i)
        for j, (ks, dils) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            r = i * nk + j
            for p in range(len(dils)):
                for which in ("convs1", "convs2"):
                    spec[f"resblocks.{r}.{which}.{p}.weight"] = ((ch, ch, ks), ("normal", 0.5 / math.sqrt(ch * ks)))
                    spec[f"resblocks.{r}.{which}.{p}.bias"] = ((ch,), ("normal", 0.02))
    spec["conv_post.weight"] = ((1, cin, 7), ("normal", 0.5 / math.sqrt(cin * 7)))
    spec["conv_post.bias"] = ((1,), ("normal", 0.02))
    return spec


def _conformer_layer_spec(prefix: str, cfg: AcousticConfig, dw_kernel: int):
    h, u, k = cfg.hidden_size, cfg.linear_units, cfg.positionwise_conv_kernel_size
    s = OrderedDict()
    a = prefix + "self_attn."
    s[a + "pos_bias_u"] = ((cfg.num_attention_heads, cfg.head_dim), ("normal", 0.1))
    s[a + "pos_bias_v"] = ((cfg.num_attention_heads, cfg.head_dim), ("normal", 0.1))
    for n in ("q", "k", "v", "out"):
        s[a + f"linear_{n}.weight"] = ((h, h), ("normal", 1.0 / math.sqrt(h)))
        s[a + f"linear_{n}.bias"] = ((h,), ("normal", 0.02))
    s[a + "linear_pos.weight"] = ((h, h), ("normal", 1.0 / math.sqrt(h)))
    for ff in ("feed_forward.", "feed_forward_macaron."):
        s[prefix + ff + "conv1.weight"] = ((u, h, k), ("normal", 1.0 / math.sqrt(h * k)))
        s[prefix + ff + "conv1.bias"] = ((u,), ("normal", 0.02))
        s[prefix + ff + "conv2.weight"] = ((h, u, k), ("normal", 1.0 / math.sqrt(u * k)))
        s[prefix + ff + "conv2.bias"] = ((h,), ("normal", 0.02))
    c = prefix + "conv_module."
    s[c + "pointwise_conv1.weight"] = ((2 * h, h, 1), ("normal", 1.0 / math.sqrt(h)))
    s[c + "pointwise_conv1.bias"] = ((2 * h,), ("normal", 0.02))
    s[c + "depthwise_conv.weight"] = ((h, 1, dw_kernel), ("normal", 1.0 / math.sqrt(dw_kernel)))
    s[c + "depthwise_conv.bias"] = ((h,), ("normal", 0.02))
    s[c + "norm.weight"] = ((h,), ("ones_n", 0.05))
    s[c + "norm.bias"] = ((h,), ("normal", 0.05))
    s[c + "norm.running_mean"] = ((h,), ("normal", 0.1))
    s[c + "norm.running_var"] = ((h,), ("uniform", (0.5, 1.5)))
    s[c + "pointwise_conv2.weight"] = ((h, h, 1), ("normal", 1.0 / math.sqrt(h)))
    s[c + "pointwise_conv2.bias"] = ((h,), ("normal", 0.02))
    for ln in ("ff_macaron_layer_norm", "self_attn_layer_norm", "conv_layer_norm", "ff_layer_norm",
               "final_layer_norm"):
        s[prefix + ln + ".weight"] = ((h,), ("ones_n", 0.05))
        s[prefix + ln + ".bias"] = ((h,), ("normal", 0.05))
    return s


def _predictor_spec(prefix: str, cfg: AcousticConfig, layers: int, chans: int, ks: int,
                    lin_w_std: float, lin_b: Tuple[str, float]):
    s = OrderedDict()
    for i in range(layers):
        cin = cfg.hidden_size if i == 0 else chans
        p = f"{prefix}conv_layers.{i}."
        s[p + "conv.weight"] = ((chans, cin, ks), ("normal", 1.0 / math.sqrt(cin * ks)))
        s[p + "conv.bias"] = ((chans,), ("normal", 0.02))
        s[p + "layer_norm.weight"] = ((chans,), ("ones_n", 0.05))
        s[p + "layer_norm.bias"] = ((chans,), ("normal", 0.05))
    s[prefix + "linear.weight"] = ((1, chans), ("normal", lin_w_std))
    s[prefix + "linear.bias"] = ((1,), lin_b)
    return s


def _acoustic_spec(cfg: AcousticConfig):
    s = OrderedDict()
    h = cfg.hidden_size
    s["encoder.embed.weight"] = ((cfg.vocab_size, h), ("embed", 1.0 / math.sqrt(h)))
    for i in range(cfg.encoder_layers):
        s.update(_conformer_layer_spec(f"encoder.conformer_layers.{i}.", cfg, cfg.encoder_kernel_size))
    # log-duration ~ ln 4 +- 0.5 -> durations mostly 1..6 frames per token
    s.update(_predictor_spec("duration_predictor.", cfg, cfg.duration_predictor_layers,
                             cfg.duration_predictor_channels, cfg.duration_predictor_kernel_size,
                             0.5 / math.sqrt(cfg.duration_predictor_channels), ("const", math.log(4.0))))
    if cfg.speaker_embed_dim:  # speaker-embedding projection (HF:1051-1053)
        e = cfg.speaker_embed_dim
        s["projection.weight"] = ((h, h + e), ("normal", 1.0 / math.sqrt(h + e)))
        s["projection.bias"] = ((h,), ("normal", 0.02))
    s.update(_predictor_spec("pitch_predictor.", cfg, cfg.pitch_predictor_layers,
                             cfg.pitch_predictor_channels, cfg.pitch_predictor_kernel_size,
                             1.0 / math.sqrt(cfg.pitch_predictor_channels), ("normal", 0.02)))
    s["pitch_embed.conv.weight"] = ((h, 1, 1), ("normal", 0.5))
    s["pitch_embed.conv.bias"] = ((h,), ("normal", 0.02))
    s.update(_predictor_spec("energy_predictor.", cfg, cfg.energy_predictor_layers,
                             cfg.energy_predictor_channels, cfg.energy_predictor_kernel_size,
                             1.0 / math.sqrt(cfg.energy_predictor_channels), ("normal", 0.02)))
    s["energy_embed.conv.weight"] = ((h, 1, 1), ("normal", 0.5))
    s["energy_embed.conv.bias"] = ((h,), ("normal", 0.02))
    for i in range(cfg.decoder_layers):
        s.update(_conformer_layer_spec(f"decoder.conformer_layers.{i}.", cfg, cfg.decoder_kernel_size))
    m = cfg.num_mel_bins
    s["speech_decoder_postnet.feat_out.weight"] = ((m, h), ("normal", 1.0 / math.sqrt(h)))
    s["speech_decoder_postnet.feat_out.bias"] = ((m,), ("normal", 0.02))
    for i in range(cfg.postnet_layers):
        cin = m if i == 0 else cfg.postnet_units
        cout = m if i == cfg.postnet_layers - 1 else cfg.postnet_units
        p = f"speech_decoder_postnet.layers.{i}."
        s[p + "conv.weight"] = ((cout, cin, cfg.postnet_kernel), ("normal", 1.0 / math.sqrt(cin * cfg.postnet_kernel)))
        s[p + "batch_norm.weight"] = ((cout,), ("ones_n", 0.05))
        s[p + "batch_norm.bias"] = ((cout,), ("normal", 0.05))
        s[p + "batch_norm.running_mean"] = ((cout,), ("normal", 0.1))
        s[p + "batch_norm.running_var"] = ((cout,), ("uniform", (0.5, 1.5)))
    return s


def vocoder_spec(cfg: VocoderConfig = None):
    return _vocoder_spec(cfg or VocoderConfig())


def acoustic_spec(cfg: AcousticConfig = None):
    return _acoustic_spec(cfg or AcousticConfig())


def _draw(name: str, shape, init, seed: int) -> np.ndarray:
    kind, scale = init
    rng = np.random.default_rng([seed & 0xFFFFFFFF, zlib.crc32(name.encode())])
    if kind == "normal":
        return (rng.standard_normal(shape) * scale).astype(np.float32)
    if kind == "ones_n":
        return (1.0 + rng.standard_normal(shape) * scale).astype(np.float32)
    if kind == "zeros":
        return np.zeros(shape, np.float32)
    if kind == "const":
        return np.full(shape, scale, np.float32)
    if kind == "uniform":
        lo, hi = scale
        return rng.uniform(lo, hi, shape).astype(np.float32)
    if kind == "embed":
        w = (rng.standard_normal(shape) * scale).astype(np.float32)
        w[0] = 0.0
        return w
    raise ValueError(kind)


def make_vocoder_weights(seed: int = 0, cfg: VocoderConfig = None) -> Dict[str, np.ndarray]:
    """Deterministic fp32 HiFi-GAN V1 weights in HF state_dict naming."""
    return OrderedDict((n, _draw(n, shp, init, seed)) for n, (shp, init) in vocoder_spec(cfg).items())


def make_acoustic_weights(seed: int = 0, cfg: AcousticConfig = None, fixed_duration: int = None
                          ) -> Dict[str, np.ndarray]:
    """Deterministic fp32 FS2-Conformer weights in HF state_dict naming.

    ``fixed_duration=d`` sets the duration predictor's output layer to weight 0,
    bias ln(d+1) so every token gets exactly d frames (the C3 benchmark input,
    BASELINE.md §2: durations forced to 6 with bias ln 7).
    """
    w = OrderedDict((n, _draw(n, shp, init, seed)) for n, (shp, init) in acoustic_spec(cfg).items())
    if fixed_duration is not None:
        w["duration_predictor.linear.weight"][:] = 0.0
        w["duration_predictor.linear.bias"][:] = math.log(fixed_duration + 1.0)
    return w
