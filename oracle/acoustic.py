"""ORACLE (test infrastructure only) — CPU NumPy restatement of the FastSpeech2-Conformer
acoustic model (text tokens -> mel frames).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this module.  The product path never calls into `oracle/`.

The reference's synthesis arithmetic lives in the un-vendored third-party
`chatterbox` package (`services/tts/core/synthesizer.py:167,185,344-350`), so
parity against the reference model itself is unpinned.  The
north star (BASELINE.json) names an FS2-style acoustic model with a duration /
pitch variance adaptor; this file restates the published FastSpeech2-Conformer
as implemented by transformers 5.15.0 `FastSpeech2ConformerModel` (cited as
``HF:<line>`` in `transformers/models/fastspeech2_conformer/
modeling_fastspeech2_conformer.py`), pinned by golden vectors from that
implementation (`tests/golden/make_golden.py`).

Semantics are B=1 per utterance (HF runs the decoder unmasked for padded
batches, HF:1228-1229, which is not padding-invariant).
Layout: channels-last [T, C] float32.
"""
from __future__ import annotations

import math

import numpy as np

from .vocoder import conv1d


def layer_norm(x, w, b, eps=1e-5):
    x64 = x.astype(np.float64)
    mu = x64.mean(-1, keepdims=True)
    var = ((x64 - mu) ** 2).mean(-1, keepdims=True)
    return ((x64 - mu) / np.sqrt(var + eps) * w + b).astype(x.dtype)


def batch_norm_eval(x, w, b, rm, rv, eps=1e-5):
    return ((x - rm) / np.sqrt(rv + eps) * w + b).astype(x.dtype)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def softmax(x, axis=-1):
    m = x.max(axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis, keepdims=True)


def rel_pos_table(length, d_model, dtype=np.float32):
    """FastSpeech2ConformerRelPositionalEncoding (HF:723-767): rows for relative
    positions L-1, L-2, ..., 0, ..., -(L-1); returns [2L-1, d_model].

    The angle p*div is rounded to float32 first, as torch computes it.
    """
    div = np.exp(np.arange(0, d_model, 2, dtype=np.float32) * np.float32(-(math.log(10000.0) / d_model)))
    pos = np.arange(length - 1, -length, -1, dtype=np.float32)[:, None]  # L-1 .. -(L-1)
    ang = (pos * div[None, :]).astype(np.float32).astype(np.float64)
    pe = np.zeros((2 * length - 1, d_model), np.float64)
    pe[:, 0::2] = np.sin(ang)
    pe[:, 1::2] = np.cos(ang)
    return pe.astype(dtype)


def ffn(x, w, p):
    """FastSpeech2ConformerMultiLayeredConv1d (HF:682-698): conv(k3) -> ReLU -> conv(k3)."""
    k = w[p + "conv1.weight"].shape[-1]
    h = conv1d(x, w[p + "conv1.weight"], w[p + "conv1.bias"], padding=(k - 1) // 2)
    h = np.maximum(h, 0)
    return conv1d(h, w[p + "conv2.weight"], w[p + "conv2.bias"], padding=(k - 1) // 2)


def rel_mha(x, pos_emb, w, p, num_heads):
    """FastSpeech2ConformerAttention.forward (HF:395-463), unmasked (B=1)."""
    L, D = x.shape
    dk = D // num_heads
    q = (x @ w[p + "linear_q.weight"].T + w[p + "linear_q.bias"]).reshape(L, num_heads, dk)
    kk = (x @ w[p + "linear_k.weight"].T + w[p + "linear_k.bias"]).reshape(L, num_heads, dk)
    v = (x @ w[p + "linear_v.weight"].T + w[p + "linear_v.bias"]).reshape(L, num_heads, dk)
    pos = (pos_emb @ w[p + "linear_pos.weight"].T).reshape(2 * L - 1, num_heads, dk)
    qu = (q + w[p + "pos_bias_u"]).transpose(1, 0, 2)  # [H, L, dk]
    qv = (q + w[p + "pos_bias_v"]).transpose(1, 0, 2)
    ac = qu @ kk.transpose(1, 2, 0)                     # [H, L, L]
    bd_full = qv @ pos.transpose(1, 2, 0)               # [H, L, 2L-1]
    # shift_relative_position_tensor (HF:381-393): bd[i, j] = bd_full[i, L-1-i+j]
    i = np.arange(L)[:, None]
    j = np.arange(L)[None, :]
    bd = bd_full[:, i, (L - 1) - i + j]
    scores = (ac + bd) / np.float32(math.sqrt(dk))
    attn = softmax(scores.astype(np.float32), -1)
    o = (attn @ v.transpose(1, 0, 2)).transpose(1, 0, 2).reshape(L, D)
    return o @ w[p + "linear_out.weight"].T + w[p + "linear_out.bias"]


def conv_module(x, w, p, eps=1e-5):
    """FastSpeech2ConformerConvolutionModule.forward (HF:501-535), unmasked (B=1)."""
    D = x.shape[1]
    a = x @ w[p + "pointwise_conv1.weight"][:, :, 0].T + w[p + "pointwise_conv1.bias"]
    g = a[:, :D] * sigmoid(a[:, D:])  # GLU over channels
    dw = w[p + "depthwise_conv.weight"][:, 0, :]  # [C, k]
    k = dw.shape[1]
    pad = (k - 1) // 2
    gp = np.zeros((g.shape[0] + 2 * pad, D), g.dtype)
    gp[pad: pad + g.shape[0]] = g
    y = np.zeros_like(g)
    for j in range(k):
        y += gp[j: j + g.shape[0]] * dw[:, j]
    y += w[p + "depthwise_conv.bias"]
    y = batch_norm_eval(y, w[p + "norm.weight"], w[p + "norm.bias"], w[p + "norm.running_mean"],
                        w[p + "norm.running_var"], eps)
    y = y * sigmoid(y)  # SiLU
    return y @ w[p + "pointwise_conv2.weight"][:, :, 0].T + w[p + "pointwise_conv2.bias"]


def conformer_layer(x, pos_emb, w, p, num_heads):
    """FastSpeech2ConformerEncoderLayer.forward (HF:574-652), post-LN, macaron."""
    x = layer_norm(x + 0.5 * ffn(x, w, p + "feed_forward_macaron."),
                   w[p + "ff_macaron_layer_norm.weight"], w[p + "ff_macaron_layer_norm.bias"])
    x = layer_norm(x + rel_mha(x, pos_emb, w, p + "self_attn.", num_heads),
                   w[p + "self_attn_layer_norm.weight"], w[p + "self_attn_layer_norm.bias"])
    x = layer_norm(x + conv_module(x, w, p + "conv_module."),
                   w[p + "conv_layer_norm.weight"], w[p + "conv_layer_norm.bias"])
    x = layer_norm(x + 0.5 * ffn(x, w, p + "feed_forward."),
                   w[p + "ff_layer_norm.weight"], w[p + "ff_layer_norm.bias"])
    return layer_norm(x, w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"])


def conformer_stack(x, w, prefix, n_layers, num_heads):
    """FastSpeech2ConformerEncoder.forward (HF:803-867) after the input embedding."""
    L, D = x.shape
    x = x * np.float32(math.sqrt(D))  # RelPositionalEncoding input_scale (HF:763)
    pos_emb = rel_pos_table(L, D, x.dtype)
    for i in range(n_layers):
        x = conformer_layer(x, pos_emb, w, f"{prefix}conformer_layers.{i}.", num_heads)
    return x


def variance_predictor(x, w, p, n_layers):
    """FastSpeech2ConformerVariancePredictor / DurationPredictor conv stack (HF:261-325,161-185).

    Returns the linear output [L] (log-domain for durations)."""
    h = x
    for i in range(n_layers):
        q = f"{p}conv_layers.{i}."
        k = w[q + "conv.weight"].shape[-1]
        h = conv1d(h, w[q + "conv.weight"], w[q + "conv.bias"], padding=(k - 1) // 2)
        h = np.maximum(h, 0)
        h = layer_norm(h, w[q + "layer_norm.weight"], w[q + "layer_norm.bias"])
    return (h @ w[p + "linear.weight"].T + w[p + "linear.bias"])[:, 0]


def durations_from_log(logd, speaking_speed=1.0):
    """HF:183 clamp(round(exp(x) - 1), 0) (round half to even, like torch.round),
    then length_regulator's speed scaling and all-zero rule (HF:104-109), per utterance."""
    d = np.maximum(np.round(np.exp(logd.astype(np.float32)) - np.float32(1.0)), 0).astype(np.int64)
    if speaking_speed != 1.0:
        d = np.round(d.astype(np.float32) * np.float32(speaking_speed)).astype(np.int64)
    if d.sum() == 0:
        d[:] = 1
    return d


def postnet(x, w, n_layers=5, eps=1e-5):
    """FastSpeech2ConformerSpeechDecoderPostnet.forward (HF:238-244)."""
    before = x @ w["speech_decoder_postnet.feat_out.weight"].T + w["speech_decoder_postnet.feat_out.bias"]
    h = before
    for i in range(n_layers):
        p = f"speech_decoder_postnet.layers.{i}."
        k = w[p + "conv.weight"].shape[-1]
        h = conv1d(h, w[p + "conv.weight"], None, padding=(k - 1) // 2)
        h = batch_norm_eval(h, w[p + "batch_norm.weight"], w[p + "batch_norm.bias"],
                            w[p + "batch_norm.running_mean"], w[p + "batch_norm.running_var"], eps)
        if i < n_layers - 1:
            h = np.tanh(h)
    return before + h


def acoustic_forward(token_ids, w, cfg=None, durations=None, dtype=np.float32, speaker_embedding=None):
    """FastSpeech2ConformerModel.forward inference path (HF:1099-1288) for one utterance.

    token_ids: int [L].  durations: optional int [L] override (otherwise predicted).
    speaker_embedding: optional [E] vector, used when the weights carry `projection.*`
    (HF:1192-1196: normalize, concat to every encoder frame, Linear back to hidden).
    Returns dict(mel [T, 80], durations [L], pitch [L], energy [L], log_durations [L]).
    """
    from gonova_tts_amd.config import AcousticConfig  # config only
    cfg = cfg or AcousticConfig()
    w = {k: np.asarray(v, dtype) if np.asarray(v).dtype.kind == "f" else v for k, v in w.items()}
    ids = np.asarray(token_ids, np.int64)
    x = w["encoder.embed.weight"][ids]
    x = conformer_stack(x, w, "encoder.", cfg.encoder_layers, cfg.num_attention_heads)
    if speaker_embedding is not None and "projection.weight" in w:  # HF:1192-1196
        e = np.asarray(speaker_embedding, dtype)
        e = e / max(float(np.sqrt((e.astype(np.float64) ** 2).sum())), 1e-12)  # F.normalize, eps 1e-12
        xe = np.concatenate([x, np.broadcast_to(e, (x.shape[0], e.shape[0]))], axis=1)
        x = xe @ w["projection.weight"].T + w["projection.bias"]
    pitch = variance_predictor(x, w, "pitch_predictor.", cfg.pitch_predictor_layers)
    energy = variance_predictor(x, w, "energy_predictor.", cfg.energy_predictor_layers)
    logd = variance_predictor(x, w, "duration_predictor.", cfg.duration_predictor_layers)
    d = durations_from_log(logd, cfg.speaking_speed) if durations is None else np.asarray(durations, np.int64)
    e_emb = energy[:, None] * w["energy_embed.conv.weight"][:, 0, 0] + w["energy_embed.conv.bias"]
    p_emb = pitch[:, None] * w["pitch_embed.conv.weight"][:, 0, 0] + w["pitch_embed.conv.bias"]
    x = (x + e_emb) + p_emb  # HF:1218 hidden + energy + pitch
    x = np.repeat(x, d, axis=0)  # length_regulator (HF:82-126)
    x = conformer_stack(x, w, "decoder.", cfg.decoder_layers, cfg.num_attention_heads)
    mel = postnet(x, w, cfg.postnet_layers)
    return dict(mel=mel, durations=d, pitch=pitch, energy=energy, log_durations=logd)
