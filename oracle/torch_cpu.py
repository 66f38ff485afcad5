"""ORACLE (test infrastructure only) — torch-CPU fp32 restatement of the pipeline, used as
the timed CPU baseline of `bench.py` ("the build's own fp32 CPU restatement
... torch-CPU conv1d / conv_transpose1d / matmul, with the same seeded synthetic weights and
the same inputs") and checked against the NumPy oracle in `tests/test_oracle_golden.py`.

Only `tests/` and `bench.py`'s `cpu_baseline` leg import this module; the product path never
does.  Same architecture and citations as `oracle/vocoder.py` / `oracle/acoustic.py`
(transformers 5.15.0 FastSpeech2-Conformer / HiFi-GAN, ``HF:<line>``), batched over
utterances of EQUAL length only (no padding, so batching keeps B=1 semantics).
Layout: torch's channels-first [B, C, T] for the convs, [B, T, C] elsewhere.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

from .acoustic import rel_pos_table


def _t(w: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in w.items()
            if np.asarray(v).dtype.kind == "f"}


class TorchVocoder:
    """HiFi-GAN V1 generator (HF:1435-1475) on [B, T, 80] mel of equal lengths."""

    def __init__(self, weights, cfg=None):
        from gonova_tts_amd.config import VocoderConfig  # config only
        self.cfg = cfg or VocoderConfig()
        self.w = _t(weights)

    @torch.no_grad()
    def __call__(self, mel: torch.Tensor) -> torch.Tensor:
        c, w = self.cfg, self.w
        x = mel
        if c.normalize_before:  # HF:1445-1446
            x = (x - w["mean"]) / w["scale"]
        x = F.conv1d(x.transpose(1, 2), w["conv_pre.weight"], w["conv_pre.bias"], padding=3)  # HF:1454
        nk = len(c.resblock_kernel_sizes)
        for i, (u, k) in enumerate(zip(c.upsample_rates, c.upsample_kernel_sizes)):
            x = F.leaky_relu(x, c.leaky_relu_slope)  # HF:1456
            x = F.conv_transpose1d(x, w[f"upsampler.{i}.weight"], w[f"upsampler.{i}.bias"], stride=u,
                                   padding=(k - u) // 2)  # HF:1457
            acc = None
            for j, (ks, dils) in enumerate(zip(c.resblock_kernel_sizes, c.resblock_dilation_sizes)):
                p = f"resblocks.{i * nk + j}"
                h = x
                for q, d in enumerate(dils):  # HF:1343-1350
                    t = F.conv1d(F.leaky_relu(h, c.leaky_relu_slope), w[f"{p}.convs1.{q}.weight"],
                                 w[f"{p}.convs1.{q}.bias"], dilation=d, padding=(ks * d - d) // 2)
                    t = F.conv1d(F.leaky_relu(t, c.leaky_relu_slope), w[f"{p}.convs2.{q}.weight"],
                                 w[f"{p}.convs2.{q}.bias"], padding=(ks - 1) // 2)
                    h = h + t
                acc = h if acc is None else acc + h  # HF:1458-1461
            x = acc / nk
        x = F.conv1d(F.leaky_relu(x, 0.01), w["conv_post.weight"], w["conv_post.bias"], padding=3)  # HF:1464-1465
        return torch.tanh(x)[:, 0]  # HF:1466


class TorchAcoustic:
    """FastSpeech2ConformerModel inference (HF:1099-1288) on [B, N] token ids of equal length
    with explicit integer durations (equal totals), or predicted ones at B=1."""

    def __init__(self, weights, cfg=None):
        from gonova_tts_amd.config import AcousticConfig  # config only
        self.cfg = cfg or AcousticConfig()
        self.w = _t(weights)
        self._pe = {}

    def _pos(self, L):
        if L not in self._pe:
            self._pe[L] = torch.from_numpy(rel_pos_table(L, self.cfg.hidden_size))
        return self._pe[L]

    def _ln(self, x, p):
        return F.layer_norm(x, (x.shape[-1],), self.w[p + ".weight"], self.w[p + ".bias"], self.cfg.layer_norm_eps)

    def _conv(self, x, wn, bn, pad):  # x [B, T, C] -> [B, T, Cout]
        return F.conv1d(x.transpose(1, 2), self.w[wn], self.w.get(bn) if bn else None, padding=pad).transpose(1, 2)

    def _ffn(self, x, p):  # HF:682-698
        k = self.w[p + "conv1.weight"].shape[-1]
        h = torch.relu(self._conv(x, p + "conv1.weight", p + "conv1.bias", (k - 1) // 2))
        return self._conv(h, p + "conv2.weight", p + "conv2.bias", (k - 1) // 2)

    def _mha(self, x, pos_emb, p):  # HF:395-463
        w, H = self.w, self.cfg.num_attention_heads
        B, L, D = x.shape
        dk = D // H
        lin = lambda t, n: F.linear(t, w[p + n + ".weight"], w.get(p + n + ".bias"))  # noqa: E731
        q = lin(x, "linear_q").view(B, L, H, dk)
        k = lin(x, "linear_k").view(B, L, H, dk).transpose(1, 2)
        v = lin(x, "linear_v").view(B, L, H, dk).transpose(1, 2)
        pos = F.linear(pos_emb, w[p + "linear_pos.weight"]).view(2 * L - 1, H, dk).permute(1, 2, 0)  # [H, dk, 2L-1]
        qu = (q + w[p + "pos_bias_u"]).transpose(1, 2)
        qv = (q + w[p + "pos_bias_v"]).transpose(1, 2)
        ac = qu @ k.transpose(-1, -2)
        bd_full = qv @ pos  # [B, H, L, 2L-1]
        i = torch.arange(L)[:, None]
        j = torch.arange(L)[None, :]
        bd = bd_full.gather(-1, ((L - 1) - i + j).expand(B, H, L, L))  # HF:381-393 shift
        attn = torch.softmax((ac + bd) / math.sqrt(dk), dim=-1)
        o = (attn @ v).transpose(1, 2).reshape(B, L, D)
        return lin(o, "linear_out")

    def _conv_module(self, x, p):  # HF:501-535
        w, eps = self.w, self.cfg.batch_norm_eps
        D = x.shape[-1]
        a = F.linear(x, w[p + "pointwise_conv1.weight"][:, :, 0], w[p + "pointwise_conv1.bias"])
        g = (a[..., :D] * torch.sigmoid(a[..., D:])).transpose(1, 2)
        k = w[p + "depthwise_conv.weight"].shape[-1]
        y = F.conv1d(g, w[p + "depthwise_conv.weight"], w[p + "depthwise_conv.bias"], padding=(k - 1) // 2, groups=D)
        y = F.batch_norm(y, w[p + "norm.running_mean"], w[p + "norm.running_var"], w[p + "norm.weight"],
                         w[p + "norm.bias"], False, 0.0, eps)
        y = F.silu(y).transpose(1, 2)
        return F.linear(y, w[p + "pointwise_conv2.weight"][:, :, 0], w[p + "pointwise_conv2.bias"])

    def _stack(self, x, prefix, n):  # HF:803-867, 574-652
        L, D = x.shape[1], x.shape[2]
        x = x * math.sqrt(D)
        pe = self._pos(L)
        for i in range(n):
            p = f"{prefix}conformer_layers.{i}."
            x = self._ln(x + 0.5 * self._ffn(x, p + "feed_forward_macaron."), p + "ff_macaron_layer_norm")
            x = self._ln(x + self._mha(x, pe, p + "self_attn."), p + "self_attn_layer_norm")
            x = self._ln(x + self._conv_module(x, p + "conv_module."), p + "conv_layer_norm")
            x = self._ln(x + 0.5 * self._ffn(x, p + "feed_forward."), p + "ff_layer_norm")
            x = self._ln(x, p + "final_layer_norm")
        return x

    def _predictor(self, x, p, n):  # HF:261-325, 161-185
        h = x
        for i in range(n):
            q = f"{p}conv_layers.{i}."
            k = self.w[q + "conv.weight"].shape[-1]
            h = self._ln(torch.relu(self._conv(h, q + "conv.weight", q + "conv.bias", (k - 1) // 2)),
                         q + "layer_norm")
        return F.linear(h, self.w[p + "linear.weight"], self.w[p + "linear.bias"])[..., 0]

    @torch.no_grad()
    def __call__(self, ids: torch.Tensor, durations: torch.Tensor = None):
        """ids int64 [B, N]; durations int64 [B, N] (equal per-utterance sums) -> mel [B, T, 80]."""
        c, w = self.cfg, self.w
        x = self._stack(w["encoder.embed.weight"][ids], "encoder.", c.encoder_layers)
        pitch = self._predictor(x, "pitch_predictor.", c.pitch_predictor_layers)
        energy = self._predictor(x, "energy_predictor.", c.energy_predictor_layers)
        logd = self._predictor(x, "duration_predictor.", c.duration_predictor_layers)
        if durations is None:  # HF:181-183, per utterance all-zero rule HF:108-109
            assert ids.shape[0] == 1, "predicted durations: one utterance at a time"
            durations = torch.clamp(torch.round(torch.exp(logd) - 1), min=0).long()
            if int(durations.sum()) == 0:
                durations = torch.ones_like(durations)
        x = x + energy[..., None] * w["energy_embed.conv.weight"][:, 0, 0] + w["energy_embed.conv.bias"]
        x = x + pitch[..., None] * w["pitch_embed.conv.weight"][:, 0, 0] + w["pitch_embed.conv.bias"]
        x = torch.stack([torch.repeat_interleave(x[b], durations[b], dim=0) for b in range(x.shape[0])])  # HF:82-126
        x = self._stack(x, "decoder.", c.decoder_layers)
        before = F.linear(x, w["speech_decoder_postnet.feat_out.weight"], w["speech_decoder_postnet.feat_out.bias"])
        h = before.transpose(1, 2)  # HF:238-244
        for i in range(c.postnet_layers):
            p = f"speech_decoder_postnet.layers.{i}."
            k = w[p + "conv.weight"].shape[-1]
            h = F.conv1d(h, w[p + "conv.weight"], None, padding=(k - 1) // 2)
            h = F.batch_norm(h, w[p + "batch_norm.running_mean"], w[p + "batch_norm.running_var"],
                             w[p + "batch_norm.weight"], w[p + "batch_norm.bias"], False, 0.0, c.batch_norm_eps)
            if i < c.postnet_layers - 1:
                h = torch.tanh(h)
        return before + h.transpose(1, 2), durations
