"""ORACLE (test infrastructure only) — CPU NumPy restatement of the HiFi-GAN V1 vocoder.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this module, and only as the checker / the timed CPU baseline.  The
product path (`gonova_tts_amd`) never calls into `oracle/`.

Where the algorithm comes from
------------------------------
The reference (`/root/reference/services/tts`) delegates all synthesis arithmetic
to the un-vendored, unpinned third-party `chatterbox` package
(`services/tts/core/synthesizer.py:167,185,344-350`); nothing of it is in the
reference tree, so parity against the reference model is **unpinned** (SURVEY.md
§8c).  The north star (BASELINE.json) asks instead for a HiFi-GAN V1 vocoder at
22.05 kHz.  This file restates the published HiFi-GAN V1 generator as described
by transformers 5.15.0 `FastSpeech2ConformerHifiGan`
(`transformers/models/fastspeech2_conformer/modeling_fastspeech2_conformer.py`,
cited below as ``HF:<line>``), the architecture pinned in this container.  The
restatement is pinned against golden vectors produced by that implementation
(`tests/golden/make_golden.py` -> `tests/golden/*.npz`,
`tests/test_oracle_golden.py`).

Layout: one utterance at a time, channels-last ``[T, C]`` float32 (the engine's
HBM layout), so a conv is k shifted ``[T, Cin] @ [Cin, Cout]`` GEMMs.
"""
from __future__ import annotations

import numpy as np

LRELU_SLOPE = 0.1  # HF config leaky_relu_slope (HifiGanResidualBlock / upsampler)


def leaky_relu(x, slope):
    return np.where(x >= 0, x, x * np.asarray(slope, x.dtype))


def conv1d(x, w, b=None, dilation=1, padding=0):
    """nn.Conv1d(stride=1) on channels-last x[T, Cin]; w[Cout, Cin, k] (PyTorch layout).

    Zero padding of `padding` rows on both sides; out length T + 2p - d(k-1).
    """
    t, cin = x.shape
    cout, cin_w, k = w.shape
    assert cin_w == cin, (cin_w, cin)
    xp = np.zeros((t + 2 * padding, cin), x.dtype)
    xp[padding:padding + t] = x
    tout = t + 2 * padding - dilation * (k - 1)
    y = np.zeros((tout, cout), x.dtype)
    for j in range(k):
        y += xp[j * dilation: j * dilation + tout] @ w[:, :, j].T.astype(x.dtype)
    if b is not None:
        y += b.astype(x.dtype)
    return y


def conv_transpose1d(x, w, b, stride, padding):
    """nn.ConvTranspose1d on channels-last x[T, Cin]; w[Cin, Cout, k] (PyTorch layout).

    out[to] = b + sum_{ti, j : to = ti*s - p + j} x[ti] @ w[:, :, j]   (HF:1376-1386)
    """
    t, cin = x.shape
    _, cout, k = w.shape
    full = np.zeros(((t - 1) * stride + k, cout), x.dtype)
    for j in range(k):
        full[j: j + (t - 1) * stride + 1: stride] += x @ w[:, :, j].astype(x.dtype)
    tout = (t - 1) * stride - 2 * padding + k
    y = full[padding: padding + tout]
    if b is not None:
        y = y + b.astype(x.dtype)
    return y


def resblock(x, weights, prefix, kernel_size, dilations, slope=LRELU_SLOPE):
    """HifiGanResidualBlock.forward (HF:1343-1350): 3 x [lrelu -> conv(d) -> lrelu -> conv(1) -> +res]."""
    h = x
    for p, d in enumerate(dilations):
        r = h
        h = leaky_relu(h, slope)
        h = conv1d(h, weights[f"{prefix}.convs1.{p}.weight"], weights[f"{prefix}.convs1.{p}.bias"],
                   dilation=d, padding=(kernel_size * d - d) // 2)
        h = leaky_relu(h, slope)
        h = conv1d(h, weights[f"{prefix}.convs2.{p}.weight"], weights[f"{prefix}.convs2.{p}.bias"],
                   dilation=1, padding=(kernel_size - 1) // 2)
        h = h + r
    return h


def vocoder_forward(mel, weights, cfg=None, dtype=np.float32):
    """FastSpeech2ConformerHifiGan.forward (HF:1435-1475) for one utterance.

    mel: [T, 80] (HF's [T, model_in_dim] layout).  Returns waveform [T * 256].
    """
    from gonova_tts_amd.config import VocoderConfig  # config only (no product code path)
    cfg = cfg or VocoderConfig()
    x = np.asarray(mel, dtype)
    if cfg.normalize_before:  # HF:1445-1446
        x = (x - weights["mean"].astype(dtype)) / weights["scale"].astype(dtype)
    x = conv1d(x, weights["conv_pre.weight"], weights["conv_pre.bias"], padding=3)  # HF:1454
    nk = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        x = leaky_relu(x, cfg.leaky_relu_slope)  # HF:1456
        x = conv_transpose1d(x, weights[f"upsampler.{i}.weight"], weights[f"upsampler.{i}.bias"],
                             stride=u, padding=(k - u) // 2)  # HF:1457
        acc = None
        for j, (ks, dils) in enumerate(zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes)):
            r = resblock(x, weights, f"resblocks.{i * nk + j}", ks, dils, cfg.leaky_relu_slope)
            acc = r if acc is None else acc + r  # HF:1458-1461
        x = acc / nk
    x = leaky_relu(x, 0.01)  # HF:1464, nn.functional.leaky_relu default slope
    x = conv1d(x, weights["conv_post.weight"], weights["conv_post.bias"], padding=3)  # HF:1465
    return np.tanh(x)[:, 0]  # HF:1466


def vocoder_forward_batch(mels, mel_lens, weights, cfg=None, dtype=np.float32):
    """Ragged batch: each utterance b uses mels[b, :mel_lens[b]] independently (B=1 semantics)."""
    out = []
    for b in range(len(mel_lens)):
        out.append(vocoder_forward(mels[b, : int(mel_lens[b])], weights, cfg, dtype))
    return out
