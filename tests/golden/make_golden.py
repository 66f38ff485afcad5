"""Generate golden vectors for the oracle from transformers 5.15.0 (run HERE, CPU).

The reference's own model (`chatterbox`, un-vendored; `services/tts/core/
synthesizer.py:167,185`) is not available offline and the reference ships no
tests or fixtures.  The architecture named by the north star
is available in this container as transformers' `FastSpeech2ConformerModel` +
`FastSpeech2ConformerHifiGan`; this script loads the engine's deterministic
seeded weights (`gonova_tts_amd.weights`) into those modules and records small
input/output pairs, one utterance at a time (B=1; HF batches are not
padding-invariant, HF:1228-1229).

Output: tests/golden/golden_v1.npz (inputs, outputs, weight checksums).
Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from gonova_tts_amd.weights import make_vocoder_weights, make_acoustic_weights  # noqa: E402


def weight_checksums(w):
    names = sorted(w)
    return np.array([float(np.asarray(w[n], np.float64).sum()) for n in names]), np.array(names)


def main():
    from transformers import (FastSpeech2ConformerConfig, FastSpeech2ConformerHifiGanConfig,
                              FastSpeech2ConformerModel, FastSpeech2ConformerHifiGan)
    torch.manual_seed(0)
    out = {}

    # ---------------- vocoder ----------------
    vw = make_vocoder_weights(seed=0)
    voc = FastSpeech2ConformerHifiGan(FastSpeech2ConformerHifiGanConfig()).eval()
    voc.load_state_dict({k: torch.from_numpy(v) for k, v in vw.items()}, strict=True)
    rng = np.random.default_rng(1234)
    for tag, T in (("voc_a", 24), ("voc_b", 37)):
        mel = rng.standard_normal((T, 80)).astype(np.float32)
        with torch.no_grad():
            wav = voc(torch.from_numpy(mel)[None]).numpy()[0]
        out[f"{tag}_mel"] = mel
        out[f"{tag}_wav"] = wav.astype(np.float32)
    s, n = weight_checksums(vw)
    out["voc_weight_sums"], out["voc_weight_names"] = s, n

    # ---------------- acoustic ----------------
    aw = make_acoustic_weights(seed=0)
    ac = FastSpeech2ConformerModel(FastSpeech2ConformerConfig()).eval()
    sd = {k: torch.from_numpy(v) for k, v in aw.items()}
    # BatchNorm counters are not weights; keep HF's
    for k, v in ac.state_dict().items():
        if k.endswith("num_batches_tracked"):
            sd[k] = v
    ac.load_state_dict(sd, strict=True)
    for tag, L in (("ac_a", 12), ("ac_b", 23)):
        ids = rng.integers(1, 78, size=(L,)).astype(np.int64)
        with torch.no_grad():
            o = ac(torch.from_numpy(ids)[None], return_dict=True)
            enc = ac.encoder(torch.from_numpy(ids)[None], torch.ones(1, 1, L), return_dict=True).last_hidden_state
        out[f"{tag}_ids"] = ids
        out[f"{tag}_mel"] = o.spectrogram.numpy()[0].astype(np.float32)
        out[f"{tag}_dur"] = o.duration_outputs.numpy()[0].astype(np.int64)
        out[f"{tag}_pitch"] = o.pitch_outputs.numpy()[0, :, 0].astype(np.float32)
        out[f"{tag}_energy"] = o.energy_outputs.numpy()[0, :, 0].astype(np.float32)
        out[f"{tag}_enc"] = enc.numpy()[0].astype(np.float32)
    s, n = weight_checksums(aw)
    out["ac_weight_sums"], out["ac_weight_names"] = s, n

    # ---------------- end to end: tokens -> mel -> wav ----------------
    ids = out["ac_a_ids"]
    with torch.no_grad():
        mel = ac(torch.from_numpy(ids)[None], return_dict=True).spectrogram
        wav = voc(mel).numpy()[0]
    out["e2e_wav"] = wav.astype(np.float32)

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_v1.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items() if not k.endswith("names")})


if __name__ == "__main__":
    main()
