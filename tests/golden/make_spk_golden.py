"""Golden vectors for speaker-embedding conditioning, from
transformers 5.15.0 `FastSpeech2ConformerModel` with `speaker_embed_dim=64`
(HF:1051-1053, 1192-1196), run HERE on CPU with the engine's seeded weights.

Output: tests/golden/golden_spk.npz -- two utterances (token ids, a speaker embedding, mel,
durations), plus the same tokens without an embedding (HF then skips the projection).
Usage:  python tests/golden/make_spk_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from gonova_tts_amd.config import AcousticConfig  # noqa: E402
from gonova_tts_amd.weights import make_acoustic_weights  # noqa: E402

E = 64


def main():
    from transformers import FastSpeech2ConformerConfig, FastSpeech2ConformerModel
    torch.manual_seed(0)
    aw = make_acoustic_weights(seed=0, cfg=AcousticConfig(speaker_embed_dim=E))
    ac = FastSpeech2ConformerModel(FastSpeech2ConformerConfig(speaker_embed_dim=E)).eval()
    sd = {k: torch.from_numpy(v) for k, v in aw.items()}
    for k, v in ac.state_dict().items():
        if k.endswith("num_batches_tracked"):
            sd[k] = v
    ac.load_state_dict(sd, strict=True)
    rng = np.random.default_rng(4321)
    out = {}
    for tag, L in (("spk_a", 11), ("spk_b", 19)):
        ids = rng.integers(1, 78, size=(L,)).astype(np.int64)
        emb = (3.0 * rng.standard_normal(E)).astype(np.float32)  # not unit norm: normalize matters
        with torch.no_grad():
            o = ac(torch.from_numpy(ids)[None], speaker_embedding=torch.from_numpy(emb)[None], return_dict=True)
            o0 = ac(torch.from_numpy(ids)[None], return_dict=True)
        out[f"{tag}_ids"] = ids
        out[f"{tag}_emb"] = emb
        out[f"{tag}_mel"] = o.spectrogram.numpy()[0].astype(np.float32)
        out[f"{tag}_dur"] = o.duration_outputs.numpy()[0].astype(np.int64)
        out[f"{tag}_mel_nospk"] = o0.spectrogram.numpy()[0].astype(np.float32)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_spk.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
