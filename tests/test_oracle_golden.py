"""Pin the CPU oracle against golden vectors produced by transformers 5.15.0
(tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from gonova_tts_amd.weights import make_vocoder_weights, make_acoustic_weights
from oracle.vocoder import vocoder_forward
from oracle.acoustic import acoustic_forward

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))


def test_weight_generator_is_pinned():
    for key, fn in (("voc", make_vocoder_weights), ("ac", make_acoustic_weights)):
        w = fn(seed=0)
        names = list(G[f"{key}_weight_names"])
        assert sorted(w) == names
        sums = np.array([float(np.asarray(w[n], np.float64).sum()) for n in names])
        np.testing.assert_allclose(sums, G[f"{key}_weight_sums"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("tag", ["voc_a", "voc_b"])
def test_vocoder_oracle_matches_golden(tag):
    w = make_vocoder_weights(seed=0)
    wav = vocoder_forward(G[f"{tag}_mel"], w)
    assert wav.shape == G[f"{tag}_wav"].shape
    np.testing.assert_allclose(wav, G[f"{tag}_wav"], atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("tag", ["ac_a", "ac_b"])
def test_acoustic_oracle_matches_golden(tag):
    w = make_acoustic_weights(seed=0)
    o = acoustic_forward(G[f"{tag}_ids"], w)
    np.testing.assert_array_equal(o["durations"], G[f"{tag}_dur"])
    np.testing.assert_allclose(o["pitch"], G[f"{tag}_pitch"], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(o["energy"], G[f"{tag}_energy"], atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(o["mel"], G[f"{tag}_mel"], atol=1e-4, rtol=1e-4)


def test_end_to_end_oracle_matches_golden():
    o = acoustic_forward(G["ac_a_ids"], make_acoustic_weights(seed=0))
    wav = vocoder_forward(o["mel"], make_vocoder_weights(seed=0))
    np.testing.assert_allclose(wav, G["e2e_wav"], atol=1e-5, rtol=1e-4)


GS = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_spk.npz"))


@pytest.mark.parametrize("tag", ["spk_a", "spk_b"])
def test_speaker_embedding_oracle_matches_golden(tag):
    """Speaker-embedding conditioning (HF:1192-1196; tests/golden/make_spk_golden.py)."""
    from gonova_tts_amd.config import AcousticConfig
    from gonova_tts_amd.weights import make_acoustic_weights
    w = make_acoustic_weights(0, AcousticConfig(speaker_embed_dim=64))
    o = acoustic_forward(GS[f"{tag}_ids"], w, speaker_embedding=GS[f"{tag}_emb"])
    np.testing.assert_array_equal(o["durations"], GS[f"{tag}_dur"])
    np.testing.assert_allclose(o["mel"], GS[f"{tag}_mel"], atol=1e-4, rtol=1e-4)
    o0 = acoustic_forward(GS[f"{tag}_ids"], w)  # no embedding: HF skips the projection
    np.testing.assert_allclose(o0["mel"], GS[f"{tag}_mel_nospk"], atol=1e-4, rtol=1e-4)


def test_torch_cpu_restatement_matches_golden_and_numpy_oracle():
    """oracle/torch_cpu.py (bench.py's timed CPU baseline) against the
    transformers goldens and the NumPy oracle: vocoder batch, acoustic with forced and with
    predicted durations."""
    import torch
    from oracle.torch_cpu import TorchAcoustic, TorchVocoder
    vw, aw = make_vocoder_weights(seed=0), make_acoustic_weights(seed=0)
    voc, ac = TorchVocoder(vw), TorchAcoustic(aw)
    for tag in ("voc_a", "voc_b"):
        wav = voc(torch.from_numpy(G[f"{tag}_mel"])[None])[0].numpy()
        np.testing.assert_allclose(wav, G[f"{tag}_wav"], atol=1e-5, rtol=1e-4)
    mel, dur = ac(torch.from_numpy(np.asarray(G["ac_a_ids"], np.int64))[None])
    np.testing.assert_array_equal(dur[0].numpy(), G["ac_a_dur"])
    np.testing.assert_allclose(mel[0].numpy(), G["ac_a_mel"], atol=1e-4, rtol=1e-4)
    rng = np.random.default_rng(5)
    ids = rng.integers(1, 78, size=(2, 9))
    d = np.full((2, 9), 2)
    mel, _ = ac(torch.from_numpy(ids), torch.from_numpy(d))
    for b in range(2):
        ref = acoustic_forward(ids[b], aw, durations=d[b])["mel"]
        np.testing.assert_allclose(mel[b].numpy(), ref, atol=1e-4, rtol=1e-4)
