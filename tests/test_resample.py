"""Waveform resampler (22,050 -> 24,000 Hz for clients that assume the
reference's hard-coded 24 kHz, synthesizer.py:119 / queue_manager.py:40).

The reference has no resampler; the oracle (oracle/resample.py) restates
scipy.signal.resample_poly and is pinned here against scipy itself, and the HIP kernel
(tts_resample_poly) is checked against both on ragged batches."""
import numpy as np
import pytest
import scipy.signal as ss

from oracle.resample import design, resample_poly
from tests.conftest import gpu_available

RATIOS = [(160, 147), (147, 160), (2, 1), (1, 2), (3, 2), (24000, 16000)]


@pytest.mark.parametrize("up,down", RATIOS)
def test_oracle_matches_scipy_resample_poly(up, down):
    rng = np.random.default_rng(up * 7 + down)
    for n in (1, 7, 150, 2205, 5000):
        x = rng.standard_normal(n)  # float64: scipy keeps float32 input in float32
        ref = ss.resample_poly(x, up, down)
        got = resample_poly(x, up, down)
        assert got.shape == ref.shape
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)


@pytest.mark.parametrize("up,down", RATIOS)
def test_library_filter_design_matches_scipy_firwin(up, down):
    """tts_resample_filter (host-only C-ABI entry, the taps the kernel uses) == scipy's design."""
    from gonova_tts_amd.engine import resample_filter
    h, npr = resample_filter(up, down)
    ref, ref_npr = design(up, down)
    g = np.gcd(up, down)
    mr = max(up, down) // g
    fw = ss.firwin(2 * 10 * mr + 1, 1.0 / mr, window=("kaiser", 5.0)) * (up // g)
    assert npr == ref_npr and len(h) == len(ref)
    np.testing.assert_allclose(h, ref, rtol=0, atol=1e-14)
    np.testing.assert_allclose(h[len(h) - len(fw):], fw, rtol=0, atol=1e-14)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")
@pytest.mark.parametrize("up,down", [(160, 147), (147, 160), (1, 2), (3, 2)])
def test_hip_resampler_matches_scipy_on_ragged_batch(up, down):
    import torch
    from gonova_tts_amd.engine import HipEngine
    eng = HipEngine("cuda:0", vocoder_dtype="f16")
    rng = np.random.default_rng(5)
    lens = [22050, 1, 0, 4097, 300]
    S = max(lens)
    x = np.zeros((len(lens), S), np.float32)
    for b, L in enumerate(lens):
        x[b, :L] = 0.5 * rng.standard_normal(L)
        x[b, L:] = 7.0  # garbage past the length must not leak in
    out, out_lens = eng.resample(torch.from_numpy(x).cuda(), torch.tensor(lens, dtype=torch.int32), up, down)
    out, out_lens = out.cpu().numpy(), out_lens.cpu().numpy()
    for b, L in enumerate(lens):
        ref = ss.resample_poly(x[b, :L].astype(np.float64), up, down) if L else np.zeros(0)
        assert out_lens[b] == len(ref)
        err = np.abs(out[b, :len(ref)] - ref).max() if len(ref) else 0.0
        assert err <= 2e-6, (b, err)
        assert np.all(out[b, len(ref):] == 0)
