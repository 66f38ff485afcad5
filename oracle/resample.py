"""CPU oracle for the waveform resampler -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product path (gonova-tts_amd/csrc/resample.hip via tts_resample_poly) never does.

Restates scipy.signal.resample_poly(x, up, down) (scipy 1.15.3, signal/_signaltools.py,
default window ('kaiser', 5.0), padtype 'constant') as an explicit polyphase sum in float64:
  h  = firwin(2*half_len + 1, 1/max(up, down), window) * up,  half_len = 10 * max(up, down)
  h' = [zeros(n_pre_pad), h],  n_pre_pad = down - half_len % down
  y[m] = sum_k h'[k] * xu[(m + n_pre_remove) * down - k],  n_pre_remove = (half_len + n_pre_pad) // down
  (xu = x upsampled by zero insertion), m < ceil(len(x) * up / down).
Pinned against scipy.signal.resample_poly itself in tests/test_resample.py (the reference
repository has no resampler; the 24 kHz rate it assumes is synthesizer.py:119).
"""
from math import gcd

import numpy as np


def design(up: int, down: int):
    """(padded taps float64, n_pre_remove) with NumPy's Kaiser window (== scipy's symmetric one)."""
    g = gcd(up, down)
    up, down = up // g, down // g
    max_rate = max(up, down)
    fc = 1.0 / max_rate
    half_len = 10 * max_rate
    n = 2 * half_len + 1
    m = np.arange(n) - 0.5 * (n - 1)
    h = fc * np.sinc(fc * m) * np.kaiser(n, 5.0)
    h = h / h.sum() * up
    n_pre_pad = down - half_len % down
    return np.concatenate([np.zeros(n_pre_pad), h]), (half_len + n_pre_pad) // down


def resample_poly(x: np.ndarray, up: int, down: int) -> np.ndarray:
    g = gcd(up, down)
    up, down = up // g, down // g
    x = np.asarray(x, np.float64)
    h, n_pre_remove = design(up, down)
    n_in = len(x)
    n_out = -(-n_in * up // down)
    nq = -(-len(h) // up)
    hp = np.zeros((up, nq))
    for k in range(len(h)):
        hp[k % up, k // up] = h[k]
    m = np.arange(n_out)
    t = (m + n_pre_remove) * down
    ph, base = t % up, t // up
    y = np.zeros(n_out)
    for q in range(nq):
        i = base - q
        ok = (i >= 0) & (i < n_in)
        y[ok] += hp[ph[ok], q] * x[i[ok]]
    return y
