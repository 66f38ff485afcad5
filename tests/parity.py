"""Error metrics shared by the GPU parity tests, and a log of every measured error.

Each parity test calls `check(name, got, ref, rel_rms_tol=..., max_abs_tol=...)`: it computes
the relative RMS error and the max absolute error against the reference, records both with
the tolerance (printed, and written as JSON to $PARITY_LOG at the end of the session, see
conftest.py) and asserts them.  Tolerances sit at about 2x the values measured on MI355X
(profiles/r04_parity_errors.json), so an error regression of 2x fails."""
import numpy as np

RECORDS = []

# (rel_rms, max_abs) bounds per path, re-derived each round from the largest errors the GPU suite
# measured (profiles/r04_parity_errors.json, round 4: fp16 vocoder 1.62e-3 / 4.0e-4, bf16 vocoder
# 8.9e-3 / 2.0e-3, fp16 acoustic mel 1.26e-3 / 5.9e-3, bf16 acoustic mel 1.02e-2 / 5.0e-2, bf16
# tokens -> waveform 1.46e-2 / 3.2e-3; waveform rms ~0.045, mel rms ~1.0): about 2x, the
# end-to-end bf16 bound at 1.7x (SURVEY.md §8c's recommended bars: fp16 5e-3, bf16 2.5e-2 rel-RMS).
TOL = {
    "voc_f16": (3.2e-3, 8e-4),
    "voc_bf16": (1.8e-2, 4e-3),
    "ac_f16": (2.5e-3, 1.2e-2),
    "ac_bf16": (2e-2, 0.1),
    "e2e_bf16": (2.5e-2, 6.5e-3),
}


def rel_rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / (np.sqrt(np.mean(b ** 2)) + 1e-30))


def max_abs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max()) if np.size(a) else 0.0


def check(name, got, ref, rel_rms_tol=None, max_abs_tol=None, kind=None):
    """kind: a TOL key supplying both bounds."""
    if kind is not None:
        rel_rms_tol, max_abs_tol = TOL[kind]
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    assert np.isfinite(got).all(), name
    e, m = rel_rms(got, ref), max_abs(got, ref)
    RECORDS.append({"name": name, "rel_rms": e, "max_abs": m, "rel_rms_tol": rel_rms_tol,
                    "max_abs_tol": max_abs_tol, "ref_rms": float(np.sqrt(np.mean(np.asarray(ref, np.float64) ** 2)))})
    print(f"[parity] {name}: rel_rms {e:.3e} (tol {rel_rms_tol}), max_abs {m:.3e} (tol {max_abs_tol})")
    if rel_rms_tol is not None:
        assert e <= rel_rms_tol, (name, "rel_rms", e, rel_rms_tol)
    if max_abs_tol is not None:
        assert m <= max_abs_tol, (name, "max_abs", m, max_abs_tol)
    return e, m
