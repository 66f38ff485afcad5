"""CPU checks of the C-ABI boundary: libtts_hip.so loads and exports every symbol
include/tts_hip.h declares (no compute calls; no GPU needed)."""
import os
import re

import pytest

from gonova_tts_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "tts_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tts_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    decl = declared_functions()
    bound = sorted(n for n, _, _ in engine.C_API)
    assert decl == bound


def test_library_exports_every_declared_symbol():
    if not os.path.exists(engine.LIB_PATH):
        from gonova_tts_amd.build import build
        build()
    lib = engine.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_parse_device():
    assert engine.parse_device("cuda:3") == 3
    assert engine.parse_device("cuda") == 0
    with pytest.raises(ValueError):
        engine.parse_device("cpu")


def test_switches_set_and_reset_without_gpu():
    """tts_set_switch needs no device: known switches accept a value and -1 (default); an
    unknown name is an error with a message."""
    engine.set_switch("TTS_MRF_CHAIN", 0)
    engine.set_switch("TTS_MRF_CHAIN", -1)
    with engine.switches(TTS_PAIR_DIV=1, TTS_REL_ATTN=0):
        pass
    with pytest.raises(RuntimeError, match="unknown switch"):
        engine.set_switch("TTS_NO_SUCH_SWITCH", 1)


def test_stream_mel_lens_host_matches_duration_rules():
    """stream_tokens computes frame counts on the host when durations are given (no sync before
    the first chunk); the rules are the durations kernel's: tokens past the length and negative
    durations count 0, an utterance whose durations are all 0 gets one frame per token, and the
    count is clamped to the frame cap."""
    import numpy as np
    from gonova_tts_amd.model import _mel_lens_host
    lens = np.array([3, 2, 0, 4])
    dur = np.array([[2, 3, 1, 9],      # 9 is past the length
                    [0, 0, 5, 5],      # all zero within the length -> one frame per token
                    [4, 4, 4, 4],      # empty utterance
                    [-1, 6, 6, 6]])    # negative counts 0; 18 clamped to the cap
    np.testing.assert_array_equal(_mel_lens_host(lens, dur, t_cap=16), [6, 2, 0, 16])


def test_abi_version_and_sized_config_without_gpu():
    """tts_config grows by appending fields; tts_engine_create_sized reads only the caller's
    bytes (advisor finding: a five-int ABI-1 struct made the engine read past it).  Config
    validation runs before the device lookup, so the rejections are checkable on the CPU."""
    import ctypes
    lib = engine.load_library()
    assert lib.tts_abi_version() == 5
    cfg = engine.TtsConfig(1, 2, 0, 0, 0, 0)
    h = ctypes.c_void_p()
    # a struct larger than the library's: a newer header than this library
    rc = lib.tts_engine_create_sized(0, ctypes.byref(cfg), ctypes.sizeof(cfg) + 4, ctypes.byref(h))
    assert rc == -1 and b"newer than this library" in lib.tts_last_error()
    # a size that is not a whole number of int fields
    rc = lib.tts_engine_create_sized(0, ctypes.byref(cfg), 10, ctypes.byref(h))
    assert rc == -1 and b"whole number" in lib.tts_last_error()
    # an ABI-1 five-int struct whose sixth int would be garbage: only 20 bytes are read, so the
    # garbage never reaches validation (the call then fails only for want of a device here)
    bad = engine.TtsConfig(1, 2, 0, 0, 0, 12345)
    rc = lib.tts_engine_create_sized(0, ctypes.byref(bad), 20, ctypes.byref(h))
    assert b"encoder_precision" not in lib.tts_last_error()
    rc = lib.tts_engine_create_sized(0, ctypes.byref(bad), ctypes.sizeof(bad), ctypes.byref(h))
    assert rc == -1 and b"bad encoder_precision" in lib.tts_last_error()


def test_switches_restore_the_previous_value():
    """switches() and the conftest fixture put back the value a switch had (an environment
    setting such as TTS_MRF_CHAIN=0 from tools/ab.sh), not the built-in default."""
    engine.set_switch("TTS_MRF_CHAIN", 0)  # stands in for an environment value
    try:
        with engine.switches(TTS_MRF_CHAIN=1, TTS_PAIR_DIV=4):
            assert engine.get_switch("TTS_MRF_CHAIN") == 1
            assert engine.get_switch("TTS_PAIR_DIV") == 4
        assert engine.get_switch("TTS_MRF_CHAIN") == 0
        assert engine.get_switch("TTS_PAIR_DIV") == -1
    finally:
        engine.set_switch("TTS_MRF_CHAIN", -1)
    with pytest.raises(RuntimeError, match="unknown switch"):
        engine.get_switch("TTS_NO_SUCH_SWITCH")
