"""ctypes binding of libtts_hip.so (include/tts_hip.h) and the device-side engine handle.

This is the layer that replaces `ChatterboxTTS.from_pretrained(device=...)`
(`services/tts/core/synthesizer.py:185`): the engine is created on HIP device N
for a "cuda:N" string, weights are handed over by HF state_dict name, and the
forwards run the hand-written gfx950 kernels.  PyTorch-ROCm only allocates the
caller-owned input/output device buffers and provides the stream.

There is no CPU fallback: if the shared library is missing or no HIP device is
visible, construction raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from typing import Dict, Optional

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# TTS_LIB: load an A/B variant build (build.py --variant, tools/ab.sh) instead of the product library
LIB_PATH = os.environ.get("TTS_LIB") or os.path.join(_PKG, "libtts_hip.so")

DTYPES = {"f32": 0, "fp32": 0, "float32": 0, "f16": 1, "fp16": 1, "float16": 1, "bf16": 2, "bfloat16": 2}

TTS_ERRORS = {-1: "invalid argument", -2: "HIP error", -3: "bad state", -4: "out of memory"}


class TtsConfig(ctypes.Structure):
    _fields_ = [("vocoder_dtype", ctypes.c_int), ("acoustic_dtype", ctypes.c_int),
                ("max_batch", ctypes.c_int), ("max_frames", ctypes.c_int), ("max_tokens", ctypes.c_int),
                ("encoder_precision", ctypes.c_int)]


ENCODER_PRECISION = {"exact": 0, "fast": 1}
ENCODER_F32 = 2  # TTS_ENCODER_F32: run-time fallback of "exact" (tts_acoustic_set_precision)


class TtsConvDesc(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p), ("sxb", ctypes.c_int64), ("sxr", ctypes.c_int32), ("x_len", ctypes.c_void_p),
        ("x_rows", ctypes.c_int32),
        ("w", ctypes.c_void_p), ("swb", ctypes.c_int64), ("w_ld", ctypes.c_int32),
        ("bias", ctypes.c_void_p),
        ("y", ctypes.c_void_p), ("syb", ctypes.c_int64), ("syr", ctypes.c_int32),
        ("r1", ctypes.c_void_p), ("r2", ctypes.c_void_p), ("srb", ctypes.c_int64), ("srr", ctypes.c_int32),
        ("y_len", ctypes.c_void_p), ("y_rows", ctypes.c_int32),
        ("M", ctypes.c_int32), ("Cin", ctypes.c_int32), ("taps", ctypes.c_int32), ("dil", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("in_slope", ctypes.c_float), ("act_out", ctypes.c_int32), ("out_slope", ctypes.c_float),
        ("alpha", ctypes.c_float), ("out_scale", ctypes.c_float),
        ("up_s", ctypes.c_int32), ("up_cout", ctypes.c_int32), ("up_p", ctypes.c_int32),
        ("up_len", ctypes.c_void_p),
        ("B", ctypes.c_int32),
    ]


# every function declared in include/tts_hip.h: (name, restype, argtypes)
_VP, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
C_API = [
    ("tts_device_count", _I, []),
    ("tts_abi_version", _I, []),
    ("tts_device_bytes", _I, [_I, ctypes.POINTER(ctypes.c_int64)]),
    ("tts_engine_create", _I, [_I, ctypes.POINTER(TtsConfig), ctypes.POINTER(_VP)]),
    ("tts_engine_create_sized", _I, [_I, ctypes.POINTER(TtsConfig), ctypes.c_size_t, ctypes.POINTER(_VP)]),
    ("tts_engine_set_weight", _I, [_VP, ctypes.c_char_p, _VP, ctypes.POINTER(ctypes.c_int64), _I]),
    ("tts_engine_finalize", _I, [_VP]),
    ("tts_engine_reserve", _I, [_VP, _I, _I, _I]),
    ("tts_engine_destroy", None, [_VP]),
    ("tts_vocoder_forward", _I, [_VP, _VP, _VP, _I, _I, _VP, _VP]),
    ("tts_vocoder_forward_chunk", _I, [_VP, _VP, _VP, _I, _I, _I, _I, _VP, _VP]),
    ("tts_acoustic_forward", _I, [_VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _I, _VP, _VP]),
    ("tts_acoustic_forward_spk", _I, [_VP, _VP, _VP, _I, _I, _VP, _VP, _I, _VP, _VP, _I, _VP, _VP]),
    ("tts_acoustic_speaker_dim", _I, [_VP, ctypes.POINTER(ctypes.c_int)]),
    ("tts_acoustic_range_flag", _I, [_VP, _VP, _VP]),
    ("tts_acoustic_set_precision", _I, [_VP, _I]),
    ("tts_engine_profile", _I, [_VP, _I]),
    ("tts_engine_profile_read", _I, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_int)]),
    ("tts_engine_profile_read_kinds", _I, [_VP, _I, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    ("tts_resample_poly", _I, [_VP, _VP, ctypes.c_int64, _VP, _I, _I, _I, _VP, ctypes.c_int64, _I, _VP, _VP]),
    ("tts_resample_filter", _I, [_I, _I, ctypes.POINTER(ctypes.c_double), _I, ctypes.POINTER(ctypes.c_int)]),
    ("tts_set_switch", _I, [ctypes.c_char_p, _I]),
    ("tts_get_switch", _I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    ("tts_last_error", ctypes.c_char_p, []),
    ("tts_op_conv1d", _I, [_I, ctypes.POINTER(TtsConvDesc), _VP]),
]

_lib = None
_lib_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load libtts_hip.so (no GPU needed); raises if it has not been built."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not found: build it with `python -m gonova_tts_amd.build` "
                               "(there is no CPU fallback)")
        lib = ctypes.CDLL(path)
        for name, res, args in C_API:
            # (an older A/B build may lack a newer entry point: it is left unbound, and a call to
            # it raises AttributeError; tests/test_capi.py checks the product library has them all)
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def resample_filter(up: int, down: int):
    """Host-side filter design of tts_resample_poly (no GPU): (taps float64, n_pre_remove)."""
    lib = load_library()
    npr = ctypes.c_int()
    n = lib.tts_resample_filter(up, down, None, 0, ctypes.byref(npr))
    if n < 0:
        check(n, "tts_resample_filter")
    h = (ctypes.c_double * n)()
    lib.tts_resample_filter(up, down, h, n, ctypes.byref(npr))
    import numpy as _np
    return _np.frombuffer(h, dtype=_np.float64).copy(), npr.value


def device_bytes(device=0) -> int:
    """Bytes of device memory libtts_hip.so holds on a HIP device (all engines' weights and
    workspaces; include/tts_hip.h tts_device_bytes).  A host-side count: no GPU work."""
    lib = load_library()
    out = ctypes.c_int64()
    check(lib.tts_device_bytes(parse_device(device) if not isinstance(device, int) else device, ctypes.byref(out)),
          "tts_device_bytes")
    return int(out.value)


def set_switch(name: str, value: int = -1):
    """Select an alternative kernel path process-wide (include/tts_hip.h tts_set_switch):
    e.g. set_switch("TTS_REL_ATTN", 0) for the unfused attention; -1 restores the default."""
    lib = load_library()
    check(lib.tts_set_switch(name.encode(), int(value)), "tts_set_switch")


def get_switch(name: str) -> int:
    """Current value of a kernel-path switch (its environment value or the last set_switch;
    -1 = not set, the built-in default)."""
    lib = load_library()
    v = ctypes.c_int()
    check(lib.tts_get_switch(name.encode(), ctypes.byref(v)), "tts_get_switch")
    return v.value


@contextlib.contextmanager
def switches(**values):
    """Context manager form of set_switch: `with switches(TTS_MRF_CHAIN=0): ...`; every named
    switch goes back to the value it had before (e.g. one set in the environment) on exit."""
    saved = {k: get_switch(k) for k in values}
    try:
        for k, v in values.items():
            set_switch(k, v)
        yield
    finally:
        for k, v in saved.items():
            set_switch(k, v)


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load_library().tts_last_error()
        msg = msg.decode() if msg else ""
        raise RuntimeError(f"{what}: {TTS_ERRORS.get(rc, rc)}: {msg}")


def parse_device(device) -> int:
    """Map a reference-style device string ("cuda", "cuda:N", int) to a HIP ordinal."""
    if isinstance(device, int):
        return device
    s = str(device)
    if s in ("cuda", "hip", "gpu"):
        return 0
    if s.startswith(("cuda:", "hip:")):
        return int(s.split(":", 1)[1])
    raise ValueError(f"unsupported device {device!r}: the engine runs on HIP devices only")


def _stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class HipEngine:
    """Device-side TTS engine (one per HIP device)."""

    def __init__(self, device=0, vocoder_dtype: str = "f16", acoustic_dtype: str = "bf16",
                 max_batch: int = 0, max_frames: int = 0, max_tokens: int = 0, encoder_precision: str = "exact"):
        """encoder_precision: "exact" (default) keeps the acoustic encoder and variance predictors in
        fp32 (GEMMs as three f16 MFMAs) so predicted integer durations match fp32; "fast" runs them
        in acoustic_dtype like the decoder (include/tts_hip.h, TTS_ENCODER_*)."""
        import torch
        self.lib = load_library()
        if not torch.cuda.is_available():
            raise RuntimeError("no HIP device visible: gonova_tts_amd has no CPU path")
        self.device_index = parse_device(device)
        self.torch_device = torch.device("cuda", self.device_index)
        self.vocoder_dtype = vocoder_dtype
        self.acoustic_dtype = acoustic_dtype
        self.encoder_precision = encoder_precision
        cfg = TtsConfig(DTYPES[vocoder_dtype], DTYPES[acoustic_dtype], max_batch, max_frames, max_tokens,
                        ENCODER_PRECISION[encoder_precision])
        h = ctypes.c_void_p()
        check(self.lib.tts_engine_create_sized(self.device_index, ctypes.byref(cfg), ctypes.sizeof(cfg),
                                               ctypes.byref(h)), "tts_engine_create")
        self.handle = h
        # range guard of the exact encoder of a 16-bit model (include/tts_hip.h, ABI 4): every
        # acoustic forward also enqueues a copy of the engine's range word, which the caller reads
        # at its next host sync (GonovaTTS) and answers with an fp32-MFMA rerun when it is set
        # the exact encoder's split-precision GEMMs (16-bit models; fp32 models too unless
        # TTS_F32_ENC_SPLIT=0) report activations outside f16's range in a word read back with the
        # lengths; a set word reruns the batch on the fp32 encoder (model.py)
        self.range_guard = encoder_precision == "exact" and (DTYPES[acoustic_dtype] != 0 or
                                                             get_switch("TTS_F32_ENC_SPLIT") != 0)
        self.range_fallbacks = 0
        self.hop = 256
        self._finalized = False
        self.has_vocoder = False
        self.has_acoustic = False

    # ------------------------------------------------------------------ weights
    def set_weight(self, name: str, arr):
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
        shape = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
        check(self.lib.tts_engine_set_weight(self.handle, name.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                             shape, a.ndim), f"set_weight({name})")

    def load_weights(self, vocoder: Optional[Dict[str, np.ndarray]] = None,
                     acoustic: Optional[Dict[str, np.ndarray]] = None, vocoder_cfg=None):
        if vocoder is not None:
            from .config import VocoderConfig
            vc = vocoder_cfg or VocoderConfig()
            for k, v in vocoder.items():
                self.set_weight(k, v)
            self.set_weight("__cfg__.upsample_rates", np.asarray(vc.upsample_rates, np.float32))
            self.set_weight("__cfg__.resblock_dilation_sizes", np.asarray(vc.resblock_dilation_sizes, np.float32))
            self.hop = vc.hop
            self.has_vocoder = True
        if acoustic is not None:
            for k, v in acoustic.items():
                if k.endswith("num_batches_tracked"):
                    continue
                self.set_weight(k, v)
            self.has_acoustic = True
        check(self.lib.tts_engine_finalize(self.handle), "finalize")
        self._finalized = True

    def reserve(self, max_batch: int, max_frames: int, max_tokens: int = 0):
        check(self.lib.tts_engine_reserve(self.handle, max_batch, max_frames, max_tokens), "reserve")

    # ------------------------------------------------------------------ forwards
    def vocoder(self, mel, mel_lens=None, out=None, stream=None):
        """mel: cuda float32 [B, T, 80]; mel_lens: cuda int32 [B] -> wav cuda float32 [B, T*hop]."""
        import torch
        assert mel.is_cuda and mel.dtype == torch.float32 and mel.dim() == 3
        mel = mel.contiguous()
        B, T, _ = mel.shape
        if mel_lens is None:
            mel_lens = torch.full((B,), T, dtype=torch.int32, device=mel.device)
        mel_lens = mel_lens.to(device=mel.device, dtype=torch.int32).contiguous()
        if out is None:
            out = torch.empty((B, T * self.hop), dtype=torch.float32, device=mel.device)
        check(self.lib.tts_vocoder_forward(self.handle, ctypes.c_void_p(mel.data_ptr()),
                                           ctypes.c_void_p(mel_lens.data_ptr()), B, T,
                                           ctypes.c_void_p(out.data_ptr()), _stream_ptr(stream)),
              "tts_vocoder_forward")
        return out

    def vocoder_chunk(self, mel_win, win_lens, ctx_left: int, t_chunk: int, out=None, stream=None):
        import torch
        mel_win = mel_win.contiguous()
        B, Tw, _ = mel_win.shape
        win_lens = win_lens.to(device=mel_win.device, dtype=torch.int32).contiguous()
        if out is None:
            out = torch.empty((B, t_chunk * self.hop), dtype=torch.float32, device=mel_win.device)
        check(self.lib.tts_vocoder_forward_chunk(self.handle, ctypes.c_void_p(mel_win.data_ptr()),
                                                 ctypes.c_void_p(win_lens.data_ptr()), B, Tw, ctx_left, t_chunk,
                                                 ctypes.c_void_p(out.data_ptr()), _stream_ptr(stream)),
              "tts_vocoder_forward_chunk")
        return out

    def resample(self, wav, lens, up: int, down: int, out=None, stream=None):
        """Per-utterance rational resampling on the device (scipy.signal.resample_poly(x, up,
        down) semantics): wav cuda float32 [B, S], lens (valid samples) [B] ->
        (out cuda float32 [B, ceil(S*up/down)], out_lens cuda int32 [B])."""
        import torch
        assert wav.is_cuda and wav.dtype == torch.float32 and wav.dim() == 2
        wav = wav.contiguous()
        B, S = wav.shape
        lens = torch.as_tensor(lens).to(device=wav.device, dtype=torch.int32).contiguous()
        cap = max(1, -(-S * up // down))
        if out is None:
            out = torch.empty((B, cap), dtype=torch.float32, device=wav.device)
        out_lens = torch.empty((B,), dtype=torch.int32, device=wav.device)
        check(self.lib.tts_resample_poly(self.handle, ctypes.c_void_p(wav.data_ptr()), S,
                                         ctypes.c_void_p(lens.data_ptr()), B, up, down,
                                         ctypes.c_void_p(out.data_ptr()), out.shape[1], cap,
                                         ctypes.c_void_p(out_lens.data_ptr()), _stream_ptr(stream)),
              "tts_resample_poly")
        return out, out_lens

    @property
    def speaker_dim(self) -> int:
        """Speaker-embedding size of the loaded acoustic model (0: single speaker)."""
        d = ctypes.c_int()
        check(self.lib.tts_acoustic_speaker_dim(self.handle, ctypes.byref(d)), "tts_acoustic_speaker_dim")
        return d.value

    def set_encoder_precision(self, precision: str):
        """"exact" (split-precision, the default) or "f32" (exact fp32 MFMA: the range guard's
        fallback) for later acoustic forwards of a 16-bit model created with "exact"."""
        code = {"exact": ENCODER_PRECISION["exact"], "f32": ENCODER_F32}[precision]
        check(self.lib.tts_acoustic_set_precision(self.handle, code), "tts_acoustic_set_precision")

    @contextlib.contextmanager
    def encoder_f32(self):
        """Acoustic forwards inside the block run the encoder on the fp32 MFMA path."""
        self.set_encoder_precision("f32")
        try:
            yield
        finally:
            self.set_encoder_precision("exact")

    def acoustic(self, tokens, tok_lens, t_cap: int, durations=None, stream=None, return_durations=False,
                 speaker_embedding=None, return_range=False):
        """tokens: cuda int32 [B, N]; returns (mel [B, t_cap, 80] f32, mel_lens int32 [B]).
        speaker_embedding: optional float32 [B, E] (HF:1192-1196), E = speaker_dim.
        return_range: also return the range word of this forward (cuda int32 [1], nonzero when a
        split-precision operand was outside f16's range; None without the guard), enqueued on the
        same stream -- read it at the next host sync."""
        import torch
        tokens = tokens.to(dtype=torch.int32).contiguous()
        tok_lens = tok_lens.to(device=tokens.device, dtype=torch.int32).contiguous()
        B, N = tokens.shape
        # (every row is written: the frames past each utterance's length as zeros, mel_out_kernel)
        mel = torch.empty((B, t_cap, 80), dtype=torch.float32, device=tokens.device)
        # the integer outputs (durations, frame counts, range word) are views of one int32 block at
        # 64-byte aligned offsets, so a caller reads them back with one copy (model._HostRead)
        o_len = -(-B * N // 16) * 16
        o_rw = o_len + -(-B // 16) * 16
        meta = torch.empty((o_rw + 16,), dtype=torch.int32, device=tokens.device)
        dur_out = meta[:B * N].view(B, N)
        mel_lens = meta[o_len:o_len + B]
        dptr = ctypes.c_void_p(0)
        if durations is not None:
            durations = durations.to(device=tokens.device, dtype=torch.int32).contiguous()
            dptr = ctypes.c_void_p(durations.data_ptr())
        sptr, sdim = ctypes.c_void_p(0), 0
        if speaker_embedding is not None:
            speaker_embedding = torch.as_tensor(speaker_embedding, dtype=torch.float32).to(tokens.device)
            speaker_embedding = speaker_embedding.reshape(B, -1).contiguous()
            sptr, sdim = ctypes.c_void_p(speaker_embedding.data_ptr()), speaker_embedding.shape[1]
        check(self.lib.tts_acoustic_forward_spk(self.handle, ctypes.c_void_p(tokens.data_ptr()),
                                                ctypes.c_void_p(tok_lens.data_ptr()), B, N, dptr, sptr, sdim,
                                                ctypes.c_void_p(mel.data_ptr()), ctypes.c_void_p(mel_lens.data_ptr()),
                                                t_cap, ctypes.c_void_p(dur_out.data_ptr()), _stream_ptr(stream)),
              "tts_acoustic_forward")
        rw = None
        # the word is copied out and cleared only for a caller that reads it: otherwise it keeps
        # accumulating, so the next caller that asks sees an earlier unread overflow too (a spurious
        # fp32 rerun at worst, never a lost one)
        if self.range_guard and return_range:
            rw = meta[o_rw:o_rw + 1]
            check(self.lib.tts_acoustic_range_flag(self.handle, ctypes.c_void_p(rw.data_ptr()), _stream_ptr(stream)),
                  "tts_acoustic_range_flag")
        out = (mel, mel_lens, dur_out) if return_durations else (mel, mel_lens)
        return out + (rw,) if return_range else out

    def profile(self, enable: bool = True):
        check(self.lib.tts_engine_profile(self.handle, int(enable)), "profile")

    def profile_read(self):
        """-> (summed implicit-GEMM kernel ms, their algorithmic FLOPs, launch count); resets."""
        ms, fl, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        check(self.lib.tts_engine_profile_read(self.handle, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(n)),
              "profile_read")
        return ms.value, fl.value, n.value

    PROFILE_KINDS = ("conv_gemm_kernel", "conv_xres_kernel", "retired", "mrf_pair_kernel", "mrf_chain_kernel",
                     "upsample_stream_kernel", "conv_split_kernel", "rel_attn_kernel", "acoustic_elementwise")

    def profile_read_kinds(self):
        """-> {kernel name: (summed ms, algorithmic FLOPs, launch count)}; resets."""
        k = len(self.PROFILE_KINDS)
        ms, fl, n = (ctypes.c_double * k)(), (ctypes.c_double * k)(), (ctypes.c_int * k)()
        check(self.lib.tts_engine_profile_read_kinds(self.handle, k, ms, fl, n), "profile_read_kinds")
        return {name: (ms[i], fl[i], n[i]) for i, name in enumerate(self.PROFILE_KINDS)}

    def close(self):
        if getattr(self, "handle", None):
            self.lib.tts_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def conv1d_op(dtype: str, desc: TtsConvDesc, stream=None):
    lib = load_library()
    check(lib.tts_op_conv1d(DTYPES[dtype], ctypes.byref(desc), _stream_ptr(stream)), "tts_op_conv1d")
