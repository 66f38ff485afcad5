"""Drop-in model for the reference's synthesis call site.

The reference constructs its model with `ChatterboxTTS.from_pretrained(device=...)`
(`services/tts/core/synthesizer.py:185`) and calls
`model.generate(text, audio_prompt_path=..., exaggeration=..., cfg_weight=0.5,
temperature=0.8)` (`synthesizer.py:344-350`), then `audio.squeeze().cpu().numpy()`
and a float32 cast (`:352-357`).  `GonovaTTS` keeps exactly that duck-typed surface
 and adds `generate_batch` for many sentences at once.

Semantics of the extra arguments: the FastSpeech2 + HiFi-GAN pipeline is
deterministic and has no voice cloning, so `audio_prompt_path`, `exaggeration`,
`cfg_weight` and `temperature` are accepted and ignored (the reference forwards a
possibly unsanitised path, `voice_manager.py:166-177`; it is never opened here).
Output rate is `self.sr` = 22,050 Hz (the reference hard-codes 24 kHz,
`synthesizer.py:119`).
"""
from __future__ import annotations

import os
import threading
from contextlib import contextmanager, nullcontext
from math import gcd
from typing import Dict, List, Optional

import numpy as np

from .config import AcousticConfig, VocoderConfig, SAMPLE_RATE
from .engine import HipEngine
from .text import tokenize_batch
from .weights import make_acoustic_weights, make_vocoder_weights


def fold_weight_norm(sd: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Fold weight-normalised convolutions into plain weights.

    HiFi-GAN checkpoints are often saved with torch weight norm on (HF's
    `apply_weight_norm`): `<name>.weight_g` / `<name>.weight_v` (torch.nn.utils.weight_norm)
    or `<name>.parametrizations.weight.original0` / `.original1` (the parametrization API).
    Both store w = g * v / ||v|| with the norm over every dim but 0 (torch's default
    dim=0, which HF uses for Conv1d and ConvTranspose1d alike); the result is written
    as `<name>.weight` and the g/v entries are dropped."""
    out = dict(sd)
    pairs = []
    for k in sd:
        if k.endswith(".weight_g"):
            pairs.append((k[: -len(".weight_g")], k, k[:-1] + "v"))
        elif k.endswith(".parametrizations.weight.original0"):
            base = k[: -len(".parametrizations.weight.original0")]
            pairs.append((base, k, k[:-1] + "1"))
    for base, kg, kv in pairs:
        if kv not in sd:
            raise ValueError(f"weight norm: {kg} without {kv}")
        g = np.asarray(sd[kg], np.float64)
        v = np.asarray(sd[kv], np.float64)
        norm = np.sqrt((v.reshape(v.shape[0], -1) ** 2).sum(axis=1)).reshape((-1,) + (1,) * (v.ndim - 1))
        out[base + ".weight"] = (g.reshape(norm.shape) * v / norm).astype(np.float32)
        del out[kg], out[kv]
    return out


def load_state_dict(path: str) -> Dict[str, np.ndarray]:
    """Load a local checkpoint without executing code from it (safetensors / npz); weight-norm
    pairs are folded (fold_weight_norm)."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        return fold_weight_norm({k: np.asarray(v, np.float32) for k, v in load_file(path).items()})
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return fold_weight_norm({k: z[k].astype(np.float32) for k in z.files})
    raise ValueError(f"unsupported checkpoint format: {path}")


class GonovaTTS:
    """FastSpeech2-Conformer + HiFi-GAN V1 on MI355X (HIP kernels via libtts_hip.so)."""

    FRAMES_PER_TOKEN_CAP = 12  # first-pass frame budget per token; exact retry if exceeded

    def __init__(self, engine: HipEngine, acoustic_cfg: AcousticConfig, vocoder_cfg: VocoderConfig,
                 sample_rate: Optional[int] = None):
        self.engine = engine
        self.acoustic_cfg = acoustic_cfg
        self.vocoder_cfg = vocoder_cfg
        # output rate: the vocoder's 22,050 Hz, or e.g. 24,000 for clients that assume the
        # reference's hard-coded rate (synthesizer.py:119); converted on the device
        # (tts_resample_poly, scipy.signal.resample_poly semantics)
        self.native_sr = SAMPLE_RATE
        self.sr = int(sample_rate) if sample_rate else SAMPLE_RATE
        self.device = f"cuda:{engine.device_index}"
        self._lock = threading.Lock()

    @classmethod
    def from_pretrained(cls, device: str = "cuda", ckpt_dir: Optional[str] = None, seed: int = 0,
                        vocoder_dtype: str = "f16", acoustic_dtype: str = "bf16", fixed_duration: Optional[int] = None,
                        max_batch: int = 0, max_frames: int = 0, max_tokens: int = 0,
                        sample_rate: Optional[int] = None, speaker_embed_dim: Optional[int] = None,
                        encoder_precision: str = "exact"):
        """Mirror of `ChatterboxTTS.from_pretrained(device=...)` (synthesizer.py:185).

        ckpt_dir: optional directory with `acoustic.safetensors` and `vocoder.safetensors`
        (HF state_dict names); without it the deterministic seeded weights are used
        (no checkpoint is reachable offline).  sample_rate: output rate (default 22,050 Hz;
        24,000 reproduces the rate the reference's clients assume).  speaker_embed_dim: seeded
        multi-speaker weights with a speaker-embedding projection of that size (a checkpoint
        carrying `projection.weight` sets it by itself).  encoder_precision: "exact" (default: the
        encoder and variance predictors keep fp32 activations, so predicted integer durations match
        fp32, HF:181-183) or "fast" (all of the acoustic model in acoustic_dtype)."""
        acfg, vcfg = AcousticConfig(speaker_embed_dim=speaker_embed_dim), VocoderConfig()
        if ckpt_dir:
            aw = load_state_dict(os.path.join(ckpt_dir, "acoustic.safetensors"))
            vw = load_state_dict(os.path.join(ckpt_dir, "vocoder.safetensors"))
            if "projection.weight" in aw:  # multi-speaker checkpoint (HF speaker_embed_dim)
                acfg.speaker_embed_dim = aw["projection.weight"].shape[1] - aw["projection.weight"].shape[0]
        else:
            aw = make_acoustic_weights(seed, acfg, fixed_duration=fixed_duration)
            vw = make_vocoder_weights(seed, vcfg)
        eng = HipEngine(device, vocoder_dtype=vocoder_dtype, acoustic_dtype=acoustic_dtype,
                        max_batch=max_batch, max_frames=max_frames, max_tokens=max_tokens,
                        encoder_precision=encoder_precision)
        eng.load_weights(vocoder=vw, acoustic=aw, vocoder_cfg=vcfg)
        return cls(eng, acfg, vcfg, sample_rate=sample_rate)

    # -------------------------------------------------------------- synthesis
    def synthesize_tokens(self, tokens: np.ndarray, lens: np.ndarray, durations: Optional[np.ndarray] = None,
                          stream=None, speaker_embedding: Optional[np.ndarray] = None, host_lens: bool = True):
        """tokens int32 [B, N], lens [B] -> (wav cuda float32 [B, T*256], wav_lens np.int64 [B]).
        host_lens=False makes no host sync, so a caller can queue several batches back to back
        (dist.ShardedSynthesis), and returns (wav, wav_lens cuda int64 [B], pending): `pending` is
        None when nothing is left to check, else a PendingRange whose `word` the caller reads with
        the lengths at its own sync and whose `resolve(...)` reruns the batch when it is set.

        Range guard (include/tts_hip.h, ABI 4): with the exact encoder of a 16-bit model the
        acoustic forward's range word travels with the one host read this path makes anyway; when a
        split-precision operand was outside f16's range the batch is synthesized again with the
        encoder on the exact fp32 MFMA kernels (`range_fallbacks` counts these)."""
        import torch
        dev = self.engine.torch_device
        B, N = tokens.shape
        tok, tl, dd = _upload_i32((tokens, lens, durations), dev, stream)
        t_cap = max(64, int(self.FRAMES_PER_TOKEN_CAP * N))
        if durations is not None:
            t_cap = max(1, int(np.asarray(durations).sum(axis=1).max()))
        args = (tok, tl, dd, t_cap, stream, speaker_embedding, host_lens)
        # the engine's device is the current one for this thread (the streams torch hands out, the
        # ops below): an executor thread of a multi-GPU service starts on device 0
        with torch.cuda.device(self.engine.device_index):
            wav, wav_lens, tripped = self._synthesize_once(*args)
            if tripped is True:  # read on the host already (predicted durations)
                with self._range_fallback():
                    wav, wav_lens, _ = self._synthesize_once(*args)
                tripped = None
            if not host_lens:  # tripped: the unread range word (device) or None; the caller reads it
                pend = PendingRange(self, args[:-1] + (True,), tripped) if isinstance(tripped, torch.Tensor) else None
                return wav, wav_lens, pend
        return wav, wav_lens

    @property
    def range_fallbacks(self) -> int:
        """Forwards rerun on the fp32 encoder because the exact encoder's range guard tripped."""
        return self.engine.range_fallbacks

    @contextmanager
    def _range_fallback(self):
        import warnings
        self.engine.range_fallbacks += 1
        warnings.warn("acoustic encoder activations outside the f16 range of the split-precision GEMMs: "
                      "rerunning this batch with the encoder on fp32 MFMA (include/tts_hip.h, TTS_ENCODER_F32)",
                      RuntimeWarning, stacklevel=3)
        with self.engine.encoder_f32():
            yield

    def _synthesize_once(self, tok, tl, dd, t_cap, stream, spk, host_lens):
        """-> (wav, wav_lens, range guard tripped: bool, or None when nothing was read); with
        host_lens=False the third item is the forward's range word itself (cuda int32 [1], None
        without the guard), unread"""
        import torch
        mel, mel_lens, dur, rw = self.engine.acoustic(tok, tl, t_cap, durations=dd, stream=stream,
                                                      return_durations=True, speaker_embedding=spk, return_range=True)
        lens_known = None
        tripped = None
        if dd is None:
            # one host read for the frames the durations need, the frame counts and the range word
            need, lens_known, tripped = _need_and_lens(dur, mel_lens, rw)
            if tripped:
                return None, None, True
            if need > t_cap:  # exact second pass with the predicted durations and a fitting cap
                mel, mel_lens, dur, rw = self.engine.acoustic(tok, tl, need, durations=dur, stream=stream,
                                                              return_durations=True, speaker_embedding=spk,
                                                              return_range=True)
                need, lens_known, tripped = _need_and_lens(dur, mel_lens, rw)
                if tripped:
                    return None, None, True
            # the vocoder (and the waveform the caller copies to the host) at the frames the
            # durations give, not the 12-per-token budget: half the grid and the bytes at C3's 6
            T_act = max(1, int(lens_known.max())) if len(lens_known) else 1
            if T_act < mel.shape[1] and os.environ.get("TTS_VOC_TRIM", "1") != "0":  # (0: A/B runs)
                mel = mel[:, :T_act].contiguous()
        wav = self.engine.vocoder(mel, mel_lens, stream=stream)
        if self.sr != self.native_sr:
            g = gcd(self.sr, self.native_sr)
            wav, out_lens = self.engine.resample(wav, mel_lens * self.vocoder_cfg.hop, self.sr // g,
                                                 self.native_sr // g, stream=stream)
            out_lens = out_lens.to(torch.int64)
            if not host_lens:
                return wav, out_lens, rw if tripped is None else None
            if tripped is None:
                h, tripped = _read_with_range(out_lens, rw)
                return wav, h, tripped
            return wav, out_lens.cpu().numpy(), tripped
        if host_lens and lens_known is not None:  # already on the host: no second sync
            return wav, lens_known * self.vocoder_cfg.hop, tripped
        wav_lens = mel_lens.to(torch.int64) * self.vocoder_cfg.hop
        if not host_lens:
            return wav, wav_lens, rw if tripped is None else None
        h, tripped = _read_with_range(wav_lens, rw)
        return wav, h, tripped

    # -------------------------------------------------------------- streaming
    STREAM_CONTEXT = 16  # mel frames of context per side; HiFi-GAN V1's receptive field is < 13

    def stream_tokens(self, tokens: np.ndarray, lens: np.ndarray, chunk_frames: int = 32,
                      context: Optional[int] = None, durations: Optional[np.ndarray] = None, stream=None,
                      speaker_embedding: Optional[np.ndarray] = None):
        """Sub-sentence streaming: one acoustic pass, then the vocoder
        runs on windows [c0 - ctx, c0 + chunk + ctx) and keeps the middle `chunk` frames.
        With ctx >= the receptive field every kept sample is computed from the same inputs
        in the same order as the full-utterance pass, so the concatenated chunks equal it.

        Yields (c0, wav_chunk cuda float32 [B, chunk*256], valid samples per utterance np [B]).
        Chunks are at the vocoder's native 22,050 Hz whatever `sr` is (a resampled stream would
        need the resampler's own filter context across chunk edges)."""
        import torch
        with torch.cuda.device(self.engine.device_index):  # (see synthesize_tokens)
            yield from self._stream_tokens(tokens, lens, chunk_frames, context, durations, stream, speaker_embedding)

    def _stream_tokens(self, tokens, lens, chunk_frames, context, durations, stream, speaker_embedding):
        import torch
        ctx = self.STREAM_CONTEXT if context is None else context
        dev = self.engine.torch_device
        B, N = tokens.shape
        tok, tl, dd = _upload_i32((tokens, lens, durations), dev, stream)
        t_cap = max(64, int(self.FRAMES_PER_TOKEN_CAP * N)) if durations is None else \
            max(1, int(np.asarray(durations).sum(axis=1).max()))
        spk = speaker_embedding
        mel, mel_lens, dur, rw = self.engine.acoustic(tok, tl, t_cap, durations=dd, stream=stream, return_durations=True,
                                                      speaker_embedding=spk, return_range=True)
        first = None  # (window end, kept frames, chunk) enqueued ahead of the host read
        if durations is None:
            # The first chunk's window needs no host value when the longest utterance covers it
            # (frames >= chunk + ctx, the usual case): enqueue it before the one host read of the
            # frame counts, so the GPU runs it instead of idling through the round trip.  It is
            # used only if the loop below would make exactly the same call (else recomputed).
            # The read's copies are enqueued before the chunk and waited for by event, so the host
            # has the frame counts while the chunk still runs and hands the chunk over when it is
            # enqueued (a read after the chunk held the host until the chunk ended, then cost a
            # second round trip for the waveform: ~0.15 ms of C5, profiles/r06m/).
            w1 = min(t_cap, chunk_frames + ctx)
            tc = min(chunk_frames, t_cap)
            early = os.environ.get("TTS_STREAM_EARLY", "1") != "0"  # (0: the host read first, A/B runs)
            rd = _HostRead(dur, mel_lens, rw, stream)
            if early:
                win_lens = torch.clamp(mel_lens, min=0, max=w1).to(torch.int32)
                first = (w1, tc, self.engine.vocoder_chunk(mel[:, :w1].contiguous(), win_lens, 0, tc, stream=stream))
            need, lens_h, tripped = rd.result()  # one host read before the first chunk is handed over
            fell_back = False
            if tripped:  # range guard: the acoustic pass again on the fp32 encoder
                first, fell_back = None, True
                with self._range_fallback():
                    mel, mel_lens, dur = self.engine.acoustic(tok, tl, t_cap, durations=None, stream=stream,
                                                              return_durations=True, speaker_embedding=spk)
                need, lens_h, _ = _need_and_lens(dur, mel_lens)
            if need > t_cap:
                first = None
                # after a fallback the second pass stays on the fp32 encoder: its activations do not
                # depend on the durations, so the split encoder would overflow again
                with (self.engine.encoder_f32() if fell_back else nullcontext()):
                    mel, mel_lens, dur, rw = self.engine.acoustic(tok, tl, need, durations=dur, stream=stream,
                                                                  return_durations=True, speaker_embedding=spk,
                                                                  return_range=True)
                need, lens_h, tripped = _need_and_lens(dur, mel_lens, rw)
                if tripped and not fell_back:
                    with self._range_fallback():
                        mel, mel_lens, dur = self.engine.acoustic(tok, tl, need, durations=dur, stream=stream,
                                                                  return_durations=True, speaker_embedding=spk)
                    need, lens_h, _ = _need_and_lens(dur, mel_lens)
        else:
            # given durations fix the frame counts on the host: no device sync between the
            # acoustic pass and the first chunk's vocoder launches (same-box C5: neutral, the
            # host enqueues faster than the GPU drains either way)
            lens_h = _mel_lens_host(lens, durations, t_cap)
        T = int(lens_h.max()) if B else 0
        hop = self.vocoder_cfg.hop
        for c0 in range(0, T, chunk_frames):
            tc = min(chunk_frames, T - c0)
            w0 = max(0, c0 - ctx)
            w1 = min(T, c0 + tc + ctx)
            if c0 == 0 and first is not None and first[:2] == (w1, tc):
                wav = first[2]
            else:
                win = mel[:, w0:w1].contiguous()
                win_lens = torch.clamp(mel_lens - w0, min=0, max=w1 - w0).to(torch.int32)
                wav = self.engine.vocoder_chunk(win, win_lens, c0 - w0, tc, stream=stream)
            if c0 == 0 and durations is not None and rw is not None:
                # given durations made no host read so far: the range word is read here, where the
                # consumer would wait for this chunk anyway; out of range -> fp32 encoder, chunk again
                if int(rw.item()) != 0:
                    with self._range_fallback():
                        mel, mel_lens = self.engine.acoustic(tok, tl, t_cap, durations=dd, stream=stream,
                                                             speaker_embedding=spk)
                    win = mel[:, w0:w1].contiguous()
                    win_lens = torch.clamp(mel_lens - w0, min=0, max=w1 - w0).to(torch.int32)
                    wav = self.engine.vocoder_chunk(win, win_lens, c0 - w0, tc, stream=stream)
            first = None
            valid = np.clip(lens_h - c0, 0, tc) * hop
            yield c0, wav, valid

    def _voice_groups(self, n: int, speaker_embeddings):
        """Sentence index groups that share one engine pass: on a multi-speaker model the
        sentences with and without a voice run as two batches (HF skips the projection when no
        embedding is given, HF:1192)."""
        if not self.acoustic_cfg.speaker_embed_dim or speaker_embeddings is None or \
                all(e is None for e in speaker_embeddings):
            return [(list(range(n)), None)]
        with_v = [i for i, e in enumerate(speaker_embeddings) if e is not None]
        without = [i for i, e in enumerate(speaker_embeddings) if e is None]
        groups = [(with_v, np.stack([np.asarray(speaker_embeddings[i], np.float32).reshape(-1) for i in with_v]))]
        if without:
            groups.append((without, None))
        return groups

    def stream_batch(self, texts: List[str], chunk_frames: int = 32,
                     speaker_embeddings: Optional[List[Optional[np.ndarray]]] = None):
        """Sub-sentence streaming of many sentences in one batched pass (the service's opt-in
        `stream_frames` mode): yields, per vocoder chunk, a list of (sentence index, float32
        samples of that chunk, sentence finished).  A sentence's pieces concatenate to the
        stream_tokens output, which equals the full pass (stream_tokens).  With an output rate
        other than the vocoder's the pieces would need the resampler's filter context across
        chunk edges, so each sentence comes as one piece then."""
        if not texts:
            return
        if self.sr != self.native_sr:
            yield [(i, a, True) for i, a in enumerate(self.generate_batch(texts, speaker_embeddings))]
            return
        with self._lock:
            for idx, spk in self._voice_groups(len(texts), speaker_embeddings):
                tokens, lens = tokenize_batch([texts[i] for i in idx])
                done = [False] * len(idx)
                for c0, wav, valid in self.stream_tokens(tokens, lens, chunk_frames, speaker_embedding=spk):
                    host = _to_host(wav)
                    full = host.shape[1]
                    out = []
                    for r, i in enumerate(idx):
                        if done[r]:
                            continue
                        v = int(valid[r])
                        done[r] = v < full  # a short (or empty) piece is the sentence's last
                        out.append((i, host[r, :v].astype(np.float32, copy=False), done[r]))
                    yield out
                last = [(i, np.zeros(0, np.float32), True) for r, i in enumerate(idx) if not done[r]]
                if last:  # sentences whose length is a whole number of chunks
                    yield last

    def generate_batch(self, texts: List[str], speaker_embeddings: Optional[List[Optional[np.ndarray]]] = None,
                       **_ignored) -> List[np.ndarray]:
        """Synthesize many sentences in one batched pass -> list of float32 waveforms.
        speaker_embeddings: optional per-sentence voice vectors (None entries: no voice)."""
        if not texts:
            return []
        groups = self._voice_groups(len(texts), speaker_embeddings)
        out: List[Optional[np.ndarray]] = [None] * len(texts)
        with self._lock:
            for idx, spk in groups:
                tokens, lens = tokenize_batch([texts[i] for i in idx])
                wav, wav_lens = self.synthesize_tokens(tokens, lens, speaker_embedding=spk)
                host = _to_host(wav)
                for r, i in enumerate(idx):
                    out[i] = host[r, : int(wav_lens[r])].astype(np.float32, copy=False)
        return out

    def speaker_embedding(self, audio_prompt_path: Optional[str]) -> Optional[np.ndarray]:
        """The voice for `audio_prompt_path` (the reference's voice_id -> path,
        server.py:127-138): a stored speaker embedding (.npy / .npz / .safetensors, one vector of
        speaker_embed_dim values, loaded without executing anything from the file) when the
        model has a speaker projection; None otherwise.  Audio prompts (.wav) carry no
        embedding here -- the speaker encoder that would compute one is not part of this
        engine -- and are ignored, as before."""
        if not audio_prompt_path or not self.acoustic_cfg.speaker_embed_dim:
            return None
        path = str(audio_prompt_path)
        if path.endswith(".npy"):
            v = np.load(path, allow_pickle=False)
        elif path.endswith(".npz"):
            with np.load(path, allow_pickle=False) as z:
                v = z["embedding"] if "embedding" in z.files else z[z.files[0]]
        elif path.endswith(".safetensors"):
            from safetensors.numpy import load_file
            d = load_file(path)
            v = d["embedding"] if "embedding" in d else next(iter(d.values()))
        else:
            return None
        v = np.asarray(v, np.float32).reshape(-1)
        if v.size != self.acoustic_cfg.speaker_embed_dim:
            raise ValueError(f"speaker embedding {path}: {v.size} values, model expects "
                             f"{self.acoustic_cfg.speaker_embed_dim}")
        return v

    def generate(self, text: str, audio_prompt_path: Optional[str] = None, exaggeration: float = 0.5,
                 cfg_weight: float = 0.5, temperature: float = 0.8, **kwargs):
        """Same call shape as the reference's `model.generate` (synthesizer.py:344-350).

        Returns a float32 torch tensor of shape (1, N) on the engine device; the
        reference's `audio.squeeze().cpu().numpy()` applies unchanged.  audio_prompt_path
        selects a stored speaker embedding on a multi-speaker model (speaker_embedding())."""
        import torch
        del exaggeration, cfg_weight, temperature, kwargs
        spk = self.speaker_embedding(audio_prompt_path)
        with self._lock:
            tokens, lens = tokenize_batch([text])
            wav, wav_lens = self.synthesize_tokens(tokens, lens,
                                                   speaker_embedding=None if spk is None else spk[None])
        return wav[:, : int(wav_lens[0])].contiguous().to(torch.float32)


# Alias with the reference's class name so `from gonova_tts_amd.model import ChatterboxTTS`
# is a one-line swap at synthesizer.py:167.
ChatterboxTTS = GonovaTTS


class PendingRange:
    """The range word of a batch synthesized with host_lens=False, not yet read (dist.ShardedSynthesis
    reads it with the wave lengths at the one sync it makes).  resolve(lens_host, word_host) returns
    the batch's final (wav, wav_lens np.int64) -- the queued result when the word is 0, else the
    batch synthesized again with the encoder on fp32 MFMA (one RuntimeWarning, range_fallbacks + 1)."""

    def __init__(self, model: "GonovaTTS", args, word):
        self.model, self.args, self.word = model, args, word

    def resolve(self, wav, lens_host, word_host: int):
        if not word_host:
            return wav, lens_host
        import torch
        m = self.model
        with torch.cuda.device(m.engine.device_index), m._range_fallback():
            wav, wav_lens, _ = m._synthesize_once(*self.args)
        return wav, np.asarray(wav_lens, np.int64)


_UPLOAD_STREAMS: Dict[int, object] = {}


def _upload_i32(arrays, dev, stream=None):
    """Host integer arrays (None passes through) -> device int32 tensors, staged through pinned
    memory and copied on a per-device upload stream that `stream` (else the device's current
    stream, the one the engine calls enqueue on) then waits for.  Copied in order on the compute
    stream, a batch's inputs went up only when the previous batch's kernels had finished -- the
    moment dist.ShardedSynthesis (C4) starts that batch's waveform download, which held the small
    uploads (and the GPU) for ~0.7-1.7 ms per batch (profiles/r05zz_c4_gaps.txt).  Issued at once
    on their own stream they land while the previous batch still computes.  The arrays share one
    pinned block and one copy (64-byte aligned segments; the device tensors are views of it):
    the host time before the first kernel of a request is on C5's critical path."""
    import torch
    target = stream if stream is not None else torch.cuda.current_stream(dev)
    idx = torch.device(dev).index if torch.device(dev).index is not None else torch.cuda.current_device()
    up = _UPLOAD_STREAMS.get(idx)
    if up is None:
        up = _UPLOAD_STREAMS[idx] = torch.cuda.Stream(device=idx)
    host = [None if a is None else np.ascontiguousarray(a, np.int32) for a in arrays]
    offs, total = [], 0
    for a in host:
        offs.append(total)
        total += 0 if a is None else -(-a.size // 16) * 16
    pinned = torch.empty((max(total, 16),), dtype=torch.int32, pin_memory=True)
    hv = pinned.numpy()
    for a, o in zip(host, offs):
        if a is not None:
            hv[o:o + a.size] = a.reshape(-1)
    with torch.cuda.stream(up):
        blk = pinned.to(dev, non_blocking=True)
    target.wait_stream(up)
    blk.record_stream(target)  # (allocated on the upload stream, used on the target)
    return [None if a is None else blk[o:o + a.size].view(a.shape) for a, o in zip(host, offs)]


def _to_host(t):
    """Device tensor -> numpy copy through a page-locked block of torch's caching host allocator:
    a pinned D2H runs at DMA speed where `.cpu()` stages a pageable copy (C1's 436 KB waveform is
    on the first frame's critical path).  The copy runs on the tensor's device's current stream,
    the one the engine launched on; the returned array keeps the block alive until dropped."""
    import torch
    with torch.cuda.device(t.device):
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        torch.cuda.current_stream().synchronize()
    return h.numpy()


class _HostRead:
    """_need_and_lens without the blocking read: the durations, frame counts and range word are
    copied into page-locked host memory on the compute stream (where the forward enqueued them)
    and an event is recorded after them; result() waits for that event only, not for work the
    caller enqueued afterwards, and sums on the host.  When the three are views of one block (as
    GonovaEngine.acoustic returns them) the block is read with one copy."""

    def __init__(self, dur, mel_lens, rw=None, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(mel_lens.device)
        ts = (dur, mel_lens, rw)
        base = getattr(mel_lens, "_base", None)
        one = base is not None and base.is_contiguous() and base.dtype == torch.int32 and \
            all(t is None or (getattr(t, "_base", None) is base and t.is_contiguous()) for t in ts)
        with torch.cuda.stream(s):
            if one:
                h = torch.empty(base.shape, dtype=base.dtype, pin_memory=True)
                h.copy_(base, non_blocking=True)
                p0 = base.data_ptr()
                self.bufs = [None if t is None else
                             h[(t.data_ptr() - p0) // 4:(t.data_ptr() - p0) // 4 + t.numel()].view(t.shape) for t in ts]
            else:
                self.bufs = []
                for t in ts:
                    if t is None:
                        self.bufs.append(None)
                        continue
                    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                    h.copy_(t, non_blocking=True)
                    self.bufs.append(h)
            self.ev = torch.cuda.Event()
            self.ev.record(s)

    def result(self):
        """-> (need, frame counts np.int64 [B], range word set), as _need_and_lens"""
        self.ev.synchronize()
        d, ln, rw = self.bufs
        lens = ln.numpy().astype(np.int64)
        sums = d.numpy().astype(np.int64).sum(axis=1)
        need = int(np.maximum(sums, lens).max()) if len(lens) else 0
        return need, lens, bool(rw is not None and int(rw.numpy()[0]) != 0)


def _need_and_lens(dur, mel_lens, rw=None):
    """One device -> host read: (frames the used durations add up to at most, the frame counts
    np.int64 [B], the range word is set) -- the durations kernel's all-zero rule gives an
    utterance len frames, so the need is the larger of the two per utterance."""
    import torch
    rows = torch.stack([dur.sum(dim=1).to(torch.int64), mel_lens.to(torch.int64)]).reshape(-1)
    if rw is not None:
        rows = torch.cat([rows, rw.to(torch.int64)])
    h = rows.cpu().numpy()
    B = mel_lens.shape[0]
    need = int(np.maximum(h[:B], h[B:2 * B]).max()) if B else 0
    return need, h[B:2 * B].astype(np.int64), bool(rw is not None and h[2 * B] != 0)


def _read_with_range(lens, rw=None):
    """lens (cuda int64 [B]) and the range word in one device -> host read."""
    import torch
    if rw is None:
        return lens.cpu().numpy(), False
    h = torch.cat([lens, rw.to(torch.int64)]).cpu().numpy()
    return h[:-1], bool(h[-1] != 0)


def _mel_lens_host(lens: np.ndarray, durations: np.ndarray, t_cap: int) -> np.ndarray:
    """Frame counts for given durations, as the engine's durations kernel computes them
    (acoustic_kernels.hip: negative durations count 0; an utterance whose durations are all 0
    gets one frame per token, HF:108-109; clamped to the frame cap)."""
    d = np.asarray(durations, np.int64)
    out = np.zeros(len(lens), np.int64)
    for b, L in enumerate(np.asarray(lens, np.int64)):
        L = int(min(L, d.shape[1]))
        s = int(np.maximum(d[b, :L], 0).sum())
        if s == 0 and L > 0:
            s = L
        out[b] = min(s, t_cap)
    return out
