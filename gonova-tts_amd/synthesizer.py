"""`StreamingSynthesizer` — the reference's synthesis adapter, re-hosted on the HIP engine.

Mirrors `services/tts/core/synthesizer.py:102-429` name for name (constructor
arguments, `load`, `synthesize_streaming`, `_generate_sentence`, `_synthesize_sync`,
`get_stats`, `cleanup`) so `server.py` needs no change beyond the import
(SURVEY.md §8b).  Behaviour kept from the reference:

* sentence segmentation (`split_into_sentences`, synthesizer.py:48-99);
* one float32 ndarray yielded per sentence, generated on the default
  ThreadPoolExecutor (synthesizer.py:296-325);
* stats keys and first-chunk latency accounting (synthesizer.py:140-145, 252-289, 411-420);
* exceptions are logged and re-raised (synthesizer.py:291-294, 323-325);
* `load()` warms up with the same three texts at exaggeration 0.5 (synthesizer.py:199-207).

Differences (documented, by design): the model is `GonovaTTS` (FS2 + HiFi-GAN on
MI355X) instead of the un-vendored `ChatterboxTTS`; output rate 22,050 Hz; the
"cuda" device string maps to a HIP device; the flag-setting / torch.compile block
(synthesizer.py:175-193) is not needed (the kernels are hand-written, not traced).
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import AsyncGenerator, List, Optional

import numpy as np

from .config import SAMPLE_RATE
from .text import split_into_sentences  # noqa: F401  (re-exported: reference module-level API)

logger = logging.getLogger(__name__)


class StreamingSynthesizer:
    def __init__(self, model_path: Optional[str] = None, device: str = "cuda", device_index: int = 0,
                 chunk_size: int = 15, sample_rate: int = SAMPLE_RATE, vocoder_dtype: str = "f16",
                 acoustic_dtype: str = "bf16"):
        self.model_path = model_path
        self.device = f"{device}:{device_index}" if device in ("cuda", "hip") else device
        self.device_index = device_index
        self.chunk_size = chunk_size
        self.sample_rate = sample_rate
        self.vocoder_dtype = vocoder_dtype
        self.acoustic_dtype = acoustic_dtype
        self.model = None
        self.is_loaded = False
        self._warmup_done = False
        self.stats = {'syntheses': 0, 'total_latency': 0.0, 'first_chunk_latency': 0.0, 'errors': 0}

    async def load(self):
        if self.is_loaded:
            logger.warning("Model already loaded")
            return
        logger.info(f"Loading MI355X TTS engine on {self.device}")
        start_time = time.time()
        try:
            from .model import GonovaTTS
            # sample_rate is the output rate, as in the reference (synthesizer.py:119); 24000 gets
            # the reference's rate through the on-device resampler
            self.model = GonovaTTS.from_pretrained(device=self.device, ckpt_dir=self.model_path,
                                                   vocoder_dtype=self.vocoder_dtype,
                                                   acoustic_dtype=self.acoustic_dtype,
                                                   sample_rate=self.sample_rate)
            self.sample_rate = self.model.sr
            loop = asyncio.get_event_loop()
            warmup_texts = [
                "Hello.",
                "Hello, this is a warmup test.",
                "The quick brown fox jumps over the lazy dog, and this is a longer sentence to warm up the model properly.",
            ]
            for i, text in enumerate(warmup_texts):
                logger.info(f"Warmup {i+1}/{len(warmup_texts)}: '{text[:30]}...'")
                _ = await loop.run_in_executor(None, self._synthesize_sync, text, None, 0.5)
            self._warmup_done = True
            logger.info(f"Model loaded and warmed up in {time.time() - start_time:.2f}s")
            self.is_loaded = True
        except Exception as e:
            logger.error(f"Failed to load model: {e}")
            raise

    async def synthesize_streaming(self, text: str, voice_embedding=None, chunk_size: Optional[int] = None,
                                   exaggeration: float = 0.25) -> AsyncGenerator[np.ndarray, None]:
        _ = chunk_size
        if not self.is_loaded:
            raise RuntimeError("Model not loaded. Call load() first")
        if not text.strip():
            return
        start_time = time.time()
        first_chunk_time = None
        try:
            sentences = split_into_sentences(text)
            logger.info(f"Split text into {len(sentences)} sentences")
            for sentence in sentences:
                if not sentence.strip():
                    continue
                async for audio_chunk in self._generate_sentence(sentence, voice_embedding, exaggeration):
                    if first_chunk_time is None:
                        first_chunk_time = time.time() - start_time
                        self.stats['first_chunk_latency'] += first_chunk_time
                    yield audio_chunk
            total_time = time.time() - start_time
            self.stats['syntheses'] += 1
            self.stats['total_latency'] += total_time
            logger.info(f"Synthesized {len(sentences)} sentences in {total_time*1000:.0f}ms")
        except Exception as e:
            self.stats['errors'] += 1
            logger.error(f"Synthesis error: {e}")
            raise

    async def _generate_sentence(self, sentence: str, voice_embedding, exaggeration: float
                                 ) -> AsyncGenerator[np.ndarray, None]:
        loop = asyncio.get_event_loop()
        try:
            audio = await loop.run_in_executor(None, self._synthesize_sync, sentence, voice_embedding, exaggeration)
            yield audio
        except Exception as e:
            logger.error(f"Sentence generation failed: {e}")
            raise

    def _synthesize_sync(self, text: str, voice_embedding: Optional[str] = None, exaggeration: float = 0.25
                         ) -> np.ndarray:
        import torch
        audio = self.model.generate(
            text,
            audio_prompt_path=voice_embedding if isinstance(voice_embedding, str) else None,
            exaggeration=exaggeration,
            cfg_weight=0.5,
            temperature=0.8,
        )
        if isinstance(audio, torch.Tensor):
            audio = audio.squeeze().cpu().numpy()
        if audio.dtype != np.float32:
            audio = audio.astype(np.float32)
        return audio

    def synthesize_batch_sync(self, texts: List[str]) -> List[np.ndarray]:
        """Batched synthesis of many sentences in one engine pass (used by the dynamic batcher)."""
        if not self.is_loaded:
            raise RuntimeError("Model not loaded. Call load() first")
        return self.model.generate_batch(texts)

    def get_stats(self) -> dict:
        stats = self.stats.copy()
        if stats['syntheses'] > 0:
            stats['avg_latency'] = stats['total_latency'] / stats['syntheses']
            stats['avg_first_chunk'] = stats['first_chunk_latency'] / stats['syntheses']
        else:
            stats['avg_latency'] = 0.0
            stats['avg_first_chunk'] = 0.0
        return stats

    async def cleanup(self):
        if self.model:
            try:
                self.model.engine.close()
            except Exception:
                pass
            self.model = None
            self.is_loaded = False
            self._warmup_done = False
            logger.info("Model unloaded")
