"""Cross-request dynamic batcher: the replacement for the reference's serial `_tts_worker`
(`services/tts/server.py:110-186`, strictly one request in flight, one `generate` call per
sentence).

Each round takes every queued request (up to `max_requests`, waiting at most `max_wait`
after the first), splits them into sentences with the reference's segmentation
(`synthesizer.py:48-99`), sorts all sentences by length and synthesizes them in engine
batches of up to `max_sentences` (one acoustic + one vocoder pass per batch, ragged
lengths handled on device).  Audio goes back per request in sentence order, one binary
frame per sentence, then the final marker -- the reference's framing
(`server.py:150-164`) -- as soon as all earlier sentences of that request are done.
Requests that ask for sub-sentence frames (`stream_frames` > 0) run through
`synth_stream` (`GonovaTTS.stream_batch`) in batches of their own: each vocoder chunk's
pieces go out as soon as they reach the host, still in sentence order per request.

Several GPUs (opt-in, `synth_batches` with one callable per local engine): the per-sentence
engine batches of a round are dealt across the engines with `dist.plan_buckets` (longest
sentence first to the least-loaded engine, each engine's share cut into length-sorted batches of
`max_sentences`), and the engines run at the same time, one executor thread each; frames still
leave in per-request sentence order.  The reference can only run one server process per GPU
behind a load balancer (`server.py:397-400,486-488`).  Streamed requests stay on the first engine.

Failure: the reference logs and swallows synthesis errors, so the client never gets a
final marker (`server.py:173-179`).  That stays the default; `notify_errors=True` sends
`{"type": "synthesis_error", "message": ...}` plus the final marker instead.
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Callable, List, Optional

import numpy as np

from ..text import split_into_sentences

logger = logging.getLogger(__name__)


class DynamicBatcher:
    def __init__(self, queues, synth_batch: Callable[[List[str]], List[np.ndarray]], max_sentences: int = 32,
                 max_requests: int = 64, max_wait: float = 0.004, notify_errors: bool = False,
                 send_error: Optional[Callable] = None, synth_stream: Optional[Callable] = None,
                 sample_rate: int = 22050, synth_batches: Optional[List[Callable]] = None):
        self.queues = queues
        self.sample_rate = float(sample_rate)  # the rate the engine's audio is in (model.sr)
        self.synth_batch = synth_batch
        # one synth_batch per local engine (GPU); a single engine is the reference-shaped default
        self.synth_batches = list(synth_batches) if synth_batches else [synth_batch]
        self.max_sentences = max_sentences
        self.max_requests = max_requests
        self.max_wait = max_wait
        self.notify_errors = notify_errors
        self.send_error = send_error
        self.synth_stream = synth_stream  # model.stream_batch: sub-sentence frames (opt-in per request)
        self.running = False
        self.stats = {"rounds": 0, "engine_batches": 0, "sentences": 0, "requests": 0, "errors": 0,
                      "audio_seconds": 0.0, "busy_seconds": 0.0, "max_batch_seen": 0,
                      "engine_sentences": [0] * len(self.synth_batches)}

    async def run(self):
        self.running = True
        loop = asyncio.get_running_loop()
        while self.running:
            try:
                reqs = await self.queues.take_batch(self.max_requests, self.max_wait)
            except asyncio.CancelledError:
                break
            if not reqs:
                continue
            t0 = time.perf_counter()
            try:
                await self._round(reqs, loop)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # never let the worker die (reference server.py:184-186)
                logger.error("batcher round failed: %s", e, exc_info=True)
            finally:
                self.stats["busy_seconds"] += time.perf_counter() - t0
                await self.queues.mark_request_done(len(reqs))

    async def _round(self, reqs, loop):
        self.stats["rounds"] += 1
        self.stats["requests"] += len(reqs)
        sentences = [split_into_sentences(r.text) for r in reqs]
        work = [(i, j, s) for i, ss in enumerate(sentences) for j, s in enumerate(ss)]
        # per sentence: audio pieces not yet sent, and whether its last piece has arrived
        pending: List[List[List[np.ndarray]]] = [[[] for _ in ss] for ss in sentences]
        done = [[False] * len(ss) for ss in sentences]
        failed = [False] * len(reqs)
        cursor = [0] * len(reqs)  # the sentence whose pieces go out next
        sent = [0] * len(reqs)    # frames sent: the chunk_id of the next frame / the final marker
        finished = [False] * len(reqs)

        flush_lock = asyncio.Lock()  # engines finishing together must not send a piece twice

        async def flush():
            async with flush_lock:
                await flush_locked()

        async def flush_locked():
            for i, r in enumerate(reqs):
                if finished[i]:
                    continue
                while cursor[i] < len(pending[i]):
                    j = cursor[i]
                    for a in pending[i][j]:
                        await self.queues.enqueue_audio_chunk(r.connection_id, a.astype(np.float32).tobytes(), sent[i])
                        sent[i] += 1
                    pending[i][j].clear()
                    if not done[i][j]:
                        break
                    cursor[i] += 1
                if cursor[i] == len(pending[i]) or failed[i]:
                    if failed[i] and not self.notify_errors:
                        finished[i] = True  # reference behaviour: no marker after a failure
                        continue
                    await self.queues.enqueue_audio_chunk(r.connection_id, b"", sent[i], is_final=True)
                    finished[i] = True

        # engine batches: sentences grouped by framing (per sentence, or sub-sentence frames of
        # one size; the streamed groups first, they are the latency-sensitive ones), each group
        # sorted by length and cut into batches of max_sentences
        def framing(i):
            f = getattr(reqs[i], "stream_frames", 0) or 0
            return f if self.synth_stream is not None else 0
        groups = {}
        for k, (i, _, _) in enumerate(work):
            groups.setdefault(framing(i), []).append(k)
        batches = []
        for f in sorted(groups, key=lambda f: (f == 0, f)):
            ks = sorted(groups[f], key=lambda k: len(work[k][2]))
            if f == 0 and len(self.synth_batches) > 1:
                continue  # dealt across the engines below
            batches += [(f, ks[b0:b0 + self.max_sentences], 0) for b0 in range(0, len(ks), self.max_sentences)]

        async def one_batch(frames, chunk, eng):
            texts = [work[k][2] for k in chunk]
            voices = [getattr(reqs[work[k][0]], "voice", None) for k in chunk]
            # per-sentence voice (registered embedding) only when one is set
            kw = {"speaker_embeddings": voices} if any(v is not None for v in voices) else {}
            synth = self.synth_batches[eng]
            try:
                if frames == 0:
                    audios = await loop.run_in_executor(None, lambda: synth(texts, **kw))
                    for k, a in zip(chunk, audios):
                        i, j, _ = work[k]
                        pending[i][j].append(a)
                        done[i][j] = True
                        self.stats["audio_seconds"] += len(a) / self.sample_rate
                    self.stats["engine_sentences"][eng] += len(chunk)
                else:
                    async def deliver(pieces):
                        for t, a, fin in pieces:
                            i, j, _ = work[chunk[t]]
                            if len(a):
                                pending[i][j].append(a)
                                self.stats["audio_seconds"] += len(a) / self.sample_rate
                            done[i][j] = done[i][j] or fin
                        await flush()
                    await self._stream(loop, texts, frames, kw, deliver)
            except Exception as e:
                self.stats["errors"] += 1
                logger.error("synthesis_failed: %s", e)
                for k in chunk:
                    i = work[k][0]
                    if not failed[i]:
                        failed[i] = True
                        if self.notify_errors and self.send_error is not None:
                            await self.send_error(reqs[i].connection_id, str(e))
                await flush()
                return
            self.stats["engine_batches"] += 1
            self.stats["sentences"] += len(chunk)
            self.stats["max_batch_seen"] = max(self.stats["max_batch_seen"], len(chunk))
            await flush()

        for frames, chunk, eng in batches:
            await one_batch(frames, chunk, eng)
        if len(self.synth_batches) > 1 and 0 in groups:
            # per-sentence batches across the engines: longest-first to the least-loaded engine
            # (load = characters), each engine's share in length-sorted batches, engines concurrent
            from ..dist import plan_buckets
            ks = groups[0]
            plan = plan_buckets([len(work[k][2]) for k in ks], len(self.synth_batches), self.max_sentences)

            async def engine_run(eng, buckets):
                for bk in buckets:
                    await one_batch(0, [ks[u] for u in bk], eng)

            await asyncio.gather(*(engine_run(e, bks) for e, bks in enumerate(plan) if bks))
        await flush()

    async def _stream(self, loop, texts, frames, kw, deliver):
        """Run `synth_stream` (a generator of per-chunk pieces) on an executor thread and hand
        each chunk to `deliver` on the event loop as soon as it is on the host, so the first
        frames go out while the vocoder still works on the rest of the batch.

        If `deliver` raises or this coroutine is cancelled, the producer is told to stop: it
        checks the event between chunks and closes the generator (which releases the model's
        lock), so no thread keeps synthesizing for nobody and the next engine batch is not
        held behind it.  The producer's future is always awaited, so its exception is read."""
        import threading
        q: asyncio.Queue = asyncio.Queue()
        end = object()
        stop = threading.Event()

        def produce():
            gen = self.synth_stream(texts, frames, **kw)
            try:
                for item in gen:
                    if stop.is_set():
                        break
                    loop.call_soon_threadsafe(q.put_nowait, item)
            except BaseException as e:  # noqa: BLE001 -- re-raised on the loop
                loop.call_soon_threadsafe(q.put_nowait, e)
                return
            finally:
                gen.close()
            loop.call_soon_threadsafe(q.put_nowait, end)

        fut = loop.run_in_executor(None, produce)
        try:
            while True:
                item = await q.get()
                if item is end:
                    break
                if isinstance(item, BaseException):
                    raise item
                await deliver(item)
        finally:
            stop.set()
            # the producer ends within one chunk; its own exception (if any) was raised above
            await asyncio.shield(asyncio.gather(fut, return_exceptions=True))

    def stop(self):
        self.running = False
