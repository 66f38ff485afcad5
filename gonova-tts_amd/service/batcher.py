"""Cross-request continuous batcher: the replacement for the reference's serial `_tts_worker`
(`services/tts/server.py:110-186`, strictly one request in flight, one `generate` call per
sentence).

Admission: requests are taken from the input queue as they arrive (while every engine is busy,
whatever arrives within `max_wait` of the first joins it; with an engine idle, within `idle_wait`,
default 0: at once), split into sentences with the reference's segmentation
(`synthesizer.py:48-99`), and their sentences join one shared work list -- up to
`max_requests` requests in flight, new ones admitted while engines are busy.

Engines: each engine (one per local GPU, `synth_batches`; a single engine is the reference's
one-GPU-per-process shape, `server.py:397-400`) runs a loop of its own: whenever it is free it
takes the next engine batch from the work list -- the pending sentence earliest in its own request
(a new request's first sentence goes ahead of an older request's later ones; streamed requests
first: they are the latency-sensitive ones) together with the pending sentences of the same framing
whose lengths are closest to it, up to `max_sentences` (one acoustic + one vocoder pass per batch,
ragged lengths handled on device) -- so no engine idles while work is queued, a fast engine never
waits for a slow one, and a request that arrives mid-stream starts before the earlier ones end.  Audio goes back per request in sentence order, one binary frame per
sentence, then the final marker -- the reference's framing (`server.py:150-164`) -- as soon as all
earlier sentences of that request are done.  Requests that ask for sub-sentence frames
(`stream_frames` > 0) run through the engine's `synth_streams` entry (`GonovaTTS.stream_batch`) in
batches of their own, on whichever engine is free: each vocoder chunk's pieces go out as soon as
they reach the host, still in sentence order per request.

Failure: the reference logs and swallows synthesis errors, so the client never gets a
final marker (`server.py:173-179`).  That stays the default; `notify_errors=True` sends
`{"type": "synthesis_error", "message": ...}` plus the final marker instead.

Stats: `get_stats()` has the reference synthesizer's keys (`synthesizer.py:140-145, 411-420`):
`syntheses` (requests completed), `total_latency` and `first_chunk_latency` (seconds, summed; per
request from admission -- the reference's `synthesize_streaming` start -- to its final marker and
to its first audio frame, `synthesizer.py:274-277`), `errors` (failed requests), `avg_latency`,
`avg_first_chunk`; plus this batcher's own counters.

Delivery: each request's frames go out from a task of their own under the request's own lock
(sentence order within the request), so a client whose output queue is full (enqueue_audio_chunk
waits up to 0.1 s per frame) delays only itself: neither other connections' frames nor the engine's
next batch wait behind it.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import time
from typing import Callable, List, Optional

import numpy as np

from ..text import split_into_sentences

logger = logging.getLogger(__name__)


class _Request:
    """One admitted request: its sentences' audio pieces not yet sent, which sentences are done,
    and how far its frames have gone out."""

    def __init__(self, req, sentences):
        self.req = req
        self.sentences = sentences
        self.pending: List[List[np.ndarray]] = [[] for _ in sentences]
        self.done = [False] * len(sentences)
        self.failed = False
        self.cursor = 0     # the sentence whose pieces go out next
        self.sent = 0       # frames sent: the chunk_id of the next frame / the final marker
        self.finished = False
        self.t_admit = time.perf_counter()
        self.first_chunk: Optional[float] = None
        self.lock = asyncio.Lock()  # this request's delivery order (no cross-request lock)


class _Item:
    __slots__ = ("state", "j", "text", "framing", "seq")

    def __init__(self, state, j, text, framing, seq):
        self.state, self.j, self.text, self.framing, self.seq = state, j, text, framing, seq


class DynamicBatcher:
    def __init__(self, queues, synth_batch: Callable[[List[str]], List[np.ndarray]], max_sentences: int = 32,
                 max_requests: int = 64, max_wait: float = 0.004, notify_errors: bool = False,
                 send_error: Optional[Callable] = None, synth_stream: Optional[Callable] = None,
                 sample_rate: int = 22050, synth_batches: Optional[List[Callable]] = None,
                 synth_streams: Optional[List[Optional[Callable]]] = None, idle_wait: float = 0.0):
        self.queues = queues
        self.sample_rate = float(sample_rate)  # the rate the engine's audio is in (model.sr)
        self.synth_batch = synth_batch
        # one synth_batch (and stream_batch) per local engine (GPU)
        self.synth_batches = list(synth_batches) if synth_batches else [synth_batch]
        self.synth_stream = synth_stream  # model.stream_batch: sub-sentence frames (opt-in per request)
        self.synth_streams = list(synth_streams) if synth_streams else [synth_stream] * len(self.synth_batches)
        self.max_sentences = max_sentences
        self.max_requests = max_requests
        self.max_wait = max_wait
        self.idle_wait = idle_wait  # the window while an engine is idle (0: start at once)
        self.notify_errors = notify_errors
        self.send_error = send_error
        self.running = False
        self._work: List[_Item] = []
        self._seq = itertools.count()
        self._inflight = 0
        self._idle = 0  # engine workers waiting for work
        self._cond: Optional[asyncio.Condition] = None
        self._flushes: set = set()  # delivery tasks in flight
        self._run_task = None  # run()'s task, and whether it waits for requests (stop())
        self._admitting = False
        self.stats = {"syntheses": 0, "total_latency": 0.0, "first_chunk_latency": 0.0, "errors": 0,
                      "rounds": 0, "engine_batches": 0, "batch_errors": 0, "sentences": 0, "requests": 0,
                      "audio_seconds": 0.0, "busy_seconds": 0.0, "max_batch_seen": 0,
                      "engine_sentences": [0] * len(self.synth_batches),
                      "engine_busy_seconds": [0.0] * len(self.synth_batches)}

    def get_stats(self) -> dict:
        """The reference synthesizer's stats shape (synthesizer.py:411-420) plus this batcher's."""
        st = dict(self.stats)
        n = st["syntheses"]
        st["avg_latency"] = st["total_latency"] / n if n else 0.0
        st["avg_first_chunk"] = st["first_chunk_latency"] / n if n else 0.0
        return st

    # ------------------------------------------------------------------ admission
    async def run(self):
        """Admission loop plus one worker per engine, until stop() / cancellation."""
        self.running = True
        self._run_task = asyncio.current_task()
        self._cond = asyncio.Condition()
        loop = asyncio.get_running_loop()
        workers = [asyncio.create_task(self._engine_loop(e, loop)) for e in range(len(self.synth_batches))]
        try:
            while self.running:
                # back-pressure: at most max_requests admitted and unfinished
                async with self._cond:
                    await self._cond.wait_for(lambda: self._inflight < self.max_requests or not self.running)
                    room = self.max_requests - self._inflight
                if not self.running:
                    break
                self._admitting = True
                try:
                    # the gathering window only while every engine is busy (what arrives then is
                    # batched by the continuous admission anyway): an idle engine starts at once,
                    # so a lone request does not pay max_wait (C1's first-frame latency)
                    reqs = await self.queues.take_batch(room, lambda: self.idle_wait if self._idle else self.max_wait)
                except asyncio.CancelledError:
                    break
                finally:
                    self._admitting = False
                if reqs:
                    await self._admit(reqs)
        finally:
            self.running = False
            for w in workers:
                w.cancel()
            await asyncio.gather(*workers, return_exceptions=True)
            for t in list(self._flushes):
                t.cancel()
            await asyncio.gather(*self._flushes, return_exceptions=True)

    async def _admit(self, reqs):
        self.stats["rounds"] += 1
        self.stats["requests"] += len(reqs)
        states = []
        for r in reqs:
            try:
                ss = split_into_sentences(r.text)
            except Exception as e:  # never let the admission die (reference server.py:184-186)
                logger.error("sentence split failed: %s", e)
                ss = []
            states.append(_Request(r, ss))
        async with self._cond:
            self._inflight += len(states)
            for st in states:
                f = self._framing(st.req)
                for j, text in enumerate(st.sentences):
                    self._work.append(_Item(st, j, text, f, next(self._seq)))
            self._cond.notify_all()
        for st in states:
            if not st.sentences:  # empty text: only the marker
                self._deliver(st)

    def _framing(self, req) -> int:
        f = getattr(req, "stream_frames", 0) or 0
        return f if any(s is not None for s in self.synth_streams) else 0

    def _take(self) -> List[_Item]:
        """The next engine batch (caller holds the condition).  Its head is the pending sentence
        that is earliest in its own request (a request's first sentence is its time to first audio;
        later sentences only have to keep pace with playback), streamed requests first, oldest
        first among equals; the batch is the head plus the pending sentences of its framing closest
        to it in length, at most max_sentences, in length order."""
        head = min(self._work, key=lambda it: (it.framing == 0, it.j, it.seq))
        group = sorted((it for it in self._work if it.framing == head.framing), key=lambda it: (len(it.text), it.seq))
        n = min(self.max_sentences, len(group))
        h = group.index(head)
        best = max(0, h - n + 1)
        for s0 in range(max(0, h - n + 1), min(h, len(group) - n) + 1):
            if len(group[s0 + n - 1].text) - len(group[s0].text) < \
                    len(group[best + n - 1].text) - len(group[best].text):
                best = s0
        batch = group[best:best + n]
        taken = set(id(it) for it in batch)
        self._work = [it for it in self._work if id(it) not in taken]
        return batch

    # ------------------------------------------------------------------ engines
    async def _engine_loop(self, eng: int, loop):
        while True:
            async with self._cond:
                self._idle += 1
                try:
                    await self._cond.wait_for(lambda: bool(self._work))
                finally:
                    self._idle -= 1
                batch = self._take()
            t0 = time.perf_counter()
            try:
                await self._one_batch(batch, eng, loop)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # never let a worker die (reference server.py:184-186)
                logger.error("engine %d batch failed: %s", eng, e, exc_info=True)
            finally:
                dt = time.perf_counter() - t0
                self.stats["busy_seconds"] += dt
                self.stats["engine_busy_seconds"][eng] += dt

    async def _one_batch(self, batch: List[_Item], eng: int, loop):
        texts = [it.text for it in batch]
        voices = [getattr(it.state.req, "voice", None) for it in batch]
        # per-sentence voice (registered embedding) only when one is set
        kw = {"speaker_embeddings": voices} if any(v is not None for v in voices) else {}
        frames = batch[0].framing
        try:
            if frames == 0:
                synth = self.synth_batches[eng]
                audios = await loop.run_in_executor(None, lambda: synth(texts, **kw))
                audios = list(audios) if audios is not None else []
                if len(audios) != len(batch) or any(a is None for a in audios):
                    # a short or partial result would leave sentences never marked done (and
                    # their request's slot never freed): the whole batch fails instead
                    raise RuntimeError(f"engine returned {len(audios)} results for {len(batch)} sentences")
                for it, a in zip(batch, audios):
                    it.state.pending[it.j].append(a)
                    it.state.done[it.j] = True
                    self.stats["audio_seconds"] += len(a) / self.sample_rate
            else:
                async def deliver(pieces):
                    touched = {}
                    for t, a, fin in pieces:
                        it = batch[t]
                        if len(a):
                            it.state.pending[it.j].append(a)
                            self.stats["audio_seconds"] += len(a) / self.sample_rate
                        it.state.done[it.j] = it.state.done[it.j] or fin
                        touched[id(it.state)] = it.state
                    for st in touched.values():
                        self._deliver(st)
                await self._stream(loop, texts, frames, kw, deliver, eng)
        except asyncio.CancelledError:
            raise
        except Exception as e:
            self.stats["batch_errors"] += 1
            logger.error("synthesis_failed: %s", e)
            for it in batch:
                st = it.state
                if not st.failed:
                    st.failed = True
                    self.stats["errors"] += 1  # per request, as the reference counts (synthesizer.py:291-294)
                    if self.notify_errors and self.send_error is not None:
                        await self.send_error(st.req.connection_id, str(e))
            for st in {id(it.state): it.state for it in batch}.values():
                self._deliver(st)
            return
        self.stats["engine_batches"] += 1
        self.stats["sentences"] += len(batch)
        self.stats["engine_sentences"][eng] += len(batch)
        self.stats["max_batch_seen"] = max(self.stats["max_batch_seen"], len(batch))
        for st in {id(it.state): it.state for it in batch}.values():
            self._deliver(st)

    def _deliver(self, st: _Request):
        """Start sending what request `st` can send, in a task of its own (see _flush)."""
        t = asyncio.get_running_loop().create_task(self._flush(st))
        self._flushes.add(t)
        t.add_done_callback(self._flushes.discard)

    async def _flush(self, st: _Request):
        """Send what request `st` can send in sentence order; its final marker once every sentence
        is done (or, after a failure, per notify_errors); a finished request frees its slot.  The
        lock is the request's own: other requests' frames never wait behind this client."""
        async with st.lock:
            if st.finished:
                return
            r = st.req
            try:
                while st.cursor < len(st.pending):
                    j = st.cursor
                    while st.pending[j]:
                        a = st.pending[j].pop(0)
                        await self.queues.enqueue_audio_chunk(r.connection_id, np.asarray(a, np.float32).tobytes(), st.sent)
                        if st.first_chunk is None:
                            st.first_chunk = time.perf_counter() - st.t_admit
                        st.sent += 1
                    if not st.done[j]:
                        break
                    st.cursor += 1
            except asyncio.CancelledError:
                raise
            except Exception as e:  # a frame that cannot be sent fails its request, not the engine
                logger.error("delivery failed for %s: %s", r.connection_id, e)
                if not st.failed:
                    st.failed = True
                    self.stats["errors"] += 1
            if st.cursor == len(st.pending) or st.failed:
                if st.failed:
                    # drop its queued sentences: nothing more goes to this client
                    async with self._cond:
                        self._work = [it for it in self._work if it.state is not st]
                else:
                    self.stats["syntheses"] += 1
                    self.stats["total_latency"] += time.perf_counter() - st.t_admit
                    self.stats["first_chunk_latency"] += st.first_chunk or 0.0
                st.finished = True
                try:
                    if not (st.failed and not self.notify_errors):  # reference behaviour: no marker after a failure
                        await self.queues.enqueue_audio_chunk(r.connection_id, b"", st.sent, is_final=True)
                finally:
                    await self.queues.mark_request_done(1)
                    async with self._cond:
                        self._inflight -= 1
                        self._cond.notify_all()

    async def _stream(self, loop, texts, frames, kw, deliver, eng: int = 0):
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

        synth_stream = self.synth_streams[eng] if eng < len(self.synth_streams) else self.synth_stream

        def produce():
            gen = synth_stream(texts, frames, **kw)
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
        if self._admitting and self._run_task is not None:
            # the admission loop waits on the input queue without a timeout: end that wait
            self._run_task.cancel()
        if self._cond is not None:
            async def wake():
                async with self._cond:
                    self._cond.notify_all()
            try:
                asyncio.get_running_loop().create_task(wake())
            except RuntimeError:
                pass
