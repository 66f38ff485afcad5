"""Request / audio queues with the reference's admission semantics
(`services/tts/core/queue_manager.py`):

* one bounded input queue (500); a put waits up to 2 s, then the request is dropped
  and counted (`queue_manager.py:131-171`);
* a bounded output queue per connection (2000); a chunk put is tried without waiting,
  then for 0.1 s, then the chunk is dropped (`queue_manager.py:200-248`);
* the same metric keys (`queue_manager.py:64-70, 282-291`), the final marker counting
  as a sent chunk (`queue_manager.py:232`).

Added for the batched engine: `take_batch(max_items, max_wait)` drains up to
`max_items` requests, waiting at most `max_wait` seconds after the first one.
"""
from __future__ import annotations

import asyncio
import logging
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

logger = logging.getLogger(__name__)


@dataclass
class SynthesisRequest:
    connection_id: str
    text: str
    voice_id: str
    timestamp: float
    chunk_size: int = 50
    exaggeration: float = 0.5
    streaming: bool = True
    voice: Optional[Any] = None  # the voice_id's registered speaker embedding (None: default voice)
    stream_frames: int = 0       # > 0: sub-sentence frames of that many mel frames (opt-in; 0 = per sentence)


@dataclass
class AudioChunk:
    connection_id: str
    audio_data: bytes
    chunk_id: int
    is_final: bool
    sample_rate: int = 22050


@dataclass
class QueueStats:
    requests_received: int = 0
    requests_processed: int = 0
    requests_dropped: int = 0
    chunks_sent: int = 0
    active_connections: int = 0

    def as_dict(self):
        return dict(self.__dict__)


class TTSQueueManager:
    def __init__(self, input_queue_size: int = 500, output_queue_size: int = 2000, sample_rate: int = 22050):
        self.input_queue: asyncio.Queue = asyncio.Queue(maxsize=input_queue_size)
        self.output_queues: Dict[str, asyncio.Queue] = {}
        self.output_queue_size = output_queue_size
        self.sample_rate = sample_rate
        self.stats = QueueStats()
        self._tasks: List[asyncio.Task] = []
        self.running = False

    # ------------------------------------------------------------------ lifecycle
    async def start(self):
        if self.running:
            return
        self.running = True
        self._tasks.append(asyncio.create_task(self._report()))

    async def stop(self):
        self.running = False
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        self._tasks.clear()

    async def _report(self):
        while self.running:
            try:
                await asyncio.sleep(10.0)
                q = self.input_queue
                logger.info("queue input=%d/%d connections=%d stats=%s", q.qsize(), q.maxsize,
                            len(self.output_queues), self.stats.as_dict())
                if q.qsize() > 0.8 * q.maxsize:
                    logger.warning("input queue almost full: %d/%d", q.qsize(), q.maxsize)
            except asyncio.CancelledError:
                break

    # ------------------------------------------------------------------ requests
    async def enqueue_request(self, connection_id: str, text: str, voice_id: str = "default", chunk_size: int = 50,
                              exaggeration: float = 0.5, streaming: bool = True, timeout: float = 2.0,
                              voice: Optional[Any] = None, stream_frames: int = 0) -> bool:
        req = SynthesisRequest(connection_id, text, voice_id, time.time(), chunk_size, exaggeration, streaming, voice,
                               stream_frames)
        try:
            # a put that fits starts no timer (wait_for's task and timer handle are a loop hop
            # on every request); a full queue waits up to `timeout`
            try:
                self.input_queue.put_nowait(req)
            except asyncio.QueueFull:
                await asyncio.wait_for(self.input_queue.put(req), timeout=timeout)
        except asyncio.TimeoutError:
            self.stats.requests_dropped += 1
            logger.warning("input queue full, dropping request of %s", connection_id)
            return False
        self.stats.requests_received += 1
        return True

    async def get_next_request(self, timeout: float = 1.0) -> Optional[SynthesisRequest]:
        try:
            return self.input_queue.get_nowait()
        except asyncio.QueueEmpty:
            pass
        try:
            return await asyncio.wait_for(self.input_queue.get(), timeout=timeout)
        except asyncio.TimeoutError:
            return None

    async def take_batch(self, max_items: int, max_wait, first_timeout: Optional[float] = None) -> List[SynthesisRequest]:
        """`max_wait`: seconds, or a callable giving them once the first request is in.
        `first_timeout`: how long to wait for the first request ([] after it); None waits until
        one comes (the batcher's admission loop, which stop() cancels): a plain queue get wakes
        on the put itself, where wait_for's inner task adds two loop hops to every request."""
        if first_timeout is None:
            first = await self.input_queue.get()
        else:
            first = await self.get_next_request(first_timeout)
        if first is None:
            return []
        batch = [first]
        deadline = time.monotonic() + (max_wait() if callable(max_wait) else max_wait)
        while len(batch) < max_items:
            try:
                batch.append(self.input_queue.get_nowait())
                continue
            except asyncio.QueueEmpty:
                pass
            left = deadline - time.monotonic()
            if left <= 0:
                break
            try:
                batch.append(await asyncio.wait_for(self.input_queue.get(), timeout=left))
            except asyncio.TimeoutError:
                break
        return batch

    async def mark_request_done(self, n: int = 1):
        for _ in range(n):
            self.input_queue.task_done()
        self.stats.requests_processed += n

    # ------------------------------------------------------------------ audio
    async def enqueue_audio_chunk(self, connection_id: str, audio_data: bytes, chunk_id: int,
                                  is_final: bool = False) -> bool:
        q = self.output_queues.get(connection_id)
        if q is None:
            return False
        chunk = AudioChunk(connection_id, audio_data, chunk_id, is_final, self.sample_rate)
        try:
            q.put_nowait(chunk)
        except asyncio.QueueFull:
            try:
                await asyncio.wait_for(q.put(chunk), timeout=0.1)
            except asyncio.TimeoutError:
                logger.warning("output queue full for %s, dropping chunk %d", connection_id, chunk_id)
                return False
        self.stats.chunks_sent += 1
        return True

    def register_connection(self, connection_id: str) -> asyncio.Queue:
        q: asyncio.Queue = asyncio.Queue(maxsize=self.output_queue_size)
        self.output_queues[connection_id] = q
        self.stats.active_connections = len(self.output_queues)
        return q

    def unregister_connection(self, connection_id: str):
        q = self.output_queues.pop(connection_id, None)
        if q is not None:
            while not q.empty():
                q.get_nowait()
        self.stats.active_connections = len(self.output_queues)

    def get_metrics(self) -> dict:
        m = self.stats.as_dict()
        m["input_queue_size"] = self.input_queue.qsize()
        m["output_queues_count"] = len(self.output_queues)
        m["total_output_queue_items"] = sum(q.qsize() for q in self.output_queues.values())
        return m

    async def wait_until_empty(self, timeout: float = 30.0) -> bool:
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            if self.input_queue.empty() and all(q.empty() for q in self.output_queues.values()):
                return True
            await asyncio.sleep(0.1)
        return False
