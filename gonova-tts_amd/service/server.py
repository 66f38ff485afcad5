"""WebSocket TTS service on the MI355X engine, protocol-compatible with the reference
(`services/tts/server.py`):

* `WS /v1/stream/tts` (`server.py:421-444`): per-IP rate limit (100 per 60 s) and a
  connection cap, both rejecting with close code 1008; messages
  `{"type":"synthesize","text",...,"voice_id","chunk_size","exaggeration","streaming"}`
  (`server.py:215-224`); replies are one binary frame of raw float32 PCM per sentence and
  `{"type":"synthesis_complete","chunk_id":N}` (`server.py:279-286`);
  `register_voice` / `list_voices` answer in the reference's message shapes
  (`server.py:226-256`) -- this engine has no voice cloning, so registration reports
  an error and the list is empty;
* opt-in sub-sentence streaming: a `"stream_frames": N` field (or the
  service's `stream_frames` default) splits each sentence's audio into frames of N mel frames
  (N x 256 samples, the last one shorter) as the vocoder produces them, in sentence order, with
  the same final marker (its chunk_id = frames sent).  The reference accepts `streaming` /
  `chunk_size` and ignores them (`core/synthesizer.py:226,245,320-321`); so does this service,
  and without `stream_frames` the framing stays one frame per sentence;
* `GET /health` 503 until the model is loaded (`server.py:450-454`), plus the sample rate
  the PCM is in (the reference never tells clients its 24 kHz);
* `GET /metrics`: the queue metrics dict (`server.py:478-481`).

The serial worker is replaced by `DynamicBatcher` (cross-request batching).  The model
comes from a factory so tests can inject a CPU fake; production uses `GonovaTTS`.
"""
import asyncio
import json
import logging
import os
import time
import uuid
from typing import Callable, Optional

import numpy as np

from .batcher import DynamicBatcher
from .queues import TTSQueueManager

logger = logging.getLogger(__name__)


# smallest sub-sentence frame (mel frames) a request gets: 2 x GonovaTTS.STREAM_CONTEXT, so a
# chunk's window is at most half context
MIN_STREAM_FRAMES = 32


# the sentences the reference warms its model up with, in order (synthesizer.py:197-207)
WARMUP_TEXTS = ("Hello.", "Hello, this is a warmup test.",
                "The quick brown fox jumps over the lazy dog, and this is a longer sentence to warm up the model properly.")


class RateLimiter:
    """Sliding-window admission per client (reference server.py:358-382)."""

    def __init__(self, max_requests: int = 100, window: float = 60.0):
        self.max_requests = max_requests
        self.window = window
        self.hits = {}

    def check(self, client: str) -> bool:
        now = time.time()
        recent = [t for t in self.hits.get(client, []) if now - t < self.window]
        if len(recent) >= self.max_requests:
            self.hits[client] = recent
            return False
        recent.append(now)
        self.hits[client] = recent
        return True


class TTSService:
    def __init__(self, model_factory: Callable, max_connections: int = 50, chunk_size: int = 50,
                 max_sentences: int = 32, max_wait: float = 0.004, notify_errors: bool = False,
                 device: str = "cuda", device_index: int = 0, stream_frames: int = 0,
                 min_stream_frames: int = MIN_STREAM_FRAMES, devices: Optional[list] = None,
                 idle_wait: float = 0.0):
        """devices: opt-in fan-out over the node's GPUs, e.g. ["cuda:0", "cuda:1"]: model_factory is
        then called once per device (model_factory(device)) and each engine pulls its next batch from
        the batcher's shared work list whenever it is free (batcher.py); default None = one model_factory() model, the
        reference's one-GPU-per-process shape (server.py:397-400)."""
        self.model_factory = model_factory
        self.devices = list(devices) if devices else None
        self.models = []
        self.max_connections = max_connections
        self.chunk_size = chunk_size
        self.device = device
        self.device_index = device_index
        self.model = None
        self.is_loaded = False
        self.queues: Optional[TTSQueueManager] = None
        self.batcher: Optional[DynamicBatcher] = None
        self.rate_limiter = RateLimiter()
        self.active_connections = 0
        self.sockets = {}
        self.voices = {}      # voice_id -> speaker embedding (register_voice)
        self.voice_info = {}  # voice_id -> description
        # the reference voice manager's counters (voice_manager.py:262-267)
        self.voice_counts = {"registrations": 0, "cache_hits": 0, "cache_misses": 0}
        self.max_sentences = max_sentences
        self.max_wait = max_wait
        self.idle_wait = idle_wait  # the gathering window while an engine is idle (batcher.py)
        self.notify_errors = notify_errors
        self.min_stream_frames = max(1, int(min_stream_frames))
        self.stream_frames = self._stream_frames(stream_frames)
        self._task = None

    async def start(self):
        loop = asyncio.get_running_loop()
        if self.devices:
            self.models = [await loop.run_in_executor(None, self.model_factory, d) for d in self.devices]
        else:
            self.models = [await loop.run_in_executor(None, self.model_factory)]
        self.model = self.models[0]
        for m in self.models:
            for text in WARMUP_TEXTS:  # the reference's three warmups (synthesizer.py:197-207)
                await loop.run_in_executor(None, m.generate_batch, [text])
        if self.stream_frames and not self.can_stream():
            raise ValueError("stream_frames needs the vocoder's native sample rate: this model resamples "
                             f"to {getattr(self.model, 'sr', None)} Hz, which needs filter context across frames")
        sr = getattr(self.model, "sr", 22050)
        self.queues = TTSQueueManager(sample_rate=sr)
        await self.queues.start()
        self.batcher = DynamicBatcher(self.queues, self.model.generate_batch, max_sentences=self.max_sentences,
                                      max_wait=self.max_wait, idle_wait=self.idle_wait,
                                      notify_errors=self.notify_errors,
                                      send_error=self._send_error,
                                      synth_stream=getattr(self.model, "stream_batch", None), sample_rate=sr,
                                      synth_batches=[m.generate_batch for m in self.models],
                                      synth_streams=[getattr(m, "stream_batch", None) for m in self.models])
        self._task = asyncio.create_task(self.batcher.run())
        self.is_loaded = True

    def can_stream(self) -> bool:
        """Sub-sentence frames come straight from the vocoder's chunks, at its native rate; a
        model that resamples (e.g. to the 24 kHz the reference's clients assume) cannot cut its
        output at chunk edges without the resampler's filter context (model.stream_batch)."""
        m = self.model
        return getattr(m, "stream_batch", None) is not None and getattr(m, "sr", 0) == getattr(m, "native_sr", getattr(m, "sr", 0))

    def _stream_frames(self, v) -> int:
        """A request's (or the service default's) `stream_frames`: 0 = one frame per sentence;
        otherwise at least `min_stream_frames`.  Each vocoder chunk runs a window of the chunk plus
        2 x STREAM_CONTEXT frames and one device-to-host copy, so a tiny value (1 frame: a 33-frame
        window and a host sync per mel frame, ~860 chunks for a 10 s sentence) would let one
        request hold the shared batcher for every other connection; smaller values round up."""
        f = _frames(v)
        return 0 if f == 0 else max(f, self.min_stream_frames)

    async def _send_error(self, conn_id: str, message: str):
        ws = self.sockets.get(conn_id)
        if ws is not None:
            try:
                await ws.send_json({"type": "synthesis_error", "message": message})
            except Exception:
                pass

    async def shutdown(self):
        if self.queues is not None:
            await self.queues.wait_until_empty(timeout=30.0)
        if self.batcher is not None:
            self.batcher.stop()
        if self._task is not None:
            self._task.cancel()
            await asyncio.gather(self._task, return_exceptions=True)
        if self.queues is not None:
            await self.queues.stop()
        for m in self.models:
            eng = getattr(m, "engine", None)
            if eng is not None:
                eng.close()
        self.is_loaded = False

    async def handle_connection(self, ws, conn_id: str):
        from starlette.websockets import WebSocketDisconnect
        out_q = self.queues.register_connection(conn_id)
        self.sockets[conn_id] = ws
        self.active_connections += 1

        async def receive():
            async for message in ws.iter_text():
                # one bad message never ends the connection: the reference wraps each message
                # in try/except and keeps going (server.py:258-263)
                try:
                    data = json.loads(message)
                    if not isinstance(data, dict):
                        raise ValueError("message is not a JSON object")
                    await self.handle_message(ws, conn_id, data)
                except WebSocketDisconnect:
                    raise
                except Exception as e:  # noqa: BLE001
                    logger.error("message handling error on %s: %s", conn_id, e)

        async def send():
            while True:
                # (wait_for, not a plain get: with a plain get, TestClient's session teardown --
                # disconnect, then its cancel scope -- ended in CancelledError ~1 run in 6)
                try:
                    chunk = await asyncio.wait_for(out_q.get(), timeout=1.0)
                except asyncio.TimeoutError:
                    continue
                try:
                    if chunk.is_final:
                        await ws.send_json({"type": "synthesis_complete", "chunk_id": chunk.chunk_id})
                    else:
                        await ws.send_bytes(chunk.audio_data)
                except WebSocketDisconnect:
                    break

        tasks = [asyncio.create_task(receive()), asyncio.create_task(send())]
        try:
            await asyncio.wait(tasks, return_when=asyncio.FIRST_COMPLETED)
        except WebSocketDisconnect:
            pass
        finally:
            # bookkeeping first, before any await: when the handler itself is cancelled (the ASGI
            # server tearing the connection down), every later await raises again and would skip it
            for t in tasks:
                t.cancel()
            self.queues.unregister_connection(conn_id)
            self.sockets.pop(conn_id, None)
            self.active_connections -= 1
            await asyncio.gather(*tasks, return_exceptions=True)

    async def handle_message(self, ws, conn_id: str, data: dict):
        """One client message (reference server.py:215-256)."""
        kind = data.get("type")
        if kind == "synthesize":
            vid = data.get("voice_id", "default")
            text = data.get("text", "")
            if not isinstance(text, str):
                raise ValueError("text must be a string")
            try:
                frames = self._stream_frames(data.get("stream_frames", self.stream_frames))
                if frames and not self.can_stream():
                    raise ValueError("stream_frames is not available: this model resamples to "
                                     f"{getattr(self.model, 'sr', None)} Hz; omit it for one frame per sentence")
            except ValueError as e:
                # a request refused before it is queued: the client is told (reference error shape,
                # server.py:244-247), instead of waiting for a marker that never comes
                await ws.send_json({"type": "error", "message": f"Synthesis request refused: {e}"})
                return
            # unknown voices fall back to the default voice (reference server.py:127-138)
            if vid != "default":
                self.voice_counts["cache_hits" if isinstance(vid, str) and vid in self.voices else "cache_misses"] += 1
            await self.queues.enqueue_request(
                connection_id=conn_id, text=text, voice_id=vid,
                chunk_size=data.get("chunk_size", self.chunk_size),
                exaggeration=data.get("exaggeration", 0.5), streaming=data.get("streaming", True),
                voice=self.voices.get(vid) if isinstance(vid, str) else None, stream_frames=frames)
        elif kind == "register_voice":
            await ws.send_json(self.register_voice(data))
        elif kind == "list_voices":
            await ws.send_json({"type": "voice_list", "voices": self.list_voices()})

    def register_voice(self, data: dict) -> dict:
        """`register_voice` (reference server.py:226-248): this engine conditions on speaker
        embeddings (HF speaker_embed_dim), so a voice is registered from
        `{"voice_id", "speaker_embedding": [E floats], "description"}`.  `reference_audio`
        alone is refused -- computing an embedding from audio needs a speaker encoder this
        engine does not have -- in the reference's error shape."""
        vid = data.get("voice_id")
        emb = data.get("speaker_embedding")
        dim = getattr(getattr(self.model, "acoustic_cfg", None), "speaker_embed_dim", None)
        if not vid or not isinstance(vid, str) or emb is None:
            return {"type": "error", "message": "Voice registration failed: send voice_id and speaker_embedding "
                                                "(no speaker encoder for reference_audio)"}
        try:
            v = np.asarray(emb, np.float32).reshape(-1)
        except (TypeError, ValueError):
            return {"type": "error", "message": "Voice registration failed: speaker_embedding must be a list of numbers"}
        if not dim or v.size != dim or not np.all(np.isfinite(v)):
            return {"type": "error", "message": f"Voice registration failed: the model takes {dim or 0}-value "
                                                f"speaker embeddings, got {v.size}"}
        self.voices[vid] = v
        self.voice_info[vid] = data.get("description", "")
        self.voice_counts["registrations"] += 1
        return {"type": "voice_registered", "voice_id": vid}

    def list_voices(self) -> list:
        return [{"voice_id": k, "description": self.voice_info.get(k, ""), "path": "", "is_cached": True}
                for k in self.voices]

    def health(self):
        info = {"status": "healthy", "device": f"{self.device}:{self.device_index}",
                "devices": list(self.devices) if self.devices else [f"{self.device}:{self.device_index}"],
                "sample_rate": getattr(self.model, "sr", 22050), "active_connections": self.active_connections,
                "queue_metrics": self.queues.get_metrics(), "synthesizer_stats": self.batcher.get_stats(),
                "voice_stats": {"total_voices": len(self.voices), "cached_in_memory": len(self.voices),
                                **self.voice_counts},
                "gpu": {}}
        try:
            import torch
            if torch.cuda.is_available():
                i = self.device_index
                gpu = {"gpu_id": i, "gpu_name": torch.cuda.get_device_name(i),
                       "memory_allocated_gb": torch.cuda.memory_allocated(i) / 1e9,
                       "memory_reserved_gb": torch.cuda.memory_reserved(i) / 1e9}
                # the engine's own weights and workspaces (hipMalloc'd in libtts_hip.so, invisible
                # to torch's allocator): per engine device, and added into memory_allocated_gb
                from ..engine import device_bytes, parse_device
                devs = sorted({parse_device(d) for d in self.devices}) if self.devices else [i]
                eng = {d: device_bytes(d) / 1e9 for d in devs}
                gpu["engine_memory_gb"] = eng.get(i, 0.0)
                gpu["engine_memory_gb_by_device"] = {str(d): v for d, v in eng.items()}
                gpu["memory_allocated_gb"] += eng.get(i, 0.0)
                info["gpu"] = gpu
        except Exception as e:  # noqa: BLE001 -- health must answer
            logger.warning("gpu info unavailable: %s", e)
        return info


def _frames(v) -> int:
    """A `stream_frames` value: a whole number of mel frames, 0 (per-sentence frames) to 4096."""
    if isinstance(v, bool) or not isinstance(v, int) or not 0 <= v <= 4096:
        raise ValueError(f"stream_frames must be an integer in [0, 4096], got {v!r}")
    return v


def create_app(model_factory: Optional[Callable] = None, **service_kwargs):
    from fastapi import FastAPI, WebSocket, status
    from fastapi.responses import JSONResponse

    if model_factory is None:
        def model_factory(device: str = "cuda:0"):
            from ..model import GonovaTTS
            sr = os.environ.get("TTS_SAMPLE_RATE")  # e.g. 24000: the rate the reference's clients assume
            return GonovaTTS.from_pretrained(device=device, ckpt_dir=os.environ.get("TTS_CKPT_DIR"),
                                             sample_rate=int(sr) if sr else None)
        if "devices" not in service_kwargs and os.environ.get("TTS_DEVICES"):
            # e.g. TTS_DEVICES=cuda:0,cuda:1: one engine per listed GPU in this process
            service_kwargs["devices"] = [d.strip() for d in os.environ["TTS_DEVICES"].split(",") if d.strip()]

    app = FastAPI(title="TTS Service (MI355X)", version="0.1.0")
    svc = TTSService(model_factory, **service_kwargs)
    app.state.service = svc

    @app.on_event("startup")
    async def _startup():
        await svc.start()

    @app.on_event("shutdown")
    async def _shutdown():
        await svc.shutdown()

    @app.websocket("/v1/stream/tts")
    async def ws_endpoint(websocket: WebSocket):
        client = websocket.client.host if websocket.client else "unknown"
        if not svc.rate_limiter.check(client):
            await websocket.close(code=status.WS_1008_POLICY_VIOLATION, reason="Rate limit exceeded")
            return
        if svc.active_connections >= svc.max_connections:
            await websocket.close(code=status.WS_1008_POLICY_VIOLATION, reason="Max connections reached")
            return
        await websocket.accept()
        await svc.handle_connection(websocket, str(uuid.uuid4()))

    @app.get("/health")
    async def health():
        if not svc.is_loaded:
            return JSONResponse(status_code=503, content={"status": "unhealthy", "reason": "Model not loaded"})
        return svc.health()

    @app.get("/metrics")
    async def metrics():
        return svc.queues.get_metrics() if svc.queues else {}

    return app


def main():  # pragma: no cover - process entry
    import uvicorn
    uvicorn.run(create_app(), host="0.0.0.0", port=int(os.getenv("TTS_PORT", "8002")), log_level="info")


if __name__ == "__main__":  # pragma: no cover
    main()
