"""Service protocol tests on CPU with a fake model (no GPU): WS framing and final marker
as in the reference (server.py:215-224, 279-286), /health 503 rule, /metrics keys,
cross-request batching, error path."""
import json
import threading
import asyncio
import time

import numpy as np
import pytest

pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from gonova_tts_amd.service.server import create_app  # noqa: E402


class FakeModel:
    sr = 22050

    def __init__(self, delay=0.0, fail_on=None):
        self.batches = []
        self.delay = delay
        self.fail_on = fail_on
        self.lock = threading.Lock()

    def generate_batch(self, texts):
        if self.fail_on and any(self.fail_on in t for t in texts):
            raise RuntimeError("boom")
        time.sleep(self.delay)
        with self.lock:
            self.batches.append(list(texts))
        return [np.full(100 * len(t), len(t), np.float32) for t in texts]


def recv_until_complete(ws):
    frames = []
    while True:
        m = ws.receive()
        if m.get("bytes") is not None:
            frames.append(np.frombuffer(m["bytes"], np.float32))
        elif m.get("text") is not None:
            return frames, json.loads(m["text"])


def test_ws_protocol_per_sentence_frames_and_final_marker():
    model = FakeModel()
    app = create_app(lambda: model)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": "Hello world. This is a test! Is it working? yes it is."}))
            frames, final = recv_until_complete(ws)
        assert final == {"type": "synthesis_complete", "chunk_id": 3}
        assert [len(f) for f in frames] == [1200, 1500, 2500]
        assert all(f.dtype == np.float32 for f in frames)
        m = c.get("/metrics").json()
        for k in ("requests_received", "requests_processed", "requests_dropped", "chunks_sent",
                  "active_connections", "input_queue_size", "output_queues_count", "total_output_queue_items"):
            assert k in m
        assert m["chunks_sent"] == 4  # final marker counts (reference queue_manager.py:232)
        h = c.get("/health").json()
        assert h["status"] == "healthy" and h["sample_rate"] == 22050


def test_empty_text_gets_only_the_marker_and_voice_routes():
    app = create_app(lambda: FakeModel())
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": "   "}))
            frames, final = recv_until_complete(ws)
            assert frames == [] and final["chunk_id"] == 0
            ws.send_text(json.dumps({"type": "list_voices"}))
            assert ws.receive_json() == {"type": "voice_list", "voices": []}
            ws.send_text(json.dumps({"type": "register_voice", "voice_id": "x", "reference_audio": "AA=="}))
            assert ws.receive_json()["type"] == "error"


def test_health_is_503_until_loaded():
    from gonova_tts_amd.service.server import TTSService
    app = create_app(lambda: FakeModel())
    svc = app.state.service
    assert isinstance(svc, TTSService) and not svc.is_loaded
    # without running the startup event the model is not loaded
    from starlette.testclient import TestClient as TC
    c = TC(app)  # no context manager -> startup not run
    r = c.get("/health")
    assert r.status_code == 503 and r.json()["status"] == "unhealthy"


def test_concurrent_connections_are_batched_together():
    model = FakeModel(delay=0.05)
    app = create_app(lambda: model, max_wait=0.05)
    results = {}
    with TestClient(app) as c:
        def client(i):
            with c.websocket_connect("/v1/stream/tts") as ws:
                ws.send_text(json.dumps({"type": "synthesize", "text": f"Sentence number {i} here. And one more."}))
                results[i] = recv_until_complete(ws)
        ts = [threading.Thread(target=client, args=(i,)) for i in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=30)
    assert len(results) == 6
    for i, (frames, final) in results.items():
        assert final["chunk_id"] == 2 and len(frames) == 2
    assert max(len(b) for b in model.batches) > 2  # sentences of different connections shared an engine pass


def test_lone_request_does_not_wait_for_the_gathering_window():
    """With the engine idle a request starts at once (idle_wait, default 0): max_wait only gathers
    while every engine is busy, so a lone sentence is not delayed by it (C1's first frame)."""
    app = create_app(lambda: FakeModel(), max_wait=1.0)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            t0 = time.perf_counter()
            ws.send_text(json.dumps({"type": "synthesize", "text": "Just one sentence."}))
            frames, final = recv_until_complete(ws)
            dt = time.perf_counter() - t0
    assert len(frames) == 1 and final["chunk_id"] == 1
    assert dt < 0.5, dt


def test_failure_follows_reference_by_default_and_notifies_when_asked():
    app = create_app(lambda: FakeModel(fail_on="bad"), notify_errors=True)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": "bad input"}))
            err = ws.receive_json()
            assert err["type"] == "synthesis_error"
            fin = ws.receive_json()
            assert fin["type"] == "synthesis_complete"


class FakeSpeakerModel(FakeModel):
    """Multi-speaker fake: records the per-sentence voices the batcher passes."""

    class acoustic_cfg:
        speaker_embed_dim = 4

    def __init__(self):
        super().__init__()
        self.voices = []

    def generate_batch(self, texts, speaker_embeddings=None):
        with self.lock:
            self.voices.append(None if speaker_embeddings is None else
                               [None if e is None else np.asarray(e).tolist() for e in speaker_embeddings])
        return super().generate_batch(texts)


def test_registered_voice_reaches_the_model_per_sentence():
    """voice_id -> registered speaker embedding -> generate_batch(speaker_embeddings=...)
    (the reference's voice_id -> audio_prompt_path, server.py:127-138, 226-256)."""
    model = FakeSpeakerModel()
    app = create_app(lambda: model)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "register_voice", "voice_id": "ann", "speaker_embedding": [1, 2, 3, 4],
                                     "description": "test"}))
            assert ws.receive_json() == {"type": "voice_registered", "voice_id": "ann"}
            ws.send_text(json.dumps({"type": "register_voice", "voice_id": "bad", "speaker_embedding": [1, 2]}))
            assert ws.receive_json()["type"] == "error"
            ws.send_text(json.dumps({"type": "list_voices"}))
            v = ws.receive_json()["voices"]
            assert [x["voice_id"] for x in v] == ["ann"] and v[0]["description"] == "test"
            ws.send_text(json.dumps({"type": "synthesize", "text": "Hi there. Bye now.", "voice_id": "ann"}))
            frames, final = recv_until_complete(ws)
            assert len(frames) == 2 and final["chunk_id"] == 2
            ws.send_text(json.dumps({"type": "synthesize", "text": "Plain voice.", "voice_id": "nobody"}))
            recv_until_complete(ws)
        assert [[1.0, 2.0, 3.0, 4.0]] * 2 in model.voices  # both sentences carried the voice
        assert None in model.voices                        # unknown voice -> default voice
        assert c.get("/health").json()["voice_stats"]["total_voices"] == 1


def test_bad_messages_do_not_end_the_connection():
    """Valid JSON that is not an object, a non-numeric embedding and a non-string text are
    logged and skipped; the connection keeps working (reference server.py:258-263)."""
    app = create_app(lambda: FakeSpeakerModel())
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text("[1, 2, 3]")
            ws.send_text("not json")
            ws.send_text(json.dumps({"type": "synthesize", "text": 12}))
            ws.send_text(json.dumps({"type": "register_voice", "voice_id": "v", "speaker_embedding": "abc"}))
            assert ws.receive_json()["type"] == "error"
            ws.send_text(json.dumps({"type": "synthesize", "text": "Still here."}))
            frames, final = recv_until_complete(ws)
            assert len(frames) == 1 and final == {"type": "synthesis_complete", "chunk_id": 1}


def test_ws_transcript_matches_reference_fixture():
    """The reference service itself, recorded under TestClient with a fake chatterbox model
    (tests/golden/make_ws_golden.py -> ws_transcript.json), against this build's
    service driven with the same fake outputs (tests/golden/ws_fake.py): /health's 503 before
    load (server.py:447-454), every binary frame of every request byte for byte (one frame of
    raw float32 PCM per sentence, server.py:150-156, 279-280), the final
    synthesis_complete message (server.py:159-164, 283-286), the sentences handed to the model
    and the warmup texts (synthesizer.py:197-207, 257), and /metrics after the session
    (queue_manager.py:282-291; the final marker counts as a chunk)."""
    import hashlib
    import os

    from tests.golden.ws_fake import REQUESTS, fake_audio

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ws_transcript.json")))
    seen = []

    class TranscriptModel:
        sr = 24000

        def generate_batch(self, texts):
            seen.extend(texts)
            return [fake_audio(t) for t in texts]

    app = create_app(lambda: TranscriptModel())
    r = TestClient(app).get("/health")  # startup has not run: no model
    assert {"status_code": r.status_code, "body": r.json()} == gold["health_before_load"]
    with TestClient(app) as c:
        warm = list(seen)
        with c.websocket_connect("/v1/stream/tts") as ws:
            for req, g in zip(REQUESTS, gold["requests"]):
                assert req == g["message"]
                ws.send_text(json.dumps(req))
                frames = []
                while True:
                    m = ws.receive()
                    if m.get("bytes") is not None:
                        frames.append({"bytes": len(m["bytes"]), "sha256": hashlib.sha256(m["bytes"]).hexdigest()})
                    elif m.get("text") is not None:
                        final = json.loads(m["text"])
                        break
                assert frames == g["frames"], req["text"]
                assert final == g["final"]
        # the server unregisters the closed connection asynchronously
        for _ in range(100):
            metrics = c.get("/metrics").json()
            if metrics["active_connections"] == 0:
                break
            time.sleep(0.02)
        # /health's 200 body keeps the reference's shape (server.py:456-475, synthesizer.py:411-420):
        # every key the reference reports at every level (this service adds its own beside them),
        # and the same request counts
        r = c.get("/health")
        hg = gold["health_after_requests"]
        assert r.status_code == hg["status_code"]
        h = r.json()
        assert set(hg["keys"]) <= set(h), sorted(set(hg["keys"]) - set(h))
        for k, keys in hg["nested_keys"].items():
            assert set(keys) <= set(h[k]), (k, sorted(set(keys) - set(h[k])))
        for k, v in hg["synthesizer_counts"].items():
            assert h["synthesizer_stats"][k] == v, k
        s = h["synthesizer_stats"]
        assert s["total_latency"] >= s["first_chunk_latency"] > 0
        assert abs(s["avg_latency"] - s["total_latency"] / s["syntheses"]) < 1e-12
    ref_texts = [x["text"] for x in gold["generate_calls"]]
    assert warm == ref_texts[:len(warm)]  # the reference's warmup sentences, in order
    # then every sentence as the reference split them (the batcher orders a batch by length, so
    # the engine sees them in another order; the frames above came back in the reference's)
    assert sorted(seen[len(warm):]) == sorted(ref_texts[len(warm):])
    for k, v in gold["metrics"].items():
        assert metrics[k] == v, (k, metrics[k], v)


class FakeStreamModel(FakeModel):
    """Fake with stream_batch: a sentence of n characters is 100 n samples of value n, cut into
    pieces of chunk_frames * 10 samples (the last shorter), yielded chunk by chunk for the batch."""

    def __init__(self):
        super().__init__()
        self.stream_calls = []

    def stream_batch(self, texts, chunk_frames, speaker_embeddings=None):
        with self.lock:
            self.stream_calls.append((list(texts), chunk_frames))
        step = chunk_frames * 10
        full = [np.full(100 * len(t), len(t), np.float32) for t in texts]
        n = max(len(a) for a in full)
        for c0 in range(0, n, step):
            yield [(i, a[c0:c0 + step], c0 + step >= len(a)) for i, a in enumerate(full) if c0 < len(a)]


def test_stream_frames_split_sentences_in_order():
    """Opt-in sub-sentence frames: a request with stream_frames gets each
    sentence in pieces, in sentence order, that concatenate to the per-sentence audio; the final
    marker's chunk_id counts the frames; a request without it in the same session keeps the
    reference's one frame per sentence; a bad stream_frames value is refused with an error message
    in the reference's error shape (nothing is queued for it)."""
    model = FakeStreamModel()
    app = create_app(lambda: model)
    text = "Hello world. This is a test! Is it working? yes it is."
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": text, "stream_frames": 40}))
            frames, final = recv_until_complete(ws)
            assert [len(f) for f in frames] == [400] * 3 + [400] * 3 + [300] + [400] * 6 + [100]
            assert final == {"type": "synthesis_complete", "chunk_id": len(frames)}
            want = np.concatenate([np.full(100 * n, n, np.float32) for n in (12, 15, 25)])
            np.testing.assert_array_equal(np.concatenate(frames), want)
            ws.send_text(json.dumps({"type": "synthesize", "text": "One. Two!", "stream_frames": -3}))
            err = ws.receive_json()
            assert err["type"] == "error" and "stream_frames" in err["message"]
            ws.send_text(json.dumps({"type": "synthesize", "text": text}))
            frames, final = recv_until_complete(ws)
            assert [len(f) for f in frames] == [1200, 1500, 2500] and final["chunk_id"] == 3
    assert model.stream_calls == [(["Hello world.", "This is a test!", "Is it working? yes it is."], 40)]


def test_stream_frames_service_default():
    model = FakeStreamModel()
    app = create_app(lambda: model, stream_frames=100)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": "Short one. And a much longer second sentence here."}))
            frames, final = recv_until_complete(ws)
            # sentence 1: 1000 samples = one piece; sentence 2: 3900 samples = 3 pieces
            assert [len(f) for f in frames] == [1000, 1000, 1000, 1000, 900] and final["chunk_id"] == 5
            ws.send_text(json.dumps({"type": "synthesize", "text": "Per sentence again.", "stream_frames": 0}))
            frames, final = recv_until_complete(ws)
            assert [len(f) for f in frames] == [1900] and final["chunk_id"] == 1


def test_stream_frames_floor_and_resampling_refusal():
    """A tiny stream_frames rounds up to the service floor (one request cannot make the shared
    batcher run a vocoder window and a host copy per mel frame); a model that resamples cannot cut
    its output at chunk edges, so the service refuses stream_frames for it with an error message
    and keeps serving per-sentence frames; the batcher's audio seconds use the model's rate."""
    model = FakeStreamModel()
    app = create_app(lambda: model)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": "Hello world.", "stream_frames": 1}))
            frames, final = recv_until_complete(ws)
            assert [len(f) for f in frames] == [320, 320, 320, 240]
        assert model.stream_calls == [(["Hello world."], 32)]

    class Resampling(FakeStreamModel):
        sr, native_sr = 24000, 22050

    model = Resampling()
    app = create_app(lambda: model)
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": "Hello world.", "stream_frames": 64}))
            err = ws.receive_json()
            assert err["type"] == "error" and "resamples" in err["message"]
            ws.send_text(json.dumps({"type": "synthesize", "text": "Hello world."}))
            frames, final = recv_until_complete(ws)
            assert [len(f) for f in frames] == [1200] and final["chunk_id"] == 1
        stats = app.state.service.batcher.stats
        assert abs(stats["audio_seconds"] - 1200 / 24000) < 1e-9
        assert model.stream_calls == []
    with pytest.raises(ValueError, match="native sample rate"):
        with TestClient(create_app(lambda: Resampling(), stream_frames=64)):
            pass


def test_stream_producer_stops_when_delivery_fails():
    """If delivering a chunk fails, the streaming producer thread stops at the next chunk and
    closes the model's generator (releasing its lock) instead of synthesizing the rest of the
    batch into a queue nobody reads."""
    import asyncio
    from gonova_tts_amd.service.batcher import DynamicBatcher

    state = {"yielded": 0, "closed": False}

    def stream(texts, frames):
        try:
            for i in range(1000):
                state["yielded"] += 1
                time.sleep(0.002)
                yield [(0, np.zeros(4, np.float32), False)]
        finally:
            state["closed"] = True

    b = DynamicBatcher(None, None, synth_stream=stream)

    async def deliver(item):
        raise OSError("socket gone")

    async def main():
        with pytest.raises(OSError):
            await b._stream(asyncio.get_running_loop(), ["x"], 32, {}, deliver)

    asyncio.run(main())
    assert state["closed"] and state["yielded"] < 50


class FakeDeviceModel(FakeModel):
    """One fake engine per 'device': records which sentences it synthesized."""

    def __init__(self, device, delay=0.0):
        super().__init__(delay=delay)
        self.device = device


def test_multi_device_fan_out_keeps_order_and_balances():
    """Opt-in fan-out over the node's GPUs (TTSService(devices=[...])):
    the factory makes one engine per device, both engines pull batches from the batcher's shared
    work list at the same time, and every request still gets its frames in sentence order followed
    by the marker -- the same frames a single engine produces."""
    made = []

    def factory(device):
        m = FakeDeviceModel(device, delay=0.05)
        made.append(m)
        return m

    app = create_app(factory, devices=["cuda:0", "cuda:1"], max_wait=0.05, max_sentences=4)
    texts = {i: " ".join(f"Sentence {i} number {j} {'x' * (3 * j + i)}." for j in range(5)) for i in range(4)}
    results = {}
    with TestClient(app) as c:
        assert c.get("/health").json()["devices"] == ["cuda:0", "cuda:1"]

        def client(i):
            with c.websocket_connect("/v1/stream/tts") as ws:
                ws.send_text(json.dumps({"type": "synthesize", "text": texts[i]}))
                results[i] = recv_until_complete(ws)
        ts = [threading.Thread(target=client, args=(i,)) for i in texts]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=30)
        stats = app.state.service.batcher.stats
    assert [m.device for m in made] == ["cuda:0", "cuda:1"]
    from gonova_tts_amd.text import split_into_sentences
    for i, (frames, final) in results.items():
        sents = split_into_sentences(texts[i])
        assert final == {"type": "synthesis_complete", "chunk_id": len(sents)}
        assert [len(f) for f in frames] == [100 * len(s) for s in sents]
        for f, s in zip(frames, sents):
            assert np.all(f == len(s))
    # both engines got work (warmups excluded) and neither carried most of it: engines pull
    # batches when they come free, so the split follows timing, not a fixed deal
    work = [sum(len(t) for b in m.batches[3:] for t in b) for m in made]
    assert all(w > 0 for w in work), work
    assert min(work) >= 0.25 * sum(work), work
    assert sum(stats["engine_sentences"]) == 20 and min(stats["engine_sentences"]) > 0


class TimedModel(FakeModel):
    """A fake engine that records when each of its batches ran."""

    def __init__(self, device="cuda:0", delay=0.0):
        super().__init__(delay=delay)
        self.device = device
        self.spans = []

    def generate_batch(self, texts):
        t0 = time.monotonic()
        out = super().generate_batch(texts)
        self.spans.append((t0, time.monotonic(), len(texts)))
        return out


def test_continuous_batcher_keeps_unequal_engines_busy():
    """Continuous batching across engines of unequal speed: each engine pulls
    its next batch from the shared work list as soon as it is free, so the fast engine is never
    held for the slow one (no gap between its batches while work is queued) and does most of the
    work; every request still gets its frames in sentence order, then the marker."""
    made = {}

    def factory(device):
        made[device] = TimedModel(device, delay=0.02 if device == "cuda:0" else 0.2)
        return made[device]

    app = create_app(factory, devices=["cuda:0", "cuda:1"], max_wait=0.05, max_sentences=2)
    texts = {i: " ".join(f"Sentence {i} number {j} {'y' * (2 * j + i)}." for j in range(6)) for i in range(4)}
    results = {}
    with TestClient(app) as c:
        for m in made.values():
            m.spans.clear()  # (warmups)

        def client(i):
            with c.websocket_connect("/v1/stream/tts") as ws:
                ws.send_text(json.dumps({"type": "synthesize", "text": texts[i]}))
                results[i] = recv_until_complete(ws)
        ts = [threading.Thread(target=client, args=(i,)) for i in texts]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
    from gonova_tts_amd.text import split_into_sentences
    for i, (frames, final) in results.items():
        sents = split_into_sentences(texts[i])
        assert final == {"type": "synthesis_complete", "chunk_id": len(sents)}
        assert [len(f) for f in frames] == [100 * len(s) for s in sents]
    fast, slow = made["cuda:0"], made["cuda:1"]
    n_fast, n_slow = sum(n for *_, n in fast.spans), sum(n for *_, n in slow.spans)
    assert n_fast + n_slow == 24 and n_fast >= 3 * n_slow > 0, (n_fast, n_slow)
    # the fast engine's batches follow each other back to back until the list runs dry (a round-
    # based batcher would park it until the slow engine's batch of the round ends)
    gaps = [b[0] - a[1] for a, b in zip(fast.spans, fast.spans[1:])]
    assert max(gaps) < 0.1, gaps


def test_request_arriving_mid_stream_starts_before_the_earlier_one_ends():
    """Admission between engine batches: a request sent while an earlier, long request is being
    synthesized gets its sentence into the next engine batch (its first sentence goes ahead of the
    earlier request's later ones) and completes before the earlier request does."""
    model = TimedModel(delay=0.05)
    app = create_app(lambda: model, max_wait=0.01, max_sentences=1)
    long_text = " ".join(f"Long request sentence number {j}." for j in range(8))
    order = []
    with TestClient(app) as c:
        with c.websocket_connect("/v1/stream/tts") as wa, c.websocket_connect("/v1/stream/tts") as wb:
            wa.send_text(json.dumps({"type": "synthesize", "text": long_text}))
            first = wa.receive()  # A's first sentence is out: A is mid-stream
            assert first.get("bytes") is not None
            wb.send_text(json.dumps({"type": "synthesize", "text": "Short one."}))
            frames_b, final_b = recv_until_complete(wb)
            order.append("b")
            frames_a, final_a = recv_until_complete(wa)
            order.append("a")
    assert final_b == {"type": "synthesis_complete", "chunk_id": 1} and len(frames_b) == 1
    assert final_a == {"type": "synthesis_complete", "chunk_id": 8} and len(frames_a) == 7
    # B finished while A still had sentences to go: B's batch ran before A's last ones
    b_batch = next(k for k, b in enumerate(model.batches) if b == ["Short one."])
    a_last = max(k for k, b in enumerate(model.batches) if b[0].startswith("Long request sentence number 7"))
    assert b_batch < a_last


class _BatcherQueues:
    """The queue-manager surface DynamicBatcher uses, with a per-connection delivery delay."""

    def __init__(self, reqs, delay=None):
        self.reqs = list(reqs)
        self.delay = delay or {}
        self.events = []
        self.done = 0

    async def take_batch(self, room, wait):
        if self.reqs:
            out, self.reqs = self.reqs[:room], self.reqs[room:]
            return out
        await asyncio.sleep(0.005)
        return []

    async def enqueue_audio_chunk(self, conn, data, chunk_id, is_final=False):
        if conn in self.delay:
            await asyncio.sleep(self.delay[conn])
        self.events.append((conn, chunk_id, is_final, time.perf_counter()))

    async def mark_request_done(self, n):
        self.done += n


def _req(conn, text):
    from types import SimpleNamespace
    return SimpleNamespace(connection_id=conn, text=text, voice=None, stream_frames=0)


async def _run_batcher(b, q, until, timeout=10.0):
    task = asyncio.create_task(b.run())
    t0 = time.perf_counter()
    while not until() and time.perf_counter() - t0 < timeout:
        await asyncio.sleep(0.005)
    b.stop()
    task.cancel()
    await asyncio.gather(task, return_exceptions=True)


def test_short_engine_result_fails_the_batch_and_frees_its_slots():
    """an engine that returns fewer results than sentences fails the whole batch (the
    reference's failure path: no marker), and every request's slot is freed -- with max_requests = 2,
    all five requests are still admitted and finished."""
    from gonova_tts_amd.service.batcher import DynamicBatcher
    q = _BatcherQueues([_req(f"c{i}", f"Sentence {i}. And one more.") for i in range(5)])
    b = DynamicBatcher(q, lambda texts, **kw: [np.zeros(8, np.float32) for _ in texts[:-1]],
                       max_sentences=4, max_requests=2)
    asyncio.run(_run_batcher(b, q, lambda: q.done >= 5))
    assert q.done == 5
    st = b.get_stats()
    assert st["errors"] == 5 and st["syntheses"] == 0 and st["batch_errors"] >= 1
    assert not any(final for _, _, final, _ in q.events)


def test_slow_client_does_not_delay_other_connections():
    """one client's frames waiting on its full output queue (0.3 s per frame
    here) do not hold back another connection's frames served by the same engine batch -- the
    delivery lock is per request."""
    from gonova_tts_amd.service.batcher import DynamicBatcher
    q = _BatcherQueues([_req("slow", "One. Two. Three."), _req("fast", "Four. Five. Six.")], delay={"slow": 0.3})
    b = DynamicBatcher(q, lambda texts, **kw: [np.full(8, len(t), np.float32) for t in texts], max_sentences=8)
    asyncio.run(_run_batcher(b, q, lambda: q.done >= 2))
    fast_end = max(t for c, _, fin, t in q.events if c == "fast" and fin)
    slow_first = min(t for c, _, _, t in q.events if c == "slow")
    assert fast_end < slow_first, q.events
    assert [cid for c, cid, _, _ in q.events if c == "fast"] == [0, 1, 2, 3]
    assert [cid for c, cid, _, _ in q.events if c == "slow"] == [0, 1, 2, 3]
    st = b.get_stats()
    assert st["syntheses"] == 2 and st["avg_latency"] > 0.9 * st["total_latency"] / 2
