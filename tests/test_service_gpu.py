"""The WebSocket service with the real HIP engine (not a fake): the reference's request /
response contract (`services/tts/server.py:143-164, 215-224, 268-298`) end to end on the GPU.

Config C1 through the service: fp32 engine, one client and two concurrent clients; every
binary frame is raw float32 PCM of one sentence (split as the reference splits,
`core/synthesizer.py:48-99`) and must equal the model's own `generate(sentence)` and the CPU
oracle pipeline (fp32 tolerance: atol 2e-5 / rtol 1e-4 against the oracle, 1e-5 / 1e-4 against
generate())."""
import json
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytest.importorskip("fastapi")
pytestmark = pytest.mark.gpu

from fastapi.testclient import TestClient  # noqa: E402

from gonova_tts_amd.model import GonovaTTS  # noqa: E402
from gonova_tts_amd.service.server import create_app  # noqa: E402
from gonova_tts_amd.text import split_into_sentences, tokenize  # noqa: E402
from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights  # noqa: E402
from oracle.acoustic import acoustic_forward  # noqa: E402
from oracle.vocoder import vocoder_forward  # noqa: E402

TEXT = "Hello world. This is a test! Is it working? yes it is."


def recv_until_complete(ws):
    frames = []
    while True:
        m = ws.receive()
        if m.get("bytes") is not None:
            frames.append(np.frombuffer(m["bytes"], np.float32))
        elif m.get("text") is not None:
            return frames, json.loads(m["text"])


def oracle_wav(sentence, aw, vw):
    o = acoustic_forward(tokenize(sentence), aw)
    return vocoder_forward(o["mel"], vw)


@pytest.fixture(scope="module")
def served():
    holder = {}

    def factory():
        holder["m"] = GonovaTTS.from_pretrained("cuda:0", vocoder_dtype="f32", acoustic_dtype="f32")
        return holder["m"]

    app = create_app(factory, max_wait=0.25, idle_wait=0.25)  # (the batching tests gather while idle too)
    with TestClient(app) as c:
        yield c, holder["m"]


def test_service_frames_equal_generate_and_oracle(served):
    c, model = served
    with c.websocket_connect("/v1/stream/tts") as ws:
        ws.send_text(json.dumps({"type": "synthesize", "text": TEXT, "voice_id": "default", "exaggeration": 0.5}))
        frames, final = recv_until_complete(ws)
    sents = split_into_sentences(TEXT)
    assert sents == ["Hello world.", "This is a test!", "Is it working? yes it is."]
    assert final == {"type": "synthesis_complete", "chunk_id": 3}
    assert len(frames) == 3
    aw, vw = make_acoustic_weights(0), make_vocoder_weights(0)
    for f, s in zip(frames, sents):
        direct = model.generate(s).squeeze().cpu().numpy()
        assert f.shape == direct.shape
        np.testing.assert_allclose(f, direct, atol=1e-5, rtol=1e-4)
        ref = oracle_wav(s, aw, vw)
        assert f.shape == ref.shape
        err = float(np.abs(f - ref).max())
        print(f"service frame {s!r}: {f.size} samples, max|err| vs oracle {err:.2e}")
        np.testing.assert_allclose(f, ref, atol=2e-5, rtol=1e-4)
    m = c.get("/metrics").json()
    assert m["chunks_sent"] >= 4 and m["requests_dropped"] == 0
    h = c.get("/health").json()
    assert h["status"] == "healthy" and h["sample_rate"] == 22050


def test_two_concurrent_connections_share_engine_batches(served):
    c, model = served
    texts = {0: "Good morning. The quick brown fox jumps.", 1: "A second client speaks. Then it stops!"}
    results = {}
    before = dict(c.app.state.service.batcher.stats)

    def client(i):
        with c.websocket_connect("/v1/stream/tts") as ws:
            ws.send_text(json.dumps({"type": "synthesize", "text": texts[i]}))
            results[i] = recv_until_complete(ws)

    ts = [threading.Thread(target=client, args=(i,)) for i in texts]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert len(results) == 2
    after = c.app.state.service.batcher.stats
    # both requests were taken in one batcher round and their 4 sentences ran as one engine pass
    assert after["rounds"] - before["rounds"] == 1
    assert after["engine_batches"] - before["engine_batches"] == 1
    for i, (frames, final) in results.items():
        sents = split_into_sentences(texts[i])
        assert final == {"type": "synthesis_complete", "chunk_id": len(sents)}
        for f, s in zip(frames, sents):
            np.testing.assert_allclose(f, model.generate(s).squeeze().cpu().numpy(), atol=1e-5, rtol=1e-4)
    assert after["sentences"] - before["sentences"] == 4


def test_stream_frames_concatenate_to_generate(served):
    """Opt-in sub-sentence frames through the service on the real engine:
    "stream_frames": 8 is below the service's floor (MIN_STREAM_FRAMES = 32) and rounds up to it:
    every frame is at most 32 x 256 samples, each sentence comes as ceil(samples / 8192) frames
    in order, and the frames concatenate to generate() of each sentence (fp32 engine, the same
    tolerance as the per-sentence test)."""
    c, model = served
    text = "Good morning to everyone in the room. The quick brown fox jumps over the lazy dog!"
    with c.websocket_connect("/v1/stream/tts") as ws:
        ws.send_text(json.dumps({"type": "synthesize", "text": text, "stream_frames": 8}))
        frames, final = recv_until_complete(ws)
    direct = [model.generate(s).squeeze().cpu().numpy() for s in split_into_sentences(text)]
    assert final == {"type": "synthesis_complete", "chunk_id": len(frames)}
    assert all(0 < len(f) <= 32 * 256 for f in frames)
    assert len(frames) == sum(-(-len(d) // 8192) for d in direct)
    got, want = np.concatenate(frames), np.concatenate(direct)
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, atol=1e-5, rtol=1e-4)


def test_two_engines_continuous_batcher_real_engine():
    """TTSService(devices=["cuda:0", "cuda:0"]): two real GonovaTTS engines (their own workspaces
    and executor threads) pull engine batches from the continuous batcher's shared work list at the
    same time.  Three concurrent clients -- one of them streamed (stream_frames,
    dealt across the engines like the others) -- get every frame in sentence order, equal to
    generate() of each sentence (fp32 engines, the per-sentence tolerance), and both engines ran
    batches."""
    made = []

    def factory(device):
        made.append(GonovaTTS.from_pretrained(device, vocoder_dtype="f32", acoustic_dtype="f32"))
        return made[-1]

    app = create_app(factory, devices=["cuda:0", "cuda:0"], max_wait=0.2, idle_wait=0.2, max_sentences=2)
    texts = {0: "Good morning. The quick brown fox jumps. Over the lazy dog!",
             1: "A second client speaks. Then it stops! And starts again.",
             2: "Streaming here. In small pieces please."}
    results = {}
    with TestClient(app) as c:
        def client(i):
            msg = {"type": "synthesize", "text": texts[i]}
            if i == 2:
                msg["stream_frames"] = 32
            with c.websocket_connect("/v1/stream/tts") as ws:
                ws.send_text(json.dumps(msg))
                results[i] = recv_until_complete(ws)
        ts = [threading.Thread(target=client, args=(i,)) for i in texts]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=180)
        stats = dict(app.state.service.batcher.stats)
        # (the service closes its engines at shutdown: the reference runs inside the client block)
        direct_all = {i: [made[0].generate(s).squeeze().cpu().numpy() for s in split_into_sentences(texts[i])]
                      for i in texts}
    assert len(results) == 3
    for i, (frames, final) in results.items():
        direct = direct_all[i]
        assert final == {"type": "synthesis_complete", "chunk_id": len(frames)}
        if i == 2:
            assert len(frames) == sum(-(-len(d) // 8192) for d in direct)
            got, want = np.concatenate(frames), np.concatenate(direct)
        else:
            assert len(frames) == len(direct)
            got, want = frames, direct
        for g, w in zip(got if i != 2 else [got], want if i != 2 else [want]):
            assert g.shape == w.shape
            np.testing.assert_allclose(g, w, atol=1e-5, rtol=1e-4)
    assert min(stats["engine_sentences"]) > 0, stats["engine_sentences"]
