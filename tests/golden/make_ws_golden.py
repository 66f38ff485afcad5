"""Record the reference service's WebSocket transcript, /metrics and /health (build container
only: it imports /root/reference, which the GPU box does not have; never shipped or imported by
the product).

    python tests/golden/make_ws_golden.py      -> tests/golden/ws_transcript.json

The reference server (`/root/reference/services/tts/server.py`) is imported as SURVEY.md §4
describes: `torchaudio`, `structlog` and `soundfile` are absent here and get inert stub
modules, the un-vendored `chatterbox.tts.ChatterboxTTS` is a fake that records every
`generate` call's arguments and returns `fake_audio(text)` (a deterministic float32 array whose
length and values depend on the text; tests/test_service_cpu.py uses the same function), and
`signal.signal` is a no-op (TestClient runs the startup hook off the main thread).  The fixture
holds what the reference did with those arrays: the frames each request produced (byte length
and sha256 of each binary frame, in order), the final JSON message, every `generate` call
(text and keyword arguments, warmups included), /metrics after the requests, /health's
503 body before startup (server.py:447-454), and the shape of its 200 body after the requests
(server.py:456-475): the key set of every nested dict, and the synthesizer's request counts.
"""
from __future__ import annotations

import hashlib
import json
import os
import signal
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/services/tts"
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden.ws_fake import REQUESTS, fake_audio  # noqa: E402


def stub_modules(calls):
    import torch

    ta = types.ModuleType("torchaudio")
    sys.modules["torchaudio"] = ta
    sf = types.ModuleType("soundfile")
    sf.read = sf.write = lambda *a, **k: (_ for _ in ()).throw(RuntimeError("soundfile stub"))
    sys.modules["soundfile"] = sf

    class _Log:
        def __getattr__(self, name):
            return lambda *a, **k: None

    sl = types.ModuleType("structlog")
    sl.configure = lambda **k: None
    sl.get_logger = lambda *a, **k: _Log()
    sl.processors = types.SimpleNamespace(TimeStamper=lambda **k: None, add_log_level=None,
                                          JSONRenderer=lambda **k: None)
    sys.modules["structlog"] = sl

    class FakeChatterbox:
        sr = 24000

        @classmethod
        def from_pretrained(cls, device=None, **kw):
            calls.append({"call": "from_pretrained", "device": device})
            return cls()

        def generate(self, text, **kw):
            calls.append({"call": "generate", "text": text, "kwargs": {k: kw[k] for k in sorted(kw)}})
            return torch.from_numpy(fake_audio(text))[None]

    cb = types.ModuleType("chatterbox")
    cbt = types.ModuleType("chatterbox.tts")
    cbt.ChatterboxTTS = FakeChatterbox
    cb.tts = cbt
    sys.modules["chatterbox"] = cb
    sys.modules["chatterbox.tts"] = cbt


def main():
    from fastapi.testclient import TestClient

    calls = []
    stub_modules(calls)
    signal.signal = lambda *a, **k: None
    sys.path.insert(0, REF)
    import server  # the reference's services/tts/server.py

    out = {"source": "services/tts/server.py (reference) under TestClient; see make_ws_golden.py",
           "requests": []}
    r = TestClient(server.app).get("/health")  # no startup yet: the model is not loaded
    out["health_before_load"] = {"status_code": r.status_code, "body": r.json()}
    with TestClient(server.app) as c:
        with c.websocket_connect("/v1/stream/tts") as ws:
            for req in REQUESTS:
                ws.send_text(json.dumps(req))
                frames = []
                while True:
                    m = ws.receive()
                    if m.get("bytes") is not None:
                        b = m["bytes"]
                        frames.append({"bytes": len(b), "sha256": hashlib.sha256(b).hexdigest()})
                    elif m.get("text") is not None:
                        final = json.loads(m["text"])
                        break
                out["requests"].append({"message": req, "frames": frames, "final": final})
        metrics = c.get("/metrics").json()
        health = c.get("/health")
    out["metrics"] = metrics
    hb = health.json()
    out["health_after_requests"] = {
        "status_code": health.status_code,
        "keys": sorted(hb),
        "nested_keys": {k: sorted(v) for k, v in hb.items() if isinstance(v, dict)},
        "synthesizer_counts": {k: hb["synthesizer_stats"][k] for k in ("syntheses", "errors")},
    }
    out["generate_calls"] = [x for x in calls if x["call"] == "generate"]
    out["from_pretrained"] = [x for x in calls if x["call"] == "from_pretrained"]
    path = os.path.join(HERE, "ws_transcript.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {path}: {len(out['requests'])} requests, "
          f"{sum(len(q['frames']) for q in out['requests'])} frames, {len(out['generate_calls'])} generate calls")


if __name__ == "__main__":
    main()
