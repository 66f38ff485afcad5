"""The fake model output and the client messages of the WebSocket transcript fixture
(tests/golden/make_ws_golden.py records the reference service with them; tests/test_service_cpu.py
drives this build's service with the same ones).  Our own data-generating code, no reference code."""
import zlib

import numpy as np

# client messages (reference server.py:215-224 fields); texts chosen to exercise the reference's
# sentence split (synthesizer.py:48-99): punctuation + capital, abbreviations, a lower-case
# continuation, comma re-chunking of a sentence over 150 characters
REQUESTS = [
    {"type": "synthesize", "text": "Hello world. This is a test! Is it working? yes it is.",
     "voice_id": "default", "exaggeration": 0.5},
    {"type": "synthesize", "text": "Dr. Smith went to Washington. He arrived at 3.14 p.m. Then he left."},
    {"type": "synthesize", "text": "Alpha beta gamma delta, " + "epsilon zeta eta theta iota kappa, " * 4 +
     "lambda mu nu xi omicron pi rho sigma tau upsilon phi chi psi omega. Done.", "voice_id": "nobody",
     "chunk_size": 20, "streaming": True},
]


def fake_audio(text: str) -> np.ndarray:
    """Deterministic float32 'waveform' for a sentence: 37 samples per character, values from
    the text's crc32 (so every sentence's frame has its own bytes)."""
    n = 37 * len(text)
    seed = zlib.crc32(text.encode())
    i = np.arange(n, dtype=np.int64)
    v = ((i * 2654435761 + seed) % 65521).astype(np.float64) / 65521.0 - 0.5
    return (0.25 * v).astype(np.float32)
