"""C5 as bench.py measures it (batch 8 x 144 tokens, predicted durations, bf16, first 32-frame
chunk on the host), 20 trials, then a 100 ms pause and one traced trial: run under
`rocprofv3 --kernel-trace` and read the last trial with tools/last_burst.py.

usage (GPU box): rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/c5_trace.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(trials=20, B=8, N=144, chunk=32):
    import torch
    from gonova_tts_amd.model import GonovaTTS
    m = GonovaTTS.from_pretrained(0, vocoder_dtype="bf16", acoustic_dtype="bf16", fixed_duration=6)
    rng = np.random.default_rng(5)
    tok = rng.integers(1, 78, size=(B, N)).astype(np.int32)
    lens = np.full(B, N, np.int32)
    lat = []

    def trial():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gen = m.stream_tokens(tok, lens, chunk_frames=chunk)
        _, wav, valid = next(gen)
        _ = wav.cpu()
        t = time.perf_counter() - t0
        gen.close()
        return t * 1e3

    for i in range(trials + 5):
        t = trial()
        if i >= 5:
            lat.append(t)
    time.sleep(0.1)
    last = trial()
    print(f"C5 first audio p50 {np.percentile(lat, 50):.3f} ms over {trials}; traced trial {last:.3f} ms")
    m.engine.close()


if __name__ == "__main__":
    main()
