"""Probe: where C1's time goes -- the fp32 engine (vocoder and acoustic fp32, 6 frames per token)
on bench.py's 71-token sentence, generate() timed on the host over 10 calls after 3 warmups.
Run under `rocprofv3 --kernel-trace` to get the per-kernel split of one call.

usage (GPU box): python3 tools/c1_prof.py
C1_BATCH=8 / 32: the same sentence as a batch of that many through generate_batch (the fp32
service under load), with the library's device bytes (the fp32 split-K workspace).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from bench import C1_TEXT
    from gonova_tts_amd.model import GonovaTTS
    m = GonovaTTS.from_pretrained(0, vocoder_dtype="f32", acoustic_dtype="f32", fixed_duration=6)
    nb = int(os.environ.get("C1_BATCH", "0"))
    if nb:
        from gonova_tts_amd.engine import device_bytes
        texts = [C1_TEXT] * nb
        for _ in range(2):
            m.generate_batch(texts)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            out = m.generate_batch(texts)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        n = sum(len(a) for a in out)
        print(f"C1 x{nb} generate_batch(): p50 {np.percentile(ts, 50):.3f} ms, {n / np.percentile(ts, 50) / 1e3:.2f} M samples/s, "
              f"library device bytes {device_bytes(0) / 1e9:.3f} GB")
        return
    for _ in range(3):
        m.generate(C1_TEXT)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        w = m.generate(C1_TEXT)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"C1 generate(): p50 {np.percentile(ts, 50):.3f} ms, min {min(ts):.3f} ms, samples {w.numel()}")


if __name__ == "__main__":
    main()
