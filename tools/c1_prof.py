"""Probe: where C1's time goes -- the fp32 engine (vocoder and acoustic fp32, 6 frames per token)
on bench.py's 71-token sentence, generate() timed on the host over 10 calls after 3 warmups.
Run under `rocprofv3 --kernel-trace` to get the per-kernel split of one call.

usage (GPU box): python3 tools/c1_prof.py
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
