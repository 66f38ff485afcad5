"""Device time of the batch-8 acoustic pass (C5's first stage) by padded frame extent t_cap:
predicted durations at t_cap = 6 N (what the frames need) vs 12 N (model.FRAMES_PER_TOKEN_CAP,
the streaming path's first-pass budget), and given durations at 6 N.

usage (GPU box): python3 tools/tcap_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(trials=40, B=8, N=144):
    import torch
    from gonova_tts_amd.model import GonovaTTS
    m = GonovaTTS.from_pretrained(0, vocoder_dtype="bf16", acoustic_dtype="bf16")
    eng = m.engine
    rng = np.random.default_rng(5)
    tok = torch.from_numpy(rng.integers(1, 78, size=(B, N)).astype(np.int32)).cuda()
    tl = torch.full((B,), N, dtype=torch.int32, device="cuda")
    dur = torch.full((B, N), 6, dtype=torch.int32, device="cuda")
    cases = {"pred_6N": (6 * N, None), "pred_12N": (12 * N, None), "given_6N": (6 * N, dur)}
    times = {k: [] for k in cases}
    for i in range(trials + 5):
        for k, (tc, d) in cases.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.acoustic(tok, tl, tc, durations=d, return_durations=True)
            e1.record()
            torch.cuda.synchronize()
            if i >= 5:
                times[k].append(e0.elapsed_time(e1) * 1e3)
    for k, v in times.items():
        print(f"{k:9s} t_cap={cases[k][0]:5d}: median {np.median(v):8.1f} us  (p10 {np.percentile(v, 10):8.1f}, p90 {np.percentile(v, 90):8.1f})")


if __name__ == "__main__":
    main()
