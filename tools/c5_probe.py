"""C5 (streaming, batch 8) latency split: host wall time vs device time of the acoustic pass
and of the first vocoder chunk, to see whether first-audio latency is launch-bound.

usage (GPU box): python3 tools/c5_probe.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(trials=30, B=8, N=144, chunk=32, ctx=16):
    import torch
    from gonova_tts_amd.model import GonovaTTS
    m = GonovaTTS.from_pretrained(0, vocoder_dtype="bf16", acoustic_dtype="bf16")
    eng = m.engine
    rng = np.random.default_rng(5)
    tok = torch.from_numpy(rng.integers(1, 78, size=(B, N)).astype(np.int32)).cuda()
    tl = torch.full((B,), N, dtype=torch.int32, device="cuda")
    dur = torch.full((B, N), 6, dtype=torch.int32, device="cuda")
    rows = {"acoustic_wall": [], "acoustic_dev": [], "voc_wall": [], "voc_dev": [], "launch_ac": []}
    for i in range(trials + 5):
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0 = time.perf_counter()
        e0.record()
        mel, mel_lens, _ = eng.acoustic(tok, tl, N * 6, durations=dur, return_durations=True)
        t_launch = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        win = mel[:, 0:chunk + ctx].contiguous()
        wl = torch.clamp(mel_lens, min=0, max=chunk + ctx).to(torch.int32)
        wav = eng.vocoder_chunk(win, wl, 0, chunk)
        e2.record()
        _ = wav.cpu()
        t2 = time.perf_counter()
        if i >= 5:
            rows["acoustic_wall"].append((t1 - t0) * 1e3)
            rows["launch_ac"].append((t_launch - t0) * 1e3)
            rows["acoustic_dev"].append(e0.elapsed_time(e1))
            rows["voc_wall"].append((t2 - t1) * 1e3)
            rows["voc_dev"].append(e1.elapsed_time(e2))
    for k, v in rows.items():
        print(f"{k:14s} p50 {np.percentile(v, 50):7.3f} ms")
    eng.close()


if __name__ == "__main__":
    main()
