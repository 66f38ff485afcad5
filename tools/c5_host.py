"""C5 host-side split (tools/c5_trace.py's workload): per trial, the host time spent in each step of
stream_tokens' first chunk -- the token upload, the acoustic call (its enqueue, including the
decoder-extent read inside it), the first chunk's enqueue, the frame-count wait and the chunk's
copy to the host -- p50 over 30 trials, with the device time of the acoustic pass and the chunk.

usage (GPU box): python3 tools/c5_host.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(trials=30, B=8, N=144, chunk=32, ctx=16):
    import torch
    from gonova_tts_amd import model as M
    m = M.GonovaTTS.from_pretrained(0, vocoder_dtype="bf16", acoustic_dtype="bf16", fixed_duration=6)
    eng = m.engine
    rng = np.random.default_rng(5)
    tok = rng.integers(1, 78, size=(B, N)).astype(np.int32)
    lens = np.full(B, N, np.int32)
    rows = {k: [] for k in ("upload", "acoustic_call", "chunk_call", "read_wait", "to_host", "total",
                            "dev_acoustic", "dev_chunk")}
    for i in range(trials + 5):
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0 = time.perf_counter()
        dev = eng.torch_device
        tk, tl, _ = M._upload_i32((tok, lens, None), dev)
        t1 = time.perf_counter()
        e0.record()
        mel, mel_lens, dur, rw = eng.acoustic(tk, tl, 12 * N, return_durations=True, return_range=True)
        e1.record()
        t2 = time.perf_counter()
        rd = M._HostRead(dur, mel_lens, rw)
        w1 = chunk + ctx
        win_lens = torch.clamp(mel_lens, min=0, max=w1).to(torch.int32)
        wav = eng.vocoder_chunk(mel[:, :w1].contiguous(), win_lens, 0, chunk)
        e2.record()
        t3 = time.perf_counter()
        rd.result()
        t4 = time.perf_counter()
        _ = wav.cpu()
        t5 = time.perf_counter()
        if i >= 5:
            for k, v in (("upload", t1 - t0), ("acoustic_call", t2 - t1), ("chunk_call", t3 - t2),
                         ("read_wait", t4 - t3), ("to_host", t5 - t4), ("total", t5 - t0)):
                rows[k].append(v * 1e3)
            rows["dev_acoustic"].append(e0.elapsed_time(e1))
            rows["dev_chunk"].append(e1.elapsed_time(e2))
    for k, v in rows.items():
        print(f"{k:14s} p50 {np.percentile(v, 50):7.3f} ms")
    eng.close()


if __name__ == "__main__":
    main()
