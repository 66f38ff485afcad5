"""C5 first-chunk launch profile: bench.py's streaming case (batch 8 x 144 tokens x 6 frames,
bf16, 32-frame chunks) run ITERS times to the first chunk; under rocprofv3 --kernel-trace,
`--summarize <csv>` prints the last trial's kernels in launch order and per-kernel totals.

usage (GPU box): rocprofv3 --kernel-trace --output-format csv -d <dir> -o run -- python3 tools/stream_prof.py
                 python3 tools/stream_prof.py --summarize <dir>/run_kernel_trace.csv
"""
import csv
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ITERS = 4


def run():
    import numpy as np
    import torch
    from gonova_tts_amd.model import GonovaTTS
    m = GonovaTTS.from_pretrained(0, vocoder_dtype="bf16", acoustic_dtype="bf16",
                                  encoder_precision=os.environ.get("STREAM_PROF_PRECISION", "exact"))
    rng = np.random.default_rng(5)
    B, N = 8, 144
    tok = rng.integers(1, 78, size=(B, N)).astype(np.int32)
    lens = np.full(B, N, np.int32)
    dur = np.full((B, N), 6, np.int32)
    for _ in range(ITERS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gen = m.stream_tokens(tok, lens, chunk_frames=32, durations=dur)
        _, wav, _ = next(gen)
        _ = wav.cpu()
        print(f"first chunk {1e3 * (time.perf_counter() - t0):.3f} ms")
        gen.close()
        torch.cuda.synchronize()
        time.sleep(0.05)  # a gap that separates the trials in the trace
    m.engine.close()


def summarize(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # the last trial: the launches after the last gap of > 20 ms
    start = 0
    for i in range(1, len(rows)):
        if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 20_000_000:
            start = i
    last = rows[start:]
    t0 = int(last[0]["Start_Timestamp"])
    tot = defaultdict(lambda: [0.0, 0])
    for r in last:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[r["Kernel_Name"][:60]][0] += us
        tot[r["Kernel_Name"][:60]][1] += 1
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {us:8.1f} us q{r.get('Queue_Id', '?')}  {r['Kernel_Name'][:80]}")
    span = (int(last[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"last trial: {len(last)} launches, kernel time {sum(v[0] for v in tot.values()):.1f} us, span {span:.1f} us")
    for k, (us, c) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print(f"{us:9.1f} us {c:4d}x  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
