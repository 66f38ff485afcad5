"""Where the host waits in a C4 step: cProfile of ShardedSynthesis.run (bench.py's C4 workload, one
rank), top entries by own time -- a call that blocks on the device shows up with the GPU time of
the work before it.

usage (GPU box): python3 tools/c4_host_probe.py
"""
import cProfile
import os
import pstats
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gonova_tts_amd.dist import ShardedSynthesis
    from gonova_tts_amd.model import GonovaTTS
    B = 256
    m = GonovaTTS.from_pretrained(0, vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=64, max_frames=864,
                                  max_tokens=144)
    rng = np.random.default_rng(7)
    lens = rng.integers(29, 145, size=B).astype(np.int32)
    tok = np.zeros((B, 144), np.int32)
    for i, L in enumerate(lens):
        tok[i, :L] = rng.integers(1, 78, size=L)

    def synth(t, l):
        d = np.where(np.arange(t.shape[1])[None, :] < l[:, None], 6, 0).astype(np.int32)
        return m.synthesize_tokens(t, l, durations=d, host_lens=False)

    sh = ShardedSynthesis(synth, torch.device("cuda:0"), bucket=64)
    for _ in range(3):
        sh.run(tok, lens)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        sh.run(tok, lens)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
