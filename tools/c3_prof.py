"""C3 full-pipeline step launch profile: tokens -> bf16 acoustic -> bf16 vocoder at B=32 x 144
tokens x 6 frames, a few steps; under rocprofv3 --kernel-trace, `--summarize <csv>` prints the
last step's kernel time, span and per-kernel totals (acoustic_prof.py's format).

usage (GPU box): rocprofv3 --kernel-trace --output-format csv -d <dir> -o run -- python3 tools/c3_prof.py
                 python3 tools/c3_prof.py --summarize <dir>/run_kernel_trace.csv
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
ITERS = 4


def run():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights
    B, N, dur = 32, 144, 6
    T = N * dur
    eng = HipEngine("cuda:0", vocoder_dtype="bf16", acoustic_dtype="bf16", max_batch=B, max_frames=T, max_tokens=N)
    eng.load_weights(vocoder=make_vocoder_weights(seed=0), acoustic=make_acoustic_weights(seed=0, fixed_duration=dur))
    g = torch.Generator(device="cpu").manual_seed(2000)
    tok = torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).cuda()
    tl = torch.full((B,), N, dtype=torch.int32, device="cuda")
    wav = torch.empty((B, T * 256), dtype=torch.float32, device="cuda")
    for _ in range(ITERS):
        mel, ml = eng.acoustic(tok, tl, T)
        eng.vocoder(mel, ml, out=wav)
    torch.cuda.synchronize()
    eng.close()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        import acoustic_prof
        acoustic_prof.ITERS = ITERS
        acoustic_prof.summarize(sys.argv[2])
    else:
        run()
