"""Experiment: C2 step as NSTREAMS (env, default 2) sub-batches on as many HIP streams (two engines, own workspaces)
against one batch-32 call on one stream.  Prints ms per step for each layout.

usage (GPU box): python3 tools/two_stream_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_vocoder_weights
    B, T = 32, 862
    w = make_vocoder_weights(seed=0)
    mel = torch.randn(B, T, 80, device="cuda")
    one = HipEngine(0, vocoder_dtype="f16", max_batch=B, max_frames=T)
    one.load_weights(vocoder=w)
    NS = int(os.environ.get("NSTREAMS", "2"))
    halves = []
    for _ in range(NS):
        e = HipEngine(0, vocoder_dtype="f16", max_batch=B // NS, max_frames=T)
        e.load_weights(vocoder=w)
        halves.append(e)
    out = torch.empty(B, T * 256, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(NS)]
    main_s = torch.cuda.current_stream()

    def step_one():
        one.vocoder(mel, out=out)

    def step_two(offset_stage=False):
        ev = torch.cuda.Event()
        ev.record(main_s)
        for i, (e, s) in enumerate(zip(halves, streams)):
            s.wait_event(ev)
            n = B // NS
            e.vocoder(mel[n * i:n * (i + 1)], out=out[n * i:n * (i + 1)], stream=s)
        for s in streams:
            main_s.wait_stream(s)

    for name, fn in [("one stream, B=32", step_one), (f"{NS} streams, B={B} split", step_two),
                     ("one stream, B=32", step_one), (f"{NS} streams, B={B} split", step_two)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        print(f"{name:24s} {(time.perf_counter() - t0) * 100:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
