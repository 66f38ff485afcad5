"""Probe: C2 (batch-32 x 862-frame mel -> HiFi-GAN, fp16) as one engine on one stream (the bench
line) against the batch split over k engines on k streams, all parts started together every
step (each launch's tail -- its last, partly filled wave of blocks -- then overlaps the other
streams' launches).  Prints ms per 32-utterance step, 10 timed steps after 3 warmups,
two alternating rounds, and checks the split outputs equal the one-stream output bit for bit.

usage (GPU box): python3 tools/c2_overlap_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_vocoder_weights
    B, T = 32, 862
    vw = make_vocoder_weights(seed=0)
    g = torch.Generator(device="cpu").manual_seed(1000)
    mel = torch.randn((B, T, 80), generator=g).cuda()
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    wav = torch.empty((B, T * 256), dtype=torch.float32, device="cuda")
    ref = torch.empty_like(wav)
    steps = int(os.environ.get("PROBE_STEPS", "10"))

    def timed(fn, warm=3):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / steps

    engines = [HipEngine("cuda:0", vocoder_dtype="f16", max_batch=B, max_frames=T)]
    engines[0].load_weights(vocoder=vw)
    for _ in range(3):
        e = HipEngine("cuda:0", vocoder_dtype="f16", max_batch=B // 2, max_frames=T)
        e.load_weights(vocoder=vw)
        engines.append(e)
    streams = [torch.cuda.Stream() for _ in range(4)]

    def one():
        engines[0].vocoder(mel, lens, out=wav)

    def split(k):
        n = B // k

        def fn():
            cur = torch.cuda.current_stream()
            for i in range(k):
                streams[i].wait_stream(cur)
            for i in range(k):
                sl = slice(i * n, (i + 1) * n)
                with torch.cuda.stream(streams[i]):
                    engines[i].vocoder(mel[sl], lens[sl], out=wav[sl], stream=streams[i])
            for i in range(k):
                cur.wait_stream(streams[i])
        return fn

    def free2():
        # the two halves' streams run free: no join between steps (a serving loop's shape); the
        # timing's synchronize at the end waits for both
        n = B // 2
        for i in range(2):
            sl = slice(i * n, (i + 1) * n)
            with torch.cuda.stream(streams[i]):
                engines[i].vocoder(mel[sl], lens[sl], out=wav[sl], stream=streams[i])

    one()
    torch.cuda.synchronize()
    ref.copy_(wav)
    for k in (2, 4):
        wav.zero_()
        split(k)()
        torch.cuda.synchronize()
        print(f"split {k}: bit-identical to one stream: {bool(torch.equal(wav, ref))}")
    for rnd in range(2):
        print(f"round {rnd}: one {timed(one):.3f} ms, two {timed(split(2)):.3f} ms, four {timed(split(4)):.3f} ms, "
              f"two free-running {timed(free2):.3f} ms", flush=True)
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
