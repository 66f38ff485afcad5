"""Probe: the C2 vocoder step eager vs replayed from a HIP graph (torch.cuda.CUDAGraph over the
engine's launches on the capturing stream).  Prints ms per step for both and checks that the
replayed output equals the eager one bit for bit.

usage (GPU box): python3 tools/graph_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def acoustic():
    """The C5 acoustic pass (batch 8 x 144 tokens, 6 frames each, bf16, exact encoder)."""
    import numpy as np
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_acoustic_weights
    B, N = int(os.environ.get("GRAPH_PROBE_B", "8")), 144
    eng = HipEngine("cuda:0", acoustic_dtype="bf16", max_batch=B, max_frames=N * 6, max_tokens=N)
    eng.load_weights(acoustic=make_acoustic_weights(seed=0))
    rng = np.random.default_rng(5)
    tok = torch.from_numpy(rng.integers(1, 78, size=(B, N)).astype(np.int32)).cuda()
    tl = torch.full((B,), N, dtype=torch.int32, device="cuda")
    dd = torch.full((B, N), 6, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    res = {}

    def step():
        res["mel"], res["lens"] = eng.acoustic(tok, tl, N * 6, durations=dd, stream=s)

    def timed(fn, n=20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    with torch.cuda.stream(s):
        for _ in range(3):
            step()
        eager_ms = timed(step)
        ref = res["mel"].clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    with torch.cuda.stream(s):
        for _ in range(3):
            g.replay()
        graph_ms = timed(g.replay)
    s.synchronize()
    print(f"acoustic B={B}: eager {eager_ms:.3f} ms, graph {graph_ms:.3f} ms; "
          f"graph output identical: {bool(torch.equal(res['mel'], ref))}")


def main():
    if os.environ.get("GRAPH_PROBE_WHAT") == "acoustic":
        return acoustic()
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_vocoder_weights
    B, T = 32, 862
    eng = HipEngine("cuda:0", vocoder_dtype=os.environ.get("GRAPH_PROBE_DTYPE", "f16"))
    eng.load_weights(vocoder=make_vocoder_weights(seed=0))
    g0 = torch.Generator(device="cpu").manual_seed(0)
    mel = torch.randn(B, T, 80, generator=g0).cuda()
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    out = torch.empty(B, T * 256, device="cuda")
    s = torch.cuda.Stream()

    def timed(fn, n=10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    with torch.cuda.stream(s):
        for _ in range(3):
            eng.vocoder(mel, lens, out=out, stream=s)
        eager_ms = timed(lambda: eng.vocoder(mel, lens, out=out, stream=s))
        ref = out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        eng.vocoder(mel, lens, out=out, stream=s)
    with torch.cuda.stream(s):
        out.zero_()
        for _ in range(3):
            g.replay()
        graph_ms = timed(g.replay)
        eager2_ms = timed(lambda: eng.vocoder(mel, lens, out=out, stream=s))
        g.replay()
    s.synchronize()
    same = bool(torch.equal(out, ref))
    print(f"eager {eager_ms:.3f} ms/step, graph {graph_ms:.3f} ms/step, eager again {eager2_ms:.3f}; "
          f"graph output identical: {same}")


if __name__ == "__main__":
    main()
