"""Barrier timeline of the warp-specialised k = 3 pair kernel (mrf_pair_ws.hip) in the C2 vocoder
step (diagnostic build only).

Build:  python -m gonova_tts_amd.build --variant wstamp -DTTS_PWS_STAMP=1
Run:    TTS_PAIR_WS=1 TTS_LIB=<repo>/gonova-tts_amd/libtts_hip_wstamp.so python3 tools/pws_stamps.py C d [C d ...]

Per block and tile the library records when compute wave 0 and the first loader wave arrive at each of
the four barriers A (G ready / output tile written), B (conv1 done / row pass done), C (T written /
DMA issued), D (conv2 done / G activated).  A barrier opens when the later role arrives, so for
each barrier this prints how long each role waited for the other, and each role's work per
segment -- the segment a role fills to the brim is the one that sets the tile time.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BARRIERS = ("A", "B", "C", "D")
SEGS = ("A->B (conv1 | row pass)", "B->C (T write | DMA issue)", "C->D (conv2 | DMA wait+activate)",
        "D->A (out write | -)")


def run(targets):
    import torch
    from gonova_tts_amd.engine import HipEngine, load_library
    from gonova_tts_amd.weights import make_vocoder_weights
    lib = load_library()
    lib.tts_debug_pws_target.argtypes = [ctypes.c_int] * 2
    lib.tts_debug_pws_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    g = torch.Generator(device="cpu").manual_seed(3)
    eng = HipEngine("cuda:0", vocoder_dtype="f16", max_batch=32, max_frames=862)
    eng.load_weights(vocoder=make_vocoder_weights(seed=0))
    mel = torch.randn((32, 862, 80), generator=g).cuda()
    wav = torch.empty((32, 862 * 256), device="cuda")
    out = {}
    for t in targets:
        assert lib.tts_debug_pws_target(*t) == 0
        for _ in range(3):
            eng.vocoder(mel, out=wav)
        torch.cuda.synchronize()
        buf = np.zeros(1 << 20, np.uint64)
        assert lib.tts_debug_pws_stamps(buf.ctypes.data, buf.size) == 0
        rec = buf.reshape(-1, 256)
        out[t] = rec[rec[:, 1] != 0].copy()
    eng.close()
    return out


def analyze(rec, t):
    n = len(rec)
    tiles = rec[:, 0].astype(np.int64)
    print(f"C={t[0]} d={t[1]}: {n} blocks, tiles per block median {np.median(tiles):.0f} (max {tiles.max()})")
    if n == 0:
        return
    waits = {b: [[], []] for b in BARRIERS}
    work = [[[], []] for _ in SEGS]
    tile_t = []
    for r, kt in zip(rec, tiles):
        kt = min(int(kt), 30)
        st = r[2:2 + 8 * (kt + 1)].astype(np.float64).reshape(-1, 2, 4)  # [tile][role][barrier]
        for k in range(kt):
            opens = []
            for j, b in enumerate(BARRIERS):
                c, l = st[k, 0, j], st[k, 1, j]
                if c == 0 or l == 0:
                    opens.append(None)
                    continue
                o = max(c, l)
                opens.append(o)
                waits[b][0].append(o - c)
                waits[b][1].append(o - l)
            nxt = st[k + 1, :, 0] if k + 1 <= kt else None
            for j in range(4):
                if opens[j] is None:
                    continue
                end = st[k, :, j + 1] if j < 3 else nxt
                if end is None or end[0] == 0 or end[1] == 0:
                    continue
                work[j][0].append(end[0] - opens[j])
                work[j][1].append(end[1] - opens[j])
            if opens[0] is not None and k + 1 <= kt and st[k + 1, 0, 0] and st[k + 1, 1, 0]:
                tile_t.append(max(st[k + 1, 0, 0], st[k + 1, 1, 0]) - opens[0])
    print(f"  tile time (cycles, barrier A to A): median {np.median(tile_t):.0f}, p90 {np.percentile(tile_t, 90):.0f}")
    print("  barrier   compute waits   loader waits   (median cycles)")
    for b in BARRIERS:
        c, l = waits[b]
        if c:
            print(f"  {b}         {np.median(c):12.0f}   {np.median(l):12.0f}")
    print("  segment                               compute work   loader work")
    for j, name in enumerate(SEGS):
        c, l = work[j]
        if c:
            print(f"  {name:36s} {np.median(c):12.0f}   {np.median(l):12.0f}")


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    targets = [tuple(a[i:i + 2]) for i in range(0, len(a), 2)] or [(128, 1), (256, 1)]
    for t, rec in run(targets).items():
        analyze(rec, t)
