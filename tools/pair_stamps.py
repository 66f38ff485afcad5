"""Per-block phase timeline of one mrf_pair launch in the C2 vocoder step (diagnostic build only).

Build:  python -m gonova_tts_amd.build --variant pstamp -DTTS_PAIR_STAMP=1
Run:    TTS_LIB=<repo>/gonova-tts_amd/libtts_hip_pstamp.so python3 tools/pair_stamps.py C k d [C k d ...]

For each (C, k, d) the library records, per block of that pair launch, s_memtime at entry, input
tile staged, conv1 done, T written, conv2 done, output tile staged and row pass issued, plus
s_memrealtime at entry and end.  Prints the per-phase split of block time and the chip-wide mix of
phases over the launch: how many blocks are in an MFMA phase (conv1 / conv2) versus a memory
phase (staging, row pass) at each moment -- lockstep phases show up as alternating bands.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ("staging", "conv1", "T write", "conv2", "out stage", "row pass")


def run(targets):
    import torch
    from gonova_tts_amd.engine import HipEngine, load_library
    from gonova_tts_amd.weights import make_vocoder_weights
    lib = load_library()
    lib.tts_debug_pair_target.argtypes = [ctypes.c_int] * 3
    lib.tts_debug_pair_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    g = torch.Generator(device="cpu").manual_seed(3)
    eng = HipEngine("cuda:0", vocoder_dtype="f16", max_batch=32, max_frames=862)
    eng.load_weights(vocoder=make_vocoder_weights(seed=0))
    mel = torch.randn((32, 862, 80), generator=g).cuda()
    wav = torch.empty((32, 862 * 256), device="cuda")
    out = {}
    for t in targets:
        assert lib.tts_debug_pair_target(*t) == 0
        for _ in range(3):
            eng.vocoder(mel, out=wav)
        torch.cuda.synchronize()
        buf = np.zeros(1 << 21, np.uint64)
        assert lib.tts_debug_pair_stamps(buf.ctypes.data, buf.size) == 0
        rec = buf.reshape(-1, 16)
        out[t] = rec[rec[:, 0] != 0].copy()
    eng.close()
    return out


def analyze(rec, t):
    if len(rec) == 0:  # e.g. a launch with conv_post fused, which returns before stamping
        print(f"C={t[0]} k={t[1]} d={t[2]}: no records")
        return
    st = rec[:, :7].astype(np.float64)
    rt0, rt1 = rec[:, 7].astype(np.float64), rec[:, 8].astype(np.float64)
    n = len(rec)
    d = np.diff(st, axis=1)  # 6 phases
    tot = st[:, 6] - st[:, 0]
    clk = tot.sum() / ((rt1 - rt0).sum() / 100e6)
    span_us = (rt1.max() - rt0.min()) / 100.0
    print(f"C={t[0]} k={t[1]} d={t[2]}: {n} blocks, launch span {span_us:.1f} us, shader clock ~{clk / 1e9:.2f} GHz")
    print(f"  block time (cycles) median {np.median(tot):.0f}, p90 {np.percentile(tot, 90):.0f}")
    for i, name in enumerate(PHASES):
        v = d[:, i]
        print(f"    {name:10s} median {np.median(v):7.0f}  p90 {np.percentile(v, 90):7.0f}  ({100 * v.sum() / tot.sum():5.1f} % of block time)")
    # phase boundaries in realtime: scale each block's memtime offsets into its realtime span
    frac = (st - st[:, :1]) / np.maximum(tot[:, None], 1)
    rtb = rt0[:, None] + frac * (rt1 - rt0)[:, None]
    ts = np.linspace(rt0.min(), rt1.max(), 61)[1:-1]
    rows = []
    for x in ts:
        inside = (rtb[:, 0] <= x) & (rtb[:, 6] > x)
        ph = np.argmax((rtb[:, 1:] > x), axis=1)  # first boundary after x -> phase index
        cnt = np.bincount(ph[inside], minlength=6)
        rows.append(cnt)
    rows = np.array(rows)
    mf = rows[:, 1] + rows[:, 3]
    mem = rows[:, 0] + rows[:, 5]
    oth = rows[:, 2] + rows[:, 4]
    print("  resident blocks in MFMA phases / memory phases (staging + row pass) / epilogues, 59 samples:")
    print("   mfma:", " ".join(str(v) for v in mf))
    print("   mem :", " ".join(str(v) for v in mem))
    print("   epi :", " ".join(str(v) for v in oth))
    busy = mf / np.maximum(mf + mem + oth, 1)
    print(f"  share of resident blocks in MFMA phases: mean {busy.mean():.2f}, min {busy.min():.2f}, max {busy.max():.2f}")


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]] or [128, 3, 1, 128, 11, 5, 256, 3, 1]
    targets = [tuple(a[i:i + 3]) for i in range(0, len(a), 3)]
    res = run(targets)
    for t in targets:
        analyze(res[t], t)
