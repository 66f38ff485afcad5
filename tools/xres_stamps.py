"""Per-block phase timeline of one conv_xres launch (diagnostic build only).

Build:  python -m gonova_tts_amd.build --variant stamp -DTTS_XRES_STAMP=1 -DTTS_SPLIT_STAMP=1
Run:    TTS_LIB=<repo>/gonova-tts_amd/libtts_hip_stamp.so python3 tools/xres_stamps.py {ffn_up|ffn_down|qkv|s0up|s1up|e_*}
The e_* targets are the exact encoder's split-precision GEMMs (conv_split.hip) at batch 8.

The target launch shape (M, Cin, taps) is set in the library; the last launch of that shape in
the workload (acoustic forward at batch 32, or the C2 vocoder step) leaves one record per block.
Prints the launch span, the per-block phase split (first X staging, MFMA loop incl. later
stagings, summed staging, epilogue), blocks resident per CU over time, and the tail.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TARGETS = {  # (M, Cin, taps, workload)
    "ffn_up": (1536, 384, 3, "acoustic"),
    "ffn_down": (384, 1536, 3, "acoustic"),
    "qkv": (1152, 384, 1, "acoustic"),
    "s0up": (2048, 512, 2, "vocoder"),
    "s1up": (1024, 256, 2, "vocoder"),
    # exact encoder (fp32 split GEMMs) in a batch-8 forward
    "e_qkv": (1152, 384, 1, "acoustic8"),
    "e_out": (384, 384, 1, "acoustic8"),
    "e_pw1": (768, 384, 1, "acoustic8"),
    "e_ffn_up": (1536, 384, 3, "acoustic8"),
    "e_ffn_down": (384, 1536, 3, "acoustic8"),
    # the same split GEMMs in a batch-32 forward (C3)
    "E_qkv": (1152, 384, 1, "acoustic32s"),
    "E_ffn_up": (1536, 384, 3, "acoustic32s"),
    "E_ffn_down": (384, 1536, 3, "acoustic32s"),
}
WARM_S = float(os.environ.get("STAMP_WARM_S", "0"))  # back-to-back steps before the recorded one (clock settles)


def run(which):
    import torch
    from gonova_tts_amd.engine import HipEngine, load_library
    from gonova_tts_amd.weights import make_acoustic_weights, make_vocoder_weights
    M, Cin, taps, wl = TARGETS[which]
    lib = load_library()
    kind = "split" if wl in ("acoustic8", "acoustic32s") else "xres"
    set_target = getattr(lib, f"tts_debug_{kind}_target")
    read = getattr(lib, f"tts_debug_{kind}_stamps")
    set_target.argtypes = [ctypes.c_int] * 3
    read.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    assert set_target(M, Cin, taps) == 0
    g = torch.Generator(device="cpu").manual_seed(3)
    if wl.startswith("acoustic"):
        B, N = (8, 144) if wl == "acoustic8" else (32, 144)
        eng = HipEngine("cuda:0", acoustic_dtype="bf16", vocoder_dtype="bf16", max_batch=B, max_frames=N * 6, max_tokens=N)
        eng.load_weights(acoustic=make_acoustic_weights(seed=0, fixed_duration=6))
        tok = torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).cuda()
        tl = torch.full((B,), N, dtype=torch.int32).cuda()
        step = lambda: eng.acoustic(tok, tl, N * 6)  # noqa: E731
    else:
        eng = HipEngine("cuda:0", vocoder_dtype="f16", max_batch=32, max_frames=862)
        eng.load_weights(vocoder=make_vocoder_weights(seed=0))
        mel = torch.randn((32, 862, 80), generator=g).cuda()
        wav = torch.empty((32, 862 * 256), device="cuda")
        step = lambda: eng.vocoder(mel, out=wav)  # noqa: E731
    import time
    t0 = time.time()
    while time.time() - t0 < WARM_S:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    buf = np.zeros(1 << (18 if kind == "split" else 20), np.uint64)
    assert read(buf.ctypes.data, buf.size) == 0
    eng.close()
    rec = buf.reshape(-1, 8)
    rec = rec[rec[:, 0] != 0]
    return rec


def analyze(rec, which):
    st0, st1, st2, st3, ssum, rt0, rt3, hw = (rec[:, i].astype(np.float64) for i in range(8))
    hwid = rec[:, 7].astype(np.uint64)
    xcc = (hwid >> np.uint64(32)) & np.uint64(0xF)
    lo = hwid & np.uint64(0xFFFFFFFF)
    cu = (lo >> np.uint64(8)) & np.uint64(0xF)
    sh = (lo >> np.uint64(12)) & np.uint64(0x1)
    se = (lo >> np.uint64(13)) & np.uint64(0x7)
    cu_key = (xcc << np.uint64(16)) | (se << np.uint64(8)) | (sh << np.uint64(4)) | cu
    n = len(rec)
    tot = st3 - st0
    first = st1 - st0
    mfma = st2 - st1 - (ssum - first)   # MFMA loops (the later groups' staging removed)
    epi = st3 - st2
    clk = (st3 - st0).sum() / ((rt3 - rt0).sum() / 100e6)  # shader cycles per second
    span_us = (rt3.max() - rt0.min()) / 100.0
    print(f"{which}: {n} blocks, launch span {span_us:.1f} us (realtime), shader clock ~{clk / 1e9:.2f} GHz")
    print(f"  per block (cycles, median / p90): total {np.median(tot):.0f} / {np.percentile(tot, 90):.0f}")
    for name, v in (("first staging", first), ("all staging", ssum), ("MFMA loops", mfma), ("epilogue", epi)):
        print(f"    {name:14s} {np.median(v):8.0f} / {np.percentile(v, 90):8.0f}  ({100 * v.sum() / tot.sum():5.1f} % of block time)")
    print(f"  distinct CUs {len(np.unique(cu_key))}, blocks per CU max {np.bincount(np.unique(cu_key, return_inverse=True)[1]).max()}")
    # residency over time (realtime ticks of 10 ns)
    t = np.linspace(rt0.min(), rt3.max(), 41)
    res = [int(((rt0 <= x) & (rt3 > x)).sum()) for x in t]
    print("  blocks resident over the launch (41 samples):", " ".join(str(r) for r in res))
    ends = np.sort(rt3 - rt0.min()) / 100.0
    print(f"  block end times (us): 50% {ends[n // 2]:.1f}, 90% {ends[int(n * 0.9)]:.1f}, last {ends[-1]:.1f}")
    starts = np.sort(rt0 - rt0.min()) / 100.0
    print(f"  block start times (us): 50% {starts[n // 2]:.1f}, 90% {starts[int(n * 0.9)]:.1f}, last {starts[-1]:.1f}")


if __name__ == "__main__":
    for w in sys.argv[1:] or ["ffn_up"]:
        analyze(run(w), w)
