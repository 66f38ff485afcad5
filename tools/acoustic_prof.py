"""Acoustic-model (C3 front half) launch profile: run the bf16 FS2-Conformer forward at
B=32 x 144 tokens x 6 frames a few times; under rocprofv3 --kernel-trace, `--summarize <csv>`
prints per-kernel time of one forward (the last) sorted by total.

usage (GPU box): rocprofv3 --kernel-trace --output-format csv -d <dir> -o run -- python3 tools/acoustic_prof.py
                 python3 tools/acoustic_prof.py --summarize <dir>/run_kernel_trace.csv
"""
import csv
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ITERS = 4


def run():
    import torch
    from gonova_tts_amd.engine import HipEngine
    from gonova_tts_amd.weights import make_acoustic_weights
    B, N, dur = int(os.environ.get("ACOUSTIC_PROF_B", "32")), 144, 6
    t_cap = int(os.environ.get("ACOUSTIC_PROF_TCAP", str(N * dur)))  # padded frame extent (predicted durations)
    eng = HipEngine("cuda:0", acoustic_dtype="bf16", max_batch=B, max_frames=t_cap, max_tokens=N)
    eng.load_weights(acoustic=make_acoustic_weights(seed=0, fixed_duration=dur))
    g = torch.Generator(device="cpu").manual_seed(2000)
    tok = torch.randint(1, 78, (B, N), generator=g, dtype=torch.int32).cuda()
    tl = torch.full((B,), N, dtype=torch.int32, device="cuda")
    for _ in range(ITERS):
        eng.acoustic(tok, tl, t_cap)
        torch.cuda.synchronize()
    eng.close()


def summarize(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "tts::" in r["Kernel_Name"] or "_ZN3tts" in r["Kernel_Name"]]
    n = len(rows) // ITERS
    last = rows[-n:]
    tot = defaultdict(lambda: [0.0, 0])
    for r in last:
        k = r["Kernel_Name"]
        k = k[:60]
        tot[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[k][1] += 1
    span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
    busy = sum(v[0] for v in tot.values())
    print(f"one forward: {n} launches, kernel time {busy:.1f} us, span {span:.1f} us")
    for k, (us, c) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print(f"{us:9.1f} us {c:4d}x  {k}")
    if os.environ.get("ACOUSTIC_PROF_LAUNCHES"):
        for r in last:
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"{us:8.1f} us grid {r.get('Grid_Size', '?'):>9} wg {r.get('Workgroup_Size', '?'):>4} "
                  f"lds {r.get('LDS_Block_Size', r.get('Lds_Size', '?')):>6}  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
