"""Effective clock and MFMA-pipe utilisation of one acoustic forward, per kernel family
(rocprofv3 --pmc pass over tools/acoustic_prof.py; pmc_clock.py's arithmetic).

usage (GPU box): rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
                 SQ_WAVE_CYCLES --kernel-trace --output-format csv -d <dir> -o run -- python3 tools/acoustic_prof.py
                 python3 tools/pmc_acoustic.py <dir>
"""
import csv
import sys
from collections import defaultdict

ITERS = 4  # tools/acoustic_prof.py


def short(name):
    for k in ("conv_xres", "conv_splitp", "conv_split_kernel", "split_reduce", "conv_gemm", "rel_attn_split",
              "rel_attn_kernel", "layernorm8", "layernorm_kernel", "glu_dwconv", "transpose_v", "ln_linear1"):
        if k in name:
            return k
    return "other"


def main():
    d = sys.argv[1]
    per, kname = defaultdict(dict), {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        kname[i] = r["Kernel_Name"]
    dur = {}
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(i for i in per if "tts::" in kname[i] or "_ZN3tts" in kname[i])
    ids = ids[-len(ids) // ITERS:]
    fam = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0.0, 0])
    for i in ids:
        c, t = per[i], dur.get(i, 0.0)
        f = fam[short(kname[i])]
        f[0] += t
        f[1] += c.get("GRBM_GUI_ACTIVE", 0) / 8
        f[2] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        f[3] += c.get("SQ_WAIT_INST_ANY", 0)
        f[4] += max(c.get("SQ_WAVE_CYCLES", 0), 1)
        f[5] += 1
    tot = sum(f[0] for f in fam.values())
    print(f"one acoustic forward (batch 32, bf16, exact encoder): {len(ids)} dispatches, {tot * 1e6:.0f} us under the profiler")
    print(f"{'family':18s} {'n':>4s} {'us':>8s} {'share':>6s} {'GHz':>5s} {'mfma%':>6s} {'@2.4':>6s}")
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        ghz = f[1] / max(f[0], 1e-12) / 1e9
        print(f"{k:18s} {f[5]:4d} {f[0] * 1e6:8.1f} {100 * f[0] / tot:5.1f}% {ghz:5.2f} "
              f"{100 * f[2] / max(f[1] * 1024, 1):6.1f} {100 * f[2] / (2.4e9 * f[0] * 1024):6.1f}")


if __name__ == "__main__":
    main()
