"""Per-layer PMC table for the unfused vocoder step (output of tools/pmc_layers.sh).

usage: python tools/pmc_layers.py gpurun_out/<dir> [B T]
Takes the last step's conv_gemm dispatches of each pass, names them with
layer_breakdown.vocoder_layers and sums counters per layer group.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(__file__))
from layer_breakdown import vocoder_layers  # noqa: E402


def main():
    d = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 862
    names = [l[0] for l in vocoder_layers(T) if l[0] != "post"]
    agg = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(float)
    for f in sorted(glob.glob(f"{d}/pass*/run_counter_collection.csv")):
        per = defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(f)):
            if not ("conv_gemm" in r["Kernel_Name"] or "conv_xres" in r["Kernel_Name"]):
                continue
            i = int(r["Dispatch_Id"])
            per[i][r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(per)[-len(names):]
        for name, i in zip(names, ids):
            for c, v in per[i].items():
                agg[name][c] += v
        kt = glob.glob(os.path.join(os.path.dirname(f), "run_kernel_trace.csv"))
        if kt and not dur:
            rows = [r for r in csv.DictReader(open(kt[0])) if "conv_gemm" in r["Kernel_Name"] or "conv_xres" in r["Kernel_Name"]]
            rows.sort(key=lambda r: int(r["Dispatch_Id"]))
            for name, r in zip(names, rows[-len(names):]):
                dur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cols = [("us", lambda c, n: dur[n]),
            ("VALU/MFMA", lambda c, n: c["SQ_INSTS_VALU"] / max(c["SQ_INSTS_MFMA"], 1)),
            ("MFMAbusy%", lambda c, n: 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(dur[n] * 1e-6 * 2.4e9 * 1024, 1)),
            ("wait%", lambda c, n: 100 * c["SQ_WAIT_ANY"] / max(c["SQ_WAVE_CYCLES"], 1)),
            ("valu%", lambda c, n: 100 * c["SQ_ACTIVE_INST_VALU"] / max(c["SQ_WAVE_CYCLES"], 1)),
            ("lds%", lambda c, n: 100 * c["SQ_ACTIVE_INST_LDS"] / max(c["SQ_WAVE_CYCLES"], 1)),
            ("vmem%", lambda c, n: 100 * c["SQ_ACTIVE_INST_VMEM"] / max(c["SQ_WAVE_CYCLES"], 1)),
            ("L2req/us", lambda c, n: c["TCP_TCC_READ_REQ_sum"] / max(dur[n], 1)),
            ("L2hit%", lambda c, n: 100 * c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)),
            ("HBM GB/s", lambda c, n: (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1.024 / max(dur[n], 1)),  # KB; FETCH x2 on gfx950
            ("bankconf%", lambda c, n: 100 * c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1))]
    print(f"{'layer':12s}" + "".join(f"{h:>11s}" for h, _ in cols))
    seen = []
    for n in names:
        if n not in seen:
            seen.append(n)
    for n in seen:
        c = agg[n]
        out = []
        for _, fn in cols:
            try:
                out.append(f"{fn(c, n):11.1f}")
            except (KeyError, ZeroDivisionError):
                out.append(f"{'-':>11s}")
        print(f"{n:12s}" + "".join(out))


if __name__ == "__main__":
    main()
