"""Per-launch / per-stage breakdown of the last default-path vocoder step from a rocprofv3
kernel trace (bench.py --no-full --no-streaming ...; tools/prof_fused.sh).

usage: python tools/step_breakdown.py gpurun_out/<dir>/run_kernel_trace.csv [B T]
Labels come from tools/pmc_traffic.fused_step_layers (pre, ups, stage-0 convs, ResBlock
pairs, post); FLOPs are algorithmic (2*M*Cin*k per produced row; a pair counts both convs).
"""
import csv
import os
import sys
from collections import OrderedDict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.pmc_traffic import family, step_launches  # noqa: E402


def main():
    path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 862
    rows = [r for r in csv.DictReader(open(path)) if family(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    step = step_launches(B, T)
    rows = rows[-len(step):]
    stage = OrderedDict()
    total = 0.0
    print(f"{'launch':12s} {'kernel':10s} {'us':>9s} {'TF/s':>8s}")
    for (lab, _, f), r in zip(step, rows):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        total += us
        s = stage.setdefault(lab.split(".")[0], [0.0, 0.0])
        s[0] += us
        s[1] += f
        print(f"{lab:12s} {family(r['Kernel_Name']):10s} {us:9.1f} {f / (us * 1e-6) / 1e12:8.1f}")
    print()
    for st, (us, f) in stage.items():
        print(f"stage {st:5s} {us:9.1f} us  {f / (us * 1e-6) / 1e12:7.1f} TF/s  {100 * us / total:5.1f} %")
    print(f"step total {total:.1f} us")


if __name__ == "__main__":
    main()
