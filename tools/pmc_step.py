"""Per-dispatch PMC table of the last vocoder step (output of tools/pmc_step.sh).

usage: python tools/pmc_step.py gpurun_out/<dir> [substring filter]
The last step = the dispatches after the second-to-last conv_post; rates use the kernel
trace's durations and 2.4 GHz x 1024 SIMDs for MFMA busy.
"""
import csv
import glob
import sys
from collections import defaultdict

KERNELS = ("conv_gemm", "conv_xres", "mrf_fused", "mrf_pair", "conv_post")


def short(n):
    for k in KERNELS:
        if k in n:
            return k + ("16" if "DF16_" in n else "bf" if "DF16b" in n else "")
    return None


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    per = defaultdict(dict)
    names, dur = {}, {}
    for f in sorted(glob.glob(f"{d}/pass*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s is None:
                continue
            i = int(r["Dispatch_Id"])
            per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[i] = s
        kt = f.replace("run_counter_collection.csv", "run_kernel_trace.csv")
        if not dur and glob.glob(kt):
            for r in csv.DictReader(open(kt)):
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ids = sorted(per)
    posts = [i for i in ids if names[i].startswith("conv_post")]
    step = [i for i in ids if i > posts[-2]] if len(posts) > 1 else ids
    cols = ["us", "VALU/MFMA", "MFMAbusy%", "wait%", "valu%", "lds%", "ldsconf%", "L2req/us", "L2hit%"]
    print(f"{'#':>3s} {'kernel':14s}" + "".join(f"{c:>10s}" for c in cols))
    for n, i in enumerate(step):
        c, t = per[i], dur.get(i, 0.0)
        if filt and filt not in names[i]:
            continue
        W = max(c.get("SQ_WAVE_CYCLES", 0), 1)
        vals = [t, c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_INSTS_MFMA", 0), 1),
                100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(t * 1e-6 * 2.4e9 * 1024, 1),
                100 * c.get("SQ_WAIT_ANY", 0) / W, 100 * c.get("SQ_ACTIVE_INST_VALU", 0) / W,
                100 * c.get("SQ_ACTIVE_INST_LDS", 0) / W,
                100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 0), 1),
                c.get("TCP_TCC_READ_REQ_sum", 0) / max(t, 1e-9),
                100 * c.get("TCC_HIT_sum", 0) / max(c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0), 1)]
        print(f"{n:3d} {names[i]:14s}" + "".join(f"{v:10.1f}" for v in vals))


if __name__ == "__main__":
    main()
