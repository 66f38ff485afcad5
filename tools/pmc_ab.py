"""Per-dispatch PMC summary of the last C2 step (tools/pmc_ab.sh output) for the MRF kernels:
    python3 tools/pmc_ab.py gpurun_out/<tag> <lib name> [--match SUBSTR]
clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs);
wait% / issue% / active% = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES;
valu/mfma, lds/mfma = instructions per MFMA; bank = LDS bank-conflict cycles per LDS instruction."""
import csv
import sys
from collections import defaultdict


def load(d):
    per, name, dur = defaultdict(dict), {}, {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[i] = r["Kernel_Name"]
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per, name, dur


def main():
    base, lib = sys.argv[1], sys.argv[2]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "mrf_"
    pa, na, da = load(f"{base}/a_{lib}")
    pb, nb, db = load(f"{base}/b_{lib}")
    ia = [i for i in sorted(pa) if match in na[i]]
    ib = [i for i in sorted(pb) if match in nb[i]]
    n = min(len(ia), len(ib))
    ia, ib = ia[-n:], ib[-n:]  # the last step's dispatches, matched in order
    print(f"{'kernel':58s} {'us':>7s} {'GHz':>5s} {'mfma%':>6s} {'wait%':>6s} {'issue%':>6s} {'act%':>5s} "
          f"{'valu/mf':>7s} {'lds/mf':>6s} {'bank':>5s} {'ldsW%':>5s}")
    for x, y in zip(ia, ib):
        a, b = pa[x], pb[y]
        t = da[x]
        clk = a["GRBM_GUI_ACTIVE"] / 8 / t
        mf = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] / 8 * 1024)
        wc = a["SQ_WAVE_CYCLES"]
        nm = na[x].split("(")[0][-58:]
        im = b["SQ_INSTS_MFMA"] or 1
        print(f"{nm:58s} {t * 1e6:7.1f} {clk / 1e9:5.2f} {100 * mf:6.1f} {100 * a['SQ_WAIT_ANY'] / wc:6.1f} "
              f"{100 * a['SQ_WAIT_INST_ANY'] / wc:6.1f} {100 * a['SQ_ACTIVE_INST_ANY'] / wc:5.1f} "
              f"{b['SQ_INSTS_VALU'] / im:7.2f} {b['SQ_INSTS_LDS'] / im:6.2f} "
              f"{b['SQ_LDS_BANK_CONFLICT'] / max(b['SQ_INSTS_LDS'], 1):5.2f} {100 * b['SQ_WAIT_INST_LDS'] / b['SQ_WAVE_CYCLES']:5.1f}")


if __name__ == "__main__":
    main()
