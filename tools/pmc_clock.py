"""Effective clock and MFMA-pipe utilisation per dispatch of the last C2 step
(tools/pmc_clock.sh output).

usage: python tools/pmc_clock.py gpurun_out/<dir>
clock = GRBM_GUI_ACTIVE / kernel duration (the GPU's own cycle count over the dispatch);
mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs): the MFMA pipes' busy fraction
at the clock the chip actually ran, next to the same at the nominal 2.4 GHz.
SQ wave-state counters are quad-cycles (MI355X_MICROARCH.md constants table).
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from tools.pmc_traffic import family, step_launches  # noqa: E402


def main():
    d = sys.argv[1]
    per, names, dur = defaultdict(dict), {}, {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        f = family(r["Kernel_Name"])
        if f is None:
            continue
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = f
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(per)
    step = step_launches(32, 862)
    ids = ids[-len(step):]
    print(f"{'launch':12s} {'kernel':10s} {'us':>8s} {'GHz':>6s} {'mfma%':>6s} {'@2.4':>6s} {'waitI%':>7s} {'wait%':>6s}")
    for (lab, _, _), i in zip(step, ids):
        c, t = per[i], dur.get(i, 0.0)
        # GRBM_GUI_ACTIVE is summed over the XCDs' GRBM instances: cycles of one = max / XCDs
        ghz = c.get("GRBM_GUI_ACTIVE", 0) / 8 / max(t, 1e-12) / 1e9
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        W = max(c.get("SQ_WAVE_CYCLES", 0), 1)
        print(f"{lab:12s} {names[i]:10s} {t * 1e6:8.1f} {ghz:6.2f} {100 * busy / max(ghz * 1e9 * t * 1024, 1):6.1f}"
              f" {100 * busy / (2.4e9 * t * 1024):6.1f} {100 * c.get('SQ_WAIT_INST_ANY', 0) / W:7.1f}"
              f" {100 * c.get('SQ_WAIT_ANY', 0) / W:6.1f}")


if __name__ == "__main__":
    main()
