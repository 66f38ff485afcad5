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


def load(d):
    per, kname = defaultdict(dict), {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        kname[i] = r["Kernel_Name"]
    dur = {}
    for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(i for i in per if "tts::" in kname[i] or "_ZN3tts" in kname[i])
    return per, kname, dur, ids[-len(ids) // ITERS:]  # the last forward


def main():
    """args: <clock/MFMA dir> [<FETCH_SIZE dir> <WRITE_SIZE dir> <instmix dir>] [batch]"""
    dirs = [a for a in sys.argv[1:] if not a.isdigit()]
    batch = next((a for a in sys.argv[1:] if a.isdigit()), "32")
    per, kname, dur, ids = load(dirs[0])
    # per family: time, GRBM cycles and time of the long dispatches, MFMA busy, waits, wave cycles, count
    fam = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0.0, 0, 0.0])
    for i in ids:
        c, t = per[i], dur.get(i, 0.0)
        f = fam[short(kname[i])]
        f[0] += t
        if t >= 20e-6:
            f[1] += c.get("GRBM_GUI_ACTIVE", 0) / 8
            f[6] += t
        f[2] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        f[3] += c.get("SQ_WAIT_INST_ANY", 0)
        f[4] += max(c.get("SQ_WAVE_CYCLES", 0), 1)
        f[5] += 1
    extra = defaultdict(lambda: defaultdict(float))
    # FETCH_SIZE / WRITE_SIZE in KB; FETCH doubled (MI355X_MICROARCH.md gfx950 correction for 16 B/lane loads)
    for d, key, mul in ((dirs[1], "FETCH_SIZE", 2.0), (dirs[2], "WRITE_SIZE", 1.0)) if len(dirs) >= 3 else ():
        p2, k2, _, ids2 = load(d)
        for i in ids2:
            extra[short(k2[i])][key] += p2[i].get(key, 0.0) * 1024 * mul
    if len(dirs) >= 4:
        p3, k3, _, ids3 = load(dirs[3])
        for i in ids3:
            e = extra[short(k3[i])]
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS",
                      "SQ_WAVE_CYCLES"):
                e[k] += p3[i].get(k, 0.0)
    tot = sum(f[0] for f in fam.values())
    print(f"one acoustic forward (batch {batch}, bf16, exact encoder): {len(ids)} dispatches, {tot * 1e6:.0f} us under the profiler")
    print("mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (clock x duration x 1024 SIMDs): GHz = GRBM_GUI_ACTIVE/8 / duration over the")
    print("family's dispatches of >= 20 us (a short dispatch's counter window outlasts its trace duration, which")
    print("overstated the clock); '-' where none is that long, '>2.4' where the quotient still exceeds the chip's")
    print("2.4 GHz peak (the window still outlasts the dispatch: clock not measurable this way), mfma% then only")
    print("at the nominal 2.4 GHz (@2.4, a lower bound on the busy fraction);")
    print("FETCH (x2 gfx950 correction) / WRITE in MB per forward; valu/mfma, lds/mfma instructions; bankconf = extra LDS cycles per LDS instruction")
    print(f"{'family':18s} {'n':>4s} {'us':>8s} {'share':>6s} {'GHz':>5s} {'mfma%':>6s} {'@2.4':>6s} {'FETCH':>8s} {'WRITE':>8s} "
          f"{'valu/mf':>7s} {'lds/mf':>6s} {'bankc':>6s}")
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        e = extra[k]
        if f[6] > 0 and f[1] / f[6] / 1e9 <= 2.4:
            ghz = f[1] / f[6] / 1e9
            g_s, m_s = f"{ghz:5.2f}", f"{100 * f[2] / (ghz * 1e9 * f[0] * 1024):6.1f}"
        elif f[6] > 0:  # above the chip's peak: not a clock
            g_s, m_s = f"{'>2.4':>5s}", f"{'-':>6s}"
        else:
            g_s, m_s = f"{'-':>5s}", f"{'-':>6s}"
        mf = e.get("SQ_INSTS_MFMA", 0.0)
        lds = e.get("SQ_INSTS_LDS", 0.0)
        r_valu = f"{e.get('SQ_INSTS_VALU', 0) / mf:7.2f}" if mf else f"{'-':>7s}"
        r_lds = f"{lds / mf:6.2f}" if mf else f"{'-':>6s}"
        r_bank = f"{e.get('SQ_LDS_BANK_CONFLICT', 0) / lds:6.2f}" if lds else f"{'-':>6s}"
        print(f"{k:18s} {f[5]:4d} {f[0] * 1e6:8.1f} {100 * f[0] / tot:5.1f}% {g_s} {m_s} "
              f"{100 * f[2] / (2.4e9 * f[0] * 1024):6.1f} "
              f"{e.get('FETCH_SIZE', 0) / 1e6:8.1f} {e.get('WRITE_SIZE', 0) / 1e6:8.1f} {r_valu} {r_lds} {r_bank}")


if __name__ == "__main__":
    main()
