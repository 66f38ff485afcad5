"""HBM traffic of the implicit-GEMM conv launches from two rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py <FETCH_SIZE dir> <WRITE_SIZE dir> [out.json] [B T]

Counters are collected in separate passes (TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2),
each with --kernel-trace only (MI355X_MICROARCH.md §rocprofv3 PMC slots).  Both are in
KB.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled; every operand
load of conv_gemm_kernel is a 16-byte-per-lane load.  WRITE_SIZE is exact for 16-B
stores and is used as is (the kernel's 8-byte stores are uncalibrated -- stated).

The last vocoder step's 77 conv launches are averaged and compared with their
algorithmic bytes (read X once, read W once, write Y once, read residuals once).
"""
import csv
import json
import sys

sys.path.insert(0, ".")
from tools.layer_breakdown import vocoder_layers  # noqa: E402


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "conv_gemm" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def algorithmic_bytes(B, T, elt=2):
    out = []
    for name, M, cin, k, n in vocoder_layers(T):
        if name == "post":
            continue
        x = B * n * cin * elt          # input rows read once
        y = B * n * M * elt            # output written once (upsampler: M = s*Cout per input row)
        w = M * cin * k * elt          # weights read once
        r = y if name.endswith(".c2") else 0  # ResBlock residual (the MRF running sum adds 2/9 more)
        out.append(x + y + w + r)
    return out


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    outp = sys.argv[3] if len(sys.argv) > 3 else None
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 862
    fetch = per_dispatch(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE")
    n = 77
    fetch, write = fetch[-n:], write[-n:]
    alg = algorithmic_bytes(B, T)
    hbm = [(2.0 * f + w) * 1024.0 for f, w in zip(fetch, write)]
    res = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), last C2 step",
        "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE halves 16-B/lane reads)",
        "launches": len(hbm),
        "traffic_bytes_per_launch": sum(hbm) / len(hbm),
        "algorithmic_bytes_per_launch": sum(alg) / len(alg),
        "ratio_traffic_over_algorithmic": (sum(hbm) / sum(alg)),
        "raw_fetch_kb_per_launch": sum(fetch) / len(fetch),
        "raw_write_kb_per_launch": sum(write) / len(write),
    }
    print(json.dumps(res, indent=1))
    if outp:
        json.dump(res, open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
