"""HBM traffic per kernel family of the default (fused) vocoder step, from two rocprofv3 PMC
passes (tools/pmc_traffic.sh).

usage: python tools/pmc_traffic.py <FETCH_SIZE dir> <WRITE_SIZE dir> [out.json] [B T]

Counters are collected in separate passes (TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2),
each with --kernel-trace only (MI355X_MICROARCH.md §rocprofv3 PMC slots).  Both are in
KB.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled; every HBM load of
these kernels is a 16-byte-per-lane load.  WRITE_SIZE is exact for 16-B stores (conv_xres
and mrf_fused write 16-B row pieces / 8-B fragments -- the latter uncalibrated, stated).

The last step's launches are mapped onto the step's launch sequence (step_launches):
  pre, s0.up, 18 x s0 conv, then per stage: up, one chain launch per chained resblock
  (k=3 at C=32/64, k=7 at C=32) or three pair launches, and post
and each family's traffic is compared with its algorithmic bytes: every conv reads its
input rows once, its weights once, writes its output once (+ the residual read of a
ResBlock's second conv); a ResBlock pair reads its input once, writes its output once,
reads both weight tensors once, and the last pair of the 2nd/3rd resblock also reads the
running MRF sum.
"""
import csv
import json
import os
import sys
from collections import defaultdict



def vocoder_layers(T):
    """(name, Cout, Cin, k, frames) of every vocoder conv for T mel frames, in launch order:
    conv_pre, then per stage the upsampler and 18 MRF convs, then conv_post."""
    layers = [("pre", 512, 80, 7, T)]
    ch, up, ks = [256, 128, 64, 32], [8, 8, 2, 2], [3, 7, 11]
    cin, t = 512, T
    for i in range(4):
        layers.append((f"s{i}.up", up[i] * ch[i], cin, 2, t))
        t *= up[i]
        for k in ks:
            for d in (1, 3, 5):
                layers.append((f"s{i}.k{k}.c1", ch[i], ch[i], k, t))
                layers.append((f"s{i}.k{k}.c2", ch[i], ch[i], k, t))
        cin = ch[i]
    layers.append(("post", 1, 32, 7, t))
    return layers


FAMILIES = ("conv_gemm", "conv_xres", "mrf_fused", "mrf_pair", "mrf_chain", "conv_post", "upsample_stream")


def family(name):
    for f in FAMILIES:
        if f in name:
            return f
    return None


def per_dispatch(path, counter):
    vals, names = {}, {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or family(r["Kernel_Name"]) is None:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
        names[d] = family(r["Kernel_Name"])
    ids = sorted(vals)
    return [vals[i] for i in ids], [names[i] for i in ids]


CHAIN = {(32, 3), (32, 7), (64, 3)}   # (C, k) resblocks run as one chain launch (mrf_chain.hip)


def step_launches(B, T, elt=2, pair_channels=(32, 64, 128, 256), chain=CHAIN, post_fused=True):
    """[(label, algorithmic bytes, algorithmic FLOPs)] of one default-path step, in launch
    order: single convs for stages whose width has no pair kernel, one chain launch per
    resblock in `chain`, ResBlock-pair launches otherwise; conv_post inside the last pair
    launch when `post_fused` (the final MRF sum is not written, the waveform is)."""
    out = []
    npairs = {}
    for name, M, cin, k, n in vocoder_layers(T):
        st = name.split(".")[0]
        f = 2.0 * M * cin * k * n * B
        if name == "post" and post_fused and out and ".pair" in out[-1][0]:
            lab, by, fl = out[-1]
            out[-1] = (lab + "+post", by - B * n * cin * elt + B * n * 4, fl + f)
        elif name == "post":
            out.append(("post", B * n * cin * elt + B * n * 4, f))
        elif name == "pre" or name.endswith(".up"):
            out.append((name, B * n * cin * elt + B * n * M * elt + M * cin * k * elt, f))
        elif M in pair_channels:
            if not name.endswith(".c2"):
                continue
            idx = npairs.get(st, 0)   # pair index within the stage (3 per resblock)
            npairs[st] = idx + 1
            accum = idx >= 3          # the 2nd/3rd resblock's output adds the running MRF sum
            act = B * n * M * elt
            if (M, k) in chain:
                if idx % 3 == 2:      # the chain launch, counted at its resblock's last pair
                    out.append((f"{st}.k{k}.chain", 2 * act + (act if accum else 0) + 6 * M * cin * k * elt,
                                3 * 2 * f))
            else:
                out.append((f"{st}.pair{idx}", 2 * act + (act if accum and idx % 3 == 2 else 0)
                            + 2 * M * cin * k * elt, 2 * f))
        else:
            r = B * n * M * elt if name.endswith(".c2") else 0
            out.append((name, B * n * cin * elt + B * n * M * elt + M * cin * k * elt + r, f))
    return out


def fused_step_layers(B, T, elt=2, pair_channels=(32, 64, 128, 256)):
    """[(label, algorithmic bytes)] of one default-path step, in launch order."""
    return [(lab, by) for lab, by, _ in step_launches(B, T, elt, pair_channels)]


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    outp = sys.argv[3] if len(sys.argv) > 3 else None
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 862
    fetch, fam = per_dispatch(f"{fdir}/run_counter_collection.csv", "FETCH_SIZE")
    write, fam_w = per_dispatch(f"{wdir}/run_counter_collection.csv", "WRITE_SIZE")
    step = fused_step_layers(B, T)
    n = len(step)
    fetch, fam, write, fam_w = fetch[-n:], fam[-n:], write[-n:], fam_w[-n:]
    if fam != fam_w:
        raise SystemExit("FETCH and WRITE passes dispatched different kernel sequences")
    fams = {}
    for f in FAMILIES:
        idx = [i for i in range(n) if fam[i] == f]
        if not idx:
            continue
        hbm = sum((2.0 * fetch[i] + write[i]) * 1024.0 for i in idx)
        alg = sum(step[i][1] for i in idx)
        fams[f] = {"launches_per_step": len(idx), "layers": [step[i][0] for i in idx],
                   "traffic_bytes_per_launch": hbm / len(idx),
                   "algorithmic_bytes_per_launch": alg / len(idx),
                   "ratio_traffic_over_algorithmic": hbm / alg,
                   "raw_fetch_kb_per_launch": sum(fetch[i] for i in idx) / len(idx),
                   "raw_write_kb_per_launch": sum(write[i] for i in idx) / len(idx)}
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace), "
                     "last C2 step of the default (fused) path",
           "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE halves 16-B/lane reads)",
           "batch": B, "frames": T, "families": fams}
    print(json.dumps(res, indent=1))
    if outp:
        json.dump(res, open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
