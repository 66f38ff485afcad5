"""Per-layer breakdown of one vocoder step from a rocprofv3 kernel-trace CSV.

usage: python tools/layer_breakdown.py gpurun_out/<dir>/run_kernel_trace.csv [B T]
Aligns the last step's dispatches (conv_pre, 4 x [upsample + 18 MRF convs], conv_post)
with the known layer list and prints time / achieved TFLOP/s / share per layer group.
"""
import csv
import sys


def vocoder_layers(T):
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


def main():
    path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 862
    rows = [r for r in csv.DictReader(open(path))
            if "conv_gemm" in r["Kernel_Name"] or "conv_xres" in r["Kernel_Name"] or "conv_post" in r["Kernel_Name"] or "pair" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    layers = vocoder_layers(T)
    last = rows[-len(layers):]
    agg, order, tot = {}, [], 0.0
    for r, (name, M, cin, k, n) in zip(last, layers):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        fl = 2.0 * M * cin * k * n * B
        tot += dur
        if name not in agg:
            agg[name] = [0.0, 0.0]
            order.append(name)
        agg[name][0] += dur
        agg[name][1] += fl
    for n in order:
        d, f = agg[n]
        print(f"{n:12s} {d:9.1f} us {f / d / 1e6:8.1f} TF/s  {d / tot * 100:5.1f}%")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
