"""Timeline of the last burst of kernels in a rocprofv3 kernel trace: the dispatches after the
last host gap longer than --gap ms (a probe sleeps before its traced trial), with each kernel's
start offset, duration and the idle time before it, then the burst's launch count, busy time
and span.
    python3 tools/last_burst.py <run_kernel_trace.csv> [--gap MS]"""
import csv
import sys


def main():
    args = sys.argv[1:]
    gap = float(args[args.index("--gap") + 1]) if "--gap" in args else 20.0
    path = [a for a in args if a.endswith(".csv")][0]
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))))
    first = 0
    for i in range(1, len(rows)):
        if (rows[i][0] - rows[i - 1][1]) / 1e6 > gap:
            first = i
    burst = rows[first:]
    t0 = burst[0][0]
    busy = 0.0
    prev_end = t0
    print(f"# {path}: last burst after a > {gap} ms gap; offset us, duration us, idle before us, kernel")
    for s, e, n in burst:
        d = (e - s) / 1e3
        busy += d
        print(f"{(s - t0) / 1e3:9.1f} {d:8.1f} {max(0.0, (s - prev_end) / 1e3):7.1f}  {n.split('(')[0][-90:]}")
        prev_end = max(prev_end, e)
    span = (burst[-1][1] - t0) / 1e3
    print(f"# {len(burst)} dispatches, busy {busy:.1f} us, span {span:.1f} us, idle {span - busy:.1f} us")


if __name__ == "__main__":
    main()
