"""Per-kernel launch count / average / total duration from rocprofv3 kernel traces:
    python3 tools/kernel_summary.py <run_kernel_trace.csv> [more ...] [--top N] [--match SUBSTR]"""
import collections
import csv
import sys


def summary(path, match=None):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if match and match not in n:
            continue
        agg[n.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return agg


if __name__ == "__main__":
    args = sys.argv[1:]
    top = int(args[args.index("--top") + 1]) if "--top" in args else 25
    match = args[args.index("--match") + 1] if "--match" in args else None
    files = [a for a in args if a.endswith(".csv")]
    for f in files:
        agg = summary(f, match)
        print(f)
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
            print(f"  {k[-70:]:70s} n={len(v):4d} avg={sum(v) / len(v):9.1f} us tot={sum(v) / 1e3:8.2f} ms")
