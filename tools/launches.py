"""Per-launch durations of the last forward in a rocprofv3 kernel trace, optionally filtered by name.
usage: python3 tools/launches.py <run_kernel_trace.csv> <launches per forward> [substring ...]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    last = rows[-int(sys.argv[2]):]
    subs = sys.argv[3:]
    for r in last:
        n = r["Kernel_Name"]
        if subs and not any(s in n for s in subs):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        blocks = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(wg, 1)
        print(f"{d:8.1f} us  blocks {blocks:6d}  lds {r['LDS_Block_Size']:>6}  {n[:70]}")


if __name__ == "__main__":
    main()
