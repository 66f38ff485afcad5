"""Print the last bench step's kernel durations from a rocprofv3 kernel trace (fused or unfused)."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if any(k in r["Kernel_Name"] for k in ("mrf_fused", "mrf_pair", "conv_gemm", "conv_xres", "conv_post"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step ends with conv_post
ends = [i for i, r in enumerate(rows) if "conv_post" in r["Kernel_Name"]]
start = ends[-2] + 1 if len(ends) > 1 else 0
tot = 0.0
for r in rows[start:ends[-1] + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].split("kernel")[0][-12:] + r["Kernel_Name"].split("kernel")[1][:28]
    print(f"{name:44s} grid {r['Grid_Size_X']:>7}x{r['Grid_Size_Y']:<3} {d:9.1f} us")
print(f"step total {tot:.1f} us")
