#!/bin/bash
# round 5: C1 (fp32 engine, one 71-token sentence) -- host time of generate() and the kernel
# trace of the same calls, summarised per kernel (one call's share = total / 13)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1.txt 2>&1 || { tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/tools/c1_prof.py > $O/c1_tr.txt 2>&1 || { tail -5 $O/c1_tr.txt; exit 1; }
python3 - $O/tr/run_kernel_trace.csv <<'PY' | tee $O/summary.txt
import csv, sys
from collections import defaultdict
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
agg = defaultdict(lambda: [0, 0.0, ""])
for r in rows:
    k = r["Kernel_Name"][:90]
    a = agg[k]; a[0] += 1; a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a[2] = f'grid {r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]} wg {r["Workgroup_Size_X"]}'
tot = sum(a[1] for a in agg.values())
print(f"kernels {len(rows)} ({len(rows)/13:.0f} per call), kernel time per call {tot/13/1e3:.3f} ms")
for k, a in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{a[1]/13:9.1f} us/call {a[0]//13:4d}x  {k}  {a[2]}")
PY
echo r05zv done
