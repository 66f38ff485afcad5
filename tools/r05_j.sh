#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c5 -o run -- python3 $R/tools/c5_probe.py > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -5 $O/c5.log
python3 - $O/c5/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "tts" in r["Kernel_Name"]]
# the last trial: find the last vocoder chunk (after the last acoustic regulate kernel)
idx = [i for i, r in enumerate(rows) if "regulate" in r["Kernel_Name"]]
last = rows[idx[-1]:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} us grid {r.get('Grid_Size', '?'):>8}  {r['Kernel_Name'][:80]}")
PY
