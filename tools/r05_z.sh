#!/bin/bash
# round 5: where a C4 step's time goes -- kernel trace of `bench.py --workload c4` (3 steps), GPU
# busy time per step vs the step's wall time, by kernel family
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/c4 -o run -- python3 $R/bench.py --workload c4 --steps 3 --warmup 1 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
cat $O/c4.json | cut -c1-400
python3 - $O/c4/run_kernel_trace.csv <<'PY'
import csv, sys
from collections import defaultdict
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "tts::" in r["Kernel_Name"] or "_ZN3tts" in r["Kernel_Name"]]
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
print(f"kernels {len(rows)}, busy {busy/1e6:.1f} ms over a span of {(t1-t0)/1e6:.1f} ms ({100*busy/(t1-t0):.1f} %)")
fam = defaultdict(float)
for r in rows:
    k = r["Kernel_Name"]
    for f in ("mrf_pair", "mrf_chain", "conv_xres", "conv_splitp", "conv_split", "rel_attn", "upsample", "conv_gemm", "layernorm", "glu"):
        if f in k:
            fam[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            break
    else:
        fam["other"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    print(f"{k:12s} {v:8.1f} ms")
PY
echo r05z done
