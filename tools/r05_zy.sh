#!/bin/bash
# round 5: C4 after the pinned asynchronous token upload -- GPU suite, the C4 kernel trace again
# (gaps between buckets), and the default bench's C4 / C3 / C5 lines (two runs)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash tools/r05_z.sh $T/trace > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -E "kernels|mrf_pair " $O/trace.txt
python3 - $O/trace/c4/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "tts::" in r["Kernel_Name"] or "_ZN3tts" in r["Kernel_Name"]]
g = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
big = sorted([x for x in g if x > 30], reverse=True)
print("gaps > 30 us:", len(big), "largest", [round(x, 1) for x in big[:12]])
PY
for rep in 1 2; do
  cd /tmp && timeout -k 10 600 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c1 > $O/b.$rep.json 2> $O/b.$rep.err || { tail -5 $O/b.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.$rep.json')); print($rep, 'C2', d['ms_per_step'], 'C3', d['full_pipeline']['ms_per_step'], 'C4', d['c4']['value'], d['c4']['ms_per_step'], 'C5', d['streaming']['p50_first_audio_ms'])"
done
echo r05zy done
