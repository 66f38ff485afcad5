#!/bin/bash
# round 5: fp32 split-K (C1) -- GPU suite, then the C1 probe + per-kernel trace (tools/r05_zv.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash tools/r05_zv.sh $T/c1 || exit 1
cd /tmp && timeout -k 10 600 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full --no-c4 --no-streaming > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print('C2', d['ms_per_step'], 'C1', d['c1'])"
echo r05zu done
