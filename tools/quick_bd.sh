#!/bin/bash
# usage (on the GPU box): bash tools/quick_bd.sh <tag> -- C2 bench line + per-launch breakdown of the last step
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python3 -u $R/bench.py --no-full --no-streaming --no-cpu-baseline --no-c1 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
bash $R/tools/prof_fused.sh $1/prof || exit 1
python3 $R/tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/breakdown.txt || exit 1
python3 -c "import json,sys; d=json.load(open('$O/bench.json')); print('ms_per_step', d['ms_per_step'], 'value', d['value'])"
cat $O/breakdown.txt
