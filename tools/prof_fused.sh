#!/bin/bash
# usage (on the GPU box): bash tools/prof_fused.sh <outdir>  -- kernel trace of a short C2 bench
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-streaming --no-cpu-baseline --no-c1 > $O/bench.log 2>&1
