#!/bin/bash
# usage (on the GPU box): bash tools/ab_conv.sh <outdir> [ENV=VAL ...]
#  -- unfused-path kernel trace of a short C2 bench under the given env (for per-layer A/B)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-streaming --no-cpu-baseline > $O/bench.log 2>&1
