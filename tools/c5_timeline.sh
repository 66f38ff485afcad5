#!/bin/bash
# usage (GPU box): bash tools/c5_timeline.sh <tag>
# Where C5's first-audio time goes -- one traced trial's kernel
# timeline (tools/c5_trace.py + tools/last_burst.py), plus the untraced C5 p50
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/c5_trace.py > $O/c5_plain.txt 2>&1 || { tail -5 $O/c5_plain.txt; exit 1; }
tail -1 $O/c5_plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c5 -o run -- python3 $R/tools/c5_trace.py > $O/c5_prof.log 2>&1 || { tail -5 $O/c5_prof.log; exit 1; }
python3 $R/tools/last_burst.py $O/c5/run_kernel_trace.csv > $O/c5_timeline.txt || exit 1
tail -3 $O/c5_timeline.txt
echo $T done
