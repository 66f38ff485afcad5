#!/bin/bash
# round 6: C1 per-kernel breakdown on the current code (one rocprofv3 kernel trace of tools/c1_prof.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06v}; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1 -o run -- python3 $R/tools/c1_prof.py > $O/c1_prof.log 2>&1 || { tail -5 $O/c1_prof.log; exit 1; }
python3 $R/tools/kernel_summary.py $O/c1/run_kernel_trace.csv --top 40 > $O/c1_kernels.txt || exit 1
python3 $R/tools/last_burst.py $O/c1/run_kernel_trace.csv --gap 0.3 > $O/c1_timeline.txt || exit 1
tail -1 $O/c1_timeline.txt
echo $T done
