#!/bin/bash
# usage (GPU box): bash tools/split_prof.sh <tag> [extra env]  -- acoustic launch profile (B=32 and B=8)
# plus the acoustic GPU tests; everything under gpurun_out/<tag>/
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for B in 32 8; do
  ACOUSTIC_PROF_B=$B timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ap$B -o run -- python3 $R/tools/acoustic_prof.py > $O/ap$B.log 2>&1 || exit 1
  python3 $R/tools/acoustic_prof.py --summarize $O/ap$B/run_kernel_trace.csv > $O/ap${B}_summary.txt || exit 1
done
