#!/bin/bash
# round 5: per-kernel trace of the batch-8 acoustic pass (predicted durations) at padded extent
# t_cap = 6 N (864) vs 12 N (1728, the streaming path's first-pass budget)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for TC in 864 1728; do
  ( export ACOUSTIC_PROF_B=8 ACOUSTIC_PROF_TCAP=$TC ACOUSTIC_PROF_LAUNCHES=1
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$TC -o run -- python3 $R/tools/acoustic_prof.py > $O/t$TC.log 2>&1 ) || { tail -5 $O/t$TC.log; exit 1; }
  ACOUSTIC_PROF_LAUNCHES=1 python3 $R/tools/acoustic_prof.py --summarize $O/t$TC/run_kernel_trace.csv > $O/sum$TC.txt || exit 1
  echo "== t_cap $TC"; head -30 $O/sum$TC.txt
done
echo r05q done
