#!/bin/bash
# usage (GPU box): bash tools/probe_ac.sh <tag> <B> <substring> <lib.so> [lib.so ...]
# acoustic forward launch profile (tools/acoustic_prof.py) per library build; per-launch times of
# the kernels matching <substring> -> gpurun_out/<tag>/<lib>.txt
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; B=$2; SUB=$3; shift 3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  TTS_LIB=$R/$L ACOUSTIC_PROF_B=$B timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$n -o run -- python3 $R/tools/acoustic_prof.py > $O/p_$n.log 2>&1 || exit 1
  python3 $R/tools/acoustic_prof.py --summarize $O/p_$n/run_kernel_trace.csv > $O/$n.sum || exit 1
  N=$(head -1 $O/$n.sum | awk '{print $3}')
  python3 $R/tools/launches.py $O/p_$n/run_kernel_trace.csv $N $SUB > $O/$n.txt || exit 1
done
