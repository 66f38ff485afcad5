#!/bin/bash
# usage (on the GPU box): bash tools/ab_acoustic.sh <tag> <variant .so> ...  -- per-kernel acoustic profile per build
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
LIBS="$R/gonova-tts_amd/libtts_hip.so"
for L in "$@"; do case $L in /*) LIBS="$LIBS $L";; *) LIBS="$LIBS $R/$L";; esac; done
cd /tmp && export TMPDIR=/tmp
for L in $LIBS; do
  n=$(basename $L .so)
  TTS_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 $R/tools/acoustic_prof.py > $O/$n.log 2>&1 || exit 1
  echo "== $n"; python3 $R/tools/acoustic_prof.py --summarize $O/$n/run_kernel_trace.csv | head -6
done
