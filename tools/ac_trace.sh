#!/bin/bash
# usage (GPU box): bash tools/ac_trace.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
# Per-kernel time of one acoustic forward (tools/acoustic_prof.py under rocprofv3 --kernel-trace)
# at batch 8 and batch 32 for each setting (TTS_LIB=<variant .so> selects an A/B library build).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for S in "$@"; do
  i=$((i+1))
  for B in 8 32; do
    ( export $S ACOUSTIC_PROF_B=$B
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$i.b$B -o run -- python3 $R/tools/acoustic_prof.py > $O/t$i.b$B.log 2>&1 ) || { tail -5 $O/t$i.b$B.log; exit 1; }
    echo "== $S batch $B"
    python3 $R/tools/acoustic_prof.py --summarize $O/t$i.b$B/run_kernel_trace.csv | head -24
  done
done
echo trace done
