#!/bin/bash
# usage (GPU box): bash tools/ab_xres.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
# Same-box A/B of runtime switches on the acoustic forward (B=32 and B=8 launch lists, per-kernel
# summary) and on the C2 step (trace + breakdown, upsamplers included).  "X=" is the default.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for S in "$@"; do
  i=$((i+1))
  for B in 32 8; do
    env $S ACOUSTIC_PROF_B=$B timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ac${B}_s$i -o run -- python3 $R/tools/acoustic_prof.py > $O/ac${B}_s$i.log 2>&1 || exit 1
    ACOUSTIC_PROF_LAUNCHES=1 python3 $R/tools/acoustic_prof.py --summarize $O/ac${B}_s$i/run_kernel_trace.csv > $O/ac${B}_s$i.sum || exit 1
    echo "$S B=$B: $(head -1 $O/ac${B}_s$i.sum)"
  done
  env $S timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2_s$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/c2_s$i.log 2>&1 || exit 1
  python3 $R/tools/step_breakdown.py $O/c2_s$i/run_kernel_trace.csv > $O/bd_s$i.txt || exit 1
  rm -rf $O/ac32_s$i $O/ac8_s$i $O/c2_s$i
done
echo ab done
