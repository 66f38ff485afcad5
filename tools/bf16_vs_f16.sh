#!/bin/bash
# usage (GPU box): bash tools/bf16_vs_f16.sh <tag>
# C2-shape vocoder step in fp16 and in bf16 (the C3 vocoder dtype): kernel traces and per-launch
# breakdowns side by side, for the bf16 epilogue / staging overhead.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for D in f16 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_$D -o run -- python3 $R/bench.py --dtype $D --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/t_$D.log 2>&1 || exit 1
  python3 $R/tools/step_breakdown.py $O/t_$D/run_kernel_trace.csv > $O/bd_$D.txt || exit 1
  rm -rf $O/t_$D
done
paste $O/bd_f16.txt $O/bd_bf16.txt | head -50
