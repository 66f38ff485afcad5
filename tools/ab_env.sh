#!/bin/bash
# usage (GPU box): bash tools/ab_env.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
# Same-box A/B of runtime switches on the C2 bench: each setting runs twice, alternating; then one
# rocprof kernel trace + C2 step breakdown per setting (the first setting's label is "a", ...).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  i=0
  for S in "$@"; do
    i=$((i+1))
    env $S timeout -k 10 200 python3 $R/bench.py --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/s$i.$rep.json 2> $O/s$i.$rep.err || { tail -5 $O/s$i.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s$i.$rep.json')); k=d['roofline']['kernels']; print('$S', $rep, d['ms_per_step'], {a: b['ms_per_step'] for a, b in k.items()})"
  done
done
cd /tmp && export TMPDIR=/tmp
i=0
for S in "$@"; do
  i=$((i+1))
  env $S timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_s$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/prof_s$i.log 2>&1 || exit 1
  python3 $R/tools/step_breakdown.py $O/prof_s$i/run_kernel_trace.csv > $O/bd_s$i.txt || exit 1
done
echo ab done
