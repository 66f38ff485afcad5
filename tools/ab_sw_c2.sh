#!/bin/bash
# usage (GPU box): bash tools/ab_sw_c2.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
# Same-box A/B of runtime switches on the C2 step (vocoder only), two runs each, alternating.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  i=0
  for S in "$@"; do
    i=$((i+1))
    env $S timeout -k 10 200 python3 $R/bench.py --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/s$i.$rep.json 2> $O/s$i.$rep.err || { tail -5 $O/s$i.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s$i.$rep.json')); k=d['roofline']['kernels']; print('$S', $rep, d['ms_per_step'], {a: b['ms_per_step'] for a, b in k.items()})"
  done
done
echo ab done
