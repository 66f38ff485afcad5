#!/bin/bash
# usage (on the GPU box): bash tools/ab_env.sh <tag> <bench flags> "<env settings A>" "<env settings B>" ...
#   e.g. bash tools/ab_env.sh r04e_ws "--no-full --no-c4 --no-streaming --no-c1" "TTS_MRF_CHAIN=0" "TTS_MRF_CHAIN=1"
# Same-box A/B of runtime switches (switches.h): each setting runs bench.py alternately, twice,
# then one rocprof kernel trace + per-launch breakdown per setting.  Box-to-box clock
# differences (~5 %) exceed most single-change effects, so compare only within one call.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; FL="$2"; shift 2; mkdir -p $O
i=0
for rep in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    env $E timeout -k 10 200 python3 $R/bench.py $FL --no-cpu-baseline > $O/v$i.$rep.json 2> $O/v$i.$rep.err || { tail -5 $O/v$i.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/v$i.$rep.json')); k=d['roofline']['kernels']; print('$E', $rep, d['ms_per_step'], {a: b['ms_per_step'] for a, b in k.items()})"
  done
done
cd /tmp && export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i + 1))
  for kv in $E; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_v$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 $FL --no-cpu-baseline > $O/prof_v$i.log 2>&1 || exit 1
  for kv in $E; do unset "${kv%%=*}"; done
  python3 $R/tools/step_breakdown.py $O/prof_v$i/run_kernel_trace.csv > $O/bd_v$i.txt || exit 1
done
echo ab done
