#!/bin/bash
# usage (on the GPU box): bash tools/ab.sh <tag> <variant .so> [more variant .so ...]
# Same-box A/B of library builds (python -m gonova_tts_amd.build --variant X -D...): the product
# library and each variant run the C2 bench alternately, twice each; then one rocprof kernel
# trace + per-launch breakdown per build.  Box-to-box clock differences (~5 %) exceed most
# single-change effects, so compare only within one call.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
LIBS="$R/gonova-tts_amd/libtts_hip.so"
for L in "$@"; do case $L in /*) LIBS="$LIBS $L";; *) LIBS="$LIBS $R/$L";; esac; done
for rep in 1 2; do
  for L in $LIBS; do
    n=$(basename $L .so)
    TTS_LIB=$L timeout -k 10 200 python3 $R/bench.py --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/$n.$rep.json 2> $O/$n.$rep.err || { tail -5 $O/$n.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$n.$rep.json')); k=d['roofline']['kernels']; print('$n', $rep, d['ms_per_step'], {a: b['ms_per_step'] for a, b in k.items()})"
  done
done
cd /tmp && export TMPDIR=/tmp
for L in $LIBS; do
  n=$(basename $L .so)
  TTS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$n -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/prof_$n.log 2>&1 || exit 1
  python3 $R/tools/step_breakdown.py $O/prof_$n/run_kernel_trace.csv > $O/bd_$n.txt || exit 1
done
echo ab done
