#!/bin/bash
# usage (on the GPU box): bash tools/ab_c5.sh <tag> <variant .so> [more variant .so ...]
# Same-box A/B of library builds on the acoustic-heavy configurations: the C5 latency split
# (tools/c5_probe.py, batch 8) and the C3 full-pipeline step (bench.py --workload full),
# product library first, alternating, twice each.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
LIBS="$R/gonova-tts_amd/libtts_hip.so"
for L in "$@"; do case $L in /*) LIBS="$LIBS $L";; *) LIBS="$LIBS $R/$L";; esac; done
for rep in 1 2; do
  for L in $LIBS; do
    n=$(basename $L .so)
    TTS_LIB=$L timeout -k 10 200 python3 $R/tools/c5_probe.py > $O/$n.$rep.c5 2>&1 || { tail -5 $O/$n.$rep.c5; exit 1; }
    TTS_LIB=$L timeout -k 10 200 python3 $R/bench.py --workload full --steps 6 --warmup 2 --no-cpu-baseline > $O/$n.$rep.json 2> $O/$n.$rep.err || { tail -5 $O/$n.$rep.err; exit 1; }
    echo "$n $rep $(grep -v amdgpu $O/$n.$rep.c5 | tr -s ' ' | tr '\n' ';')"
    python3 -c "import json; d=json.load(open('$O/$n.$rep.json')); print('   C3', d['ms_per_step'], 'acoustic', d['acoustic_ms_per_step'])"
  done
done
echo ab_c5 done
