#!/bin/bash
# usage (GPU box): bash tools/ab_full.sh <tag> <variant .so> [more variant .so ...]
# Same-box A/B of library builds on the C3 full pipeline (bf16 vocoder at 864 frames + acoustic):
# product and variants alternate, twice each; prints C3 ms, acoustic ms and the vocoder families.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
LIBS="$R/gonova-tts_amd/libtts_hip.so"
for L in "$@"; do case $L in /*) LIBS="$LIBS $L";; *) LIBS="$LIBS $R/$L";; esac; done
for rep in 1 2; do
  for L in $LIBS; do
    n=$(basename $L .so)
    TTS_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/$n.$rep.json 2> $O/$n.$rep.err || { tail -5 $O/$n.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$n.$rep.json')); f=d['full_pipeline']; k=f.get('roofline', {}).get('kernels', {}); print('$n', $rep, 'C2', d['ms_per_step'], 'C3', f['ms_per_step'], 'ac', f['acoustic_ms_per_step'], {a: b['ms_per_step'] for a, b in k.items()})"
  done
done
echo ab done
