#!/bin/bash
# usage (GPU box): bash tools/ab_ac.sh <tag> "<ENV=V ...>" ["<ENV=V ...>" ...]
# Same-box A/B of runtime switches on the acoustic side measurements (C3 full pipeline, C5
# streaming): each setting runs twice, alternating.  ENV=V may be "X=" for the default.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  i=0
  for S in "$@"; do
    i=$((i+1))
    env $S timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-c4 --no-cpu-baseline --no-c1 > $O/s$i.$rep.json 2> $O/s$i.$rep.err || { tail -5 $O/s$i.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s$i.$rep.json')); f=d['full_pipeline']; s=d['streaming']; print('$S', $rep, 'C3', f['ms_per_step'], 'ac', f['acoustic_ms_per_step'], f.get('acoustic_ms_per_step_fast_encoder'), 'C5', s['p50_first_audio_ms'], s['fast_encoder']['p50_first_audio_ms'])"
  done
done
echo ab done
