#!/bin/bash
# round 5: same-box A/B of the C2 step, the library before the fp32 split-K commits
# (TTS_LIB=libtts_hip_old.so, built from 0ddb4d4) vs the current one, alternated three times
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp
for rep in 1 2 3; do
  for v in old new; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = old ] && L=$R/gonova-tts_amd/libtts_hip_old.so
    TTS_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full --no-c4 --no-streaming --no-c1 > $O/c2.$v.$rep.json 2> $O/c2.$v.$rep.err || { tail -5 $O/c2.$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2.$v.$rep.json')); print('$v', $rep, d['ms_per_step'], d['roofline']['frac'])"
  done
done
echo r05zq done
