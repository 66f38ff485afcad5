#!/bin/bash
# round 5: C4 root waveform download -- per-bucket copies overlapped with the next bucket
# (default) vs all copies after the last bucket (TTS_C4_DEFER=1); same box, alternated
set -o pipefail
# (TTS_C4_DEFER was a temporary knob in dist.py for this A/B; removed after it, overlap kept)
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
env | grep -i -E "sdma|blit|^hsa_|^hip_|^gpu_|^roc" | sort > $O/env.txt; cat $O/env.txt
cd /tmp
for rep in 1 2 3; do
  for d in 0 1; do
    TTS_C4_DEFER=$d timeout -k 10 300 python3 $R/bench.py --workload c4 --steps 5 --warmup 2 > $O/c4.$d.$rep.json 2> $O/c4.$d.$rep.err || { tail -5 $O/c4.$d.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c4.$d.$rep.json')); print('defer $d rep $rep', d['value'], d['ms_per_step'])"
  done
done
echo r05zw done
