#!/bin/bash
# round-6 final evidence, part B: tools/evidence.sh (PMC traffic, the default bench line, rocprof
# stats of the same command, C2 breakdown, clock / MFMA)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
bash tools/evidence.sh $T > $O/evidence.log 2>&1 || { tail -20 $O/evidence.log; exit 1; }
tail -1 $O/evidence.log
python3 -c "import json; d=json.load(open('$O/bench.json')); f=d['full_pipeline']; print('C2', d['ms_per_step'], d['roofline']['frac'], 'C3', f['ms_per_step'], f.get('one_stream_ms_per_step'), 'ac', f['acoustic_ms_per_step'], 'C5', d.get('streaming', {}).get('p50_first_audio_ms'), 'C1', d.get('c1', {}).get('p50_first_frame_ms'), 'C4', d.get('c4', {}).get('ms_per_step'))"
echo "$T part B done"
