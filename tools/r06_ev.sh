#!/bin/bash
# round-6 evidence on the current code: GPU suite + smoke, then tools/evidence.sh (PMC traffic,
# bench line, rocprof stats, C2 breakdown, clock/MFMA) and the acoustic PMC tables
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
PARITY_LOG=$O/parity_errors.json timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/evidence.sh $T > $O/evidence.log 2>&1 || { tail -20 $O/evidence.log; exit 1; }
tail -1 $O/evidence.log
bash tools/pmc_acoustic.sh $T/pmc_ac > $O/pmc_ac.log 2>&1 || { tail -20 $O/pmc_ac.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); f=d['full_pipeline']; print('C2', d['ms_per_step'], d['roofline']['frac'], 'C3', f['ms_per_step'], f.get('one_stream_ms_per_step'), 'ac', f['acoustic_ms_per_step'], 'C5', d.get('streaming', {}).get('p50_first_audio_ms'), 'C1', d.get('c1', {}).get('p50_first_frame_ms'), 'C4', d.get('c4', {}).get('ms_per_step'))"
echo "r06 evidence $T done"
