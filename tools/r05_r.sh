#!/bin/bash
# round 5: decoder extent trimmed to the longest utterance with predicted durations (TTS_DEC_TRIM,
# default on): GPU suite, the t_cap probe with and without, and the C3 / C5 bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for S in "X=" "TTS_DEC_TRIM=0"; do
  echo "== tcap_probe $S"; env $S timeout -k 10 200 python3 tools/tcap_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/ab_ac.sh $T/ab "X=" "TTS_DEC_TRIM=0" 2>&1 | tail -5
echo r05r done
