#!/bin/bash
# round 5: the vocoder at the frames the predicted durations give (model._synthesize_once) vs at
# the 12-per-token budget (TTS_VOC_TRIM=0): GPU suite, then C1 (the service path) A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for rep in 1 2; do
  for S in "X=" "TTS_VOC_TRIM=0"; do
    env $S timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline > $O/c1.$rep.json 2> $O/c1.$rep.err || { tail -5 $O/c1.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c1.$rep.json')); c=d['c1']; print('$S', $rep, 'C1 first frame', c['p50_first_frame_ms'], 'request', c['p50_request_ms'])"
  done
done
echo r05v done
