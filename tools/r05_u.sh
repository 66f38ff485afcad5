#!/bin/bash
# round 5: cost of the decoder-extent read with a pinned host buffer: C3 (exact budget) with the
# read forced (TTS_DEC_TRIM=1) vs never (0), and C5 default vs never; the trim test
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py -k "trim or predicted" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ab_ac.sh $T/ab "X=" "TTS_DEC_TRIM=1" "TTS_DEC_TRIM=0" 2>&1 | tail -7
echo r05u done
