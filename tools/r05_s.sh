#!/bin/bash
# round 5: 96-row conv_xres tiles for unevenly filled small grids (product) vs none
# (libtts_hip_nont3.so): acoustic GPU tests, batch-8 / 32 acoustic traces, C3 / C5 bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ac_trace.sh $T/trace "X=" "TTS_LIB=$R/gonova-tts_amd/libtts_hip_nont3.so" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -E "==|one forward|conv_xres" $O/trace.txt
bash tools/ab_ac.sh $T/ab "X=" "TTS_LIB=$R/gonova-tts_amd/libtts_hip_nont3.so" 2>&1 | tail -5
echo r05s done
