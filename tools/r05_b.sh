#!/bin/bash
# round-5 GPU check: full GPU suite, then per-launch acoustic traces (conv_mt on / off) and the
# acoustic PMC passes on the current code
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
bash tools/ac_trace.sh $T/trace "ACOUSTIC_PROF_LAUNCHES=1 TTS_CONV_MT=1" "ACOUSTIC_PROF_LAUNCHES=1 TTS_CONV_MT=0" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -A24 "==" $O/trace.txt | grep -v "grid" | head -120
bash tools/pmc_acoustic.sh $T/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cat $O/pmc/pmc_acoustic_b32.txt $O/pmc/pmc_acoustic_b8.txt
