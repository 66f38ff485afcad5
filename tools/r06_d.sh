#!/bin/bash
# round 6: fp32 vocoder stages 0-1 on split-precision GEMMs (C1): the whole GPU suite on the new
# library, then C1 generate() against the round-5 library (base), alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06d}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 1000 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { grep -E "FAIL|Error|error" $O/gputest.log | head -20; tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
grep -E "range-guard fallback|service frame" $O/gputest.log | head
cd /tmp
for rep in 1 2; do
  for v in base new; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = base ] && L=$R/gonova-tts_amd/libtts_hip_base.so
    TTS_LIB=$L timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_$v.$rep.txt 2>&1 || { tail -5 $O/c1_$v.$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/c1_$v.$rep.txt)"
  done
done
for nb in 8 32; do
  C1_BATCH=$nb timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_new_b$nb.txt 2>&1 || { tail -5 $O/c1_new_b$nb.txt; exit 1; }
  echo "new batch $nb: $(tail -1 $O/c1_new_b$nb.txt)"
done
echo $T done
