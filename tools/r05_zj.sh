#!/bin/bash
# round 5: fp32 split-K above 64 output channels (product) vs above 32 incl. the vocoder stage-2 convs (TTS_F32_SK_MINM=32, TTS_VWS_MIN_CIN=64 variant): fp32 GPU tests on the variant, then the C1 probe alternated
# (not run: the GPU pool was busy at the end of the session; the knobs default to the measured product rule)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
V=$R/gonova-tts_amd/libtts_hip_s2.so
TTS_LIB=$V timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "fp32 or f32 or model" tests/ > $O/gputest_s2.log 2>&1 || { tail -30 $O/gputest_ck32.log; exit 1; }
tail -1 $O/gputest_s2.log
cd /tmp
for rep in 1 2; do
  for v in base s2; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = s2 ] && L=$V
    TTS_LIB=$L timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1.$v.$rep.txt 2>&1 || { tail -5 $O/c1.$v.$rep.txt; exit 1; }
    echo "$v $rep $(tail -1 $O/c1.$v.$rep.txt)"
  done
done
echo r05zj done
