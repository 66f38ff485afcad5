#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for L in "" attnold; do
  lib=$R/gonova-tts_amd/libtts_hip${L:+_$L}.so
  echo "== bitcmp ${L:-product}"; TTS_LIB=$lib timeout -k 10 200 python3 tools/bitcmp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ac_trace.sh $T/trace "X=" "TTS_LIB=$R/gonova-tts_amd/libtts_hip_attnold.so" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -E "==|one forward|rel_attn" $O/trace.txt
bash tools/ab_ac.sh $T/lnab "X=" "TTS_LN_FUSE=7" 2>&1 | tail -5
