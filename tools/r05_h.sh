#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for L in tp5 tp6 tp7; do for S in "TTS_MT_TILE=5" "TTS_MT_TILE=10"; do
  echo "== $L $S"; env $S TTS_LIB=$R/gonova-tts_amd/libtts_hip_$L.so timeout -k 10 120 python3 tools/mt_bench.py ffn_up ffn_down 2>&1 | grep -v amdgpu.ids || exit 1
done; done
