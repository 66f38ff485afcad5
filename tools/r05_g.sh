#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py -k "macro_tile" > $O/t_mt.txt 2>&1 || { tail -40 $O/t_mt.txt; exit 1; }
tail -1 $O/t_mt.txt
for B in 32 8; do for S in "X=" "TTS_MT_TILE=4" "TTS_MT_TILE=5" "TTS_MT_TILE=6" "TTS_MT_TILE=7" "TTS_MT_TILE=8" "TTS_MT_TILE=9" "TTS_MT_TILE=10" "TTS_CONV_MT=2"; do
  echo "== b$B $S"; env $S MT_B=$B timeout -k 10 120 python3 tools/mt_bench.py ffn_up ffn_down 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for S in "TTS_MT_TILE=4" "TTS_MT_TILE=5"; do
echo "== tp5 $S"; env $S TTS_LIB=$R/gonova-tts_amd/libtts_hip_tp5.so timeout -k 10 120 python3 tools/mt_bench.py ffn_up ffn_down 2>&1 | grep -v amdgpu.ids || exit 1
done
