#!/bin/bash
# conv_tap (multi-tap conv_mt form): correctness, per-config timing, traces
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py -k "macro_tile" > $O/t_mt.txt 2>&1 || { tail -40 $O/t_mt.txt; exit 1; }
tail -2 $O/t_mt.txt
for S in "X=" "TTS_MT_TILE=4" "TTS_MT_TILE=5" "TTS_MT_TILE=6" "TTS_MT_TILE=7" "TTS_MT_TILE=8" "TTS_CONV_MT=2"; do
  echo "== $S"; env $S timeout -k 10 120 python3 tools/mt_bench.py ffn_up ffn_down 2>&1 | grep -v amdgpu.ids || exit 1
done
for S in "X=" "TTS_MT_TILE=4" "TTS_MT_TILE=5" "TTS_MT_TILE=7" "TTS_MT_TILE=8" "TTS_CONV_MT=2"; do
  echo "== b8 $S"; env $S MT_B=8 timeout -k 10 120 python3 tools/mt_bench.py ffn_up ffn_down 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
bash tools/ac_trace.sh $T/trace "ACOUSTIC_PROF_LAUNCHES=1 X=" "ACOUSTIC_PROF_LAUNCHES=1 TTS_CONV_MT=0" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -A8 "==" $O/trace.txt | grep -v grid
