#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_vocoder_gpu.py tests/test_configs_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
echo "== c5 split default"; timeout -k 10 200 python3 tools/c5_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== c5 split off"; TTS_PAIR_SPLIT=0 timeout -k 10 200 python3 tools/c5_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/r05_j.sh $T/trace > $O/trace.txt 2>&1 || { tail -5 $O/trace.txt; exit 1; }
grep -E "mrf_pair|upsample|chain" $O/trace.txt | tail -40
