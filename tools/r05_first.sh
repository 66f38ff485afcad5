#!/bin/bash
# round-5 first GPU check: conv_mt vs conv_xres per layer, the new GPU tests, C3/C5 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd $R
echo "== mt_bench conv_mt"; timeout -k 10 150 python3 -u tools/mt_bench.py > $O/mt_on.txt 2>&1 || { tail -20 $O/mt_on.txt; exit 1; }
cat $O/mt_on.txt
echo "== mt_bench conv_xres"; TTS_CONV_MT=0 timeout -k 10 150 python3 -u tools/mt_bench.py > $O/mt_off.txt 2>&1 || { tail -20 $O/mt_off.txt; exit 1; }
cat $O/mt_off.txt
echo "== tests"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_service_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
echo "== C3/C5 A/B"
bash tools/ab_ac.sh $1/ab "TTS_CONV_MT=" "TTS_CONV_MT=0"
