#!/bin/bash
# round 5: C = 32 k = 11 pairs with the residual rows in registers at three blocks per CU
# (254-row tiles: libtts_hip_rr32_254.so) vs the product (502 rows, residual re-read) and vs
# 254-row tiles alone (libtts_hip_bn32_254.so): C2 A/B and mrf_pair traffic
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
TTS_LIB=$R/gonova-tts_amd/libtts_hip_rr32_254.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_vocoder_gpu.py > $O/tests_rr.txt 2>&1 || { tail -30 $O/tests_rr.txt; exit 1; }
tail -1 $O/tests_rr.txt
bash tools/ab.sh $T/ab gonova-tts_amd/libtts_hip_rr32_254.so gonova-tts_amd/libtts_hip_bn32_254.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for L in rr32_254; do
  TTS_LIB=$R/gonova-tts_amd/libtts_hip_$L.so bash tools/pmc_traffic.sh $T/pmc_$L > $O/pmc_$L.log 2>&1 || { tail -5 $O/pmc_$L.log; exit 1; }
  python3 tools/pmc_traffic.py $O/pmc_$L/FETCH_SIZE $O/pmc_$L/WRITE_SIZE $O/pmc_$L.json > $O/pmc_$L.txt 2>&1 || { tail -5 $O/pmc_$L.txt; exit 1; }
done
echo r05y done
