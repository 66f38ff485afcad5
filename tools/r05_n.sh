#!/bin/bash
# round 5: (1) lazy attention rescale (product) vs eager (libtts_hip_eager.so): acoustic GPU tests
# and per-kernel acoustic traces; (2) row-pass store cache policy of the pair / chain kernels
# (nt vs sc1 vs sc0 sc1): same-box C2 A/B, then FETCH/WRITE passes per build (mrf_pair traffic)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ac_trace.sh $T/trace "X=" "TTS_LIB=$R/gonova-tts_amd/libtts_hip_eager.so" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -E "==|one forward|rel_attn" $O/trace.txt
bash tools/ab.sh $T/ab gonova-tts_amd/libtts_hip_rs16.so gonova-tts_amd/libtts_hip_rs17.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for L in "" rs16 rs17; do
  lib=$R/gonova-tts_amd/libtts_hip${L:+_$L}.so
  TTS_LIB=$lib bash tools/pmc_traffic.sh $T/pmc_${L:-prod} > $O/pmc_${L:-prod}.log 2>&1 || { tail -5 $O/pmc_${L:-prod}.log; exit 1; }
  python3 tools/pmc_traffic.py $O/pmc_${L:-prod}/FETCH_SIZE $O/pmc_${L:-prod}/WRITE_SIZE $O/pmc_${L:-prod}.json > $O/pmc_${L:-prod}.txt 2>&1 || { tail -5 $O/pmc_${L:-prod}.txt; exit 1; }
  grep -i "mrf_pair\|total" $O/pmc_${L:-prod}.txt
done
echo r05n done
