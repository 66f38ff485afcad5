#!/bin/bash
# round 5: register-resident residual rows in the pair kernel (libtts_hip_resreg.so, OCC 2) vs the
# product (OCC 3, residual re-read at the row pass): bit-identity, same-box C2 A/B, FETCH/WRITE traffic
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for L in "" resreg; do
  echo "== bitcmp ${L:-product}"; TTS_LIB=$R/gonova-tts_amd/libtts_hip${L:+_$L}.so timeout -k 10 200 python3 tools/bitcmp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/ab.sh $T/ab gonova-tts_amd/libtts_hip_resreg.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
TTS_LIB=$R/gonova-tts_amd/libtts_hip_resreg.so bash tools/pmc_traffic.sh $T/pmc_resreg > $O/pmc_resreg.log 2>&1 || { tail -5 $O/pmc_resreg.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_resreg/FETCH_SIZE $O/pmc_resreg/WRITE_SIZE $O/pmc_resreg.json > $O/pmc_resreg.txt 2>&1 || { tail -5 $O/pmc_resreg.txt; exit 1; }
echo r05o done
