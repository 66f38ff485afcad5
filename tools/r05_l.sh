#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for rep in 1 2; do
for L in "" psw1 psw2 psw2n2 psw4n2 off; do
  lib=$R/gonova-tts_amd/libtts_hip${L:+_$L}.so; env=""
  if [ "$L" = off ]; then lib=$R/gonova-tts_amd/libtts_hip.so; env="TTS_PAIR_SPLIT=0"; fi
  echo "== ${L:-product} $rep"; env $env TTS_LIB=$lib timeout -k 10 200 python3 tools/c5_probe.py 2>&1 | grep -E "voc_dev|acoustic_dev" || exit 1
done; done
