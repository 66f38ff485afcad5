#!/bin/bash
# diagnostic: fused-LN bits vs separate launches for the product and variant libraries
R=$GRAFT_REPO_ROOT
for L in "" "$@"; do
  echo "== lib ${L:-product}"
  if [ -n "$L" ]; then export TTS_LIB=$R/gonova-tts_amd/$L; else unset TTS_LIB; fi
  timeout -k 10 200 python3 $R/tools/ln_bisect.py || exit 1
done
