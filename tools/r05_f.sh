#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for L in "" tp1 tp2 tp4 tp5; do
  lib=$R/gonova-tts_amd/libtts_hip${L:+_$L}.so
  echo "== ${L:-product}"; TTS_LIB=$lib timeout -k 10 120 python3 tools/mt_bench.py ffn_up ffn_down 2>&1 | grep -v amdgpu.ids || exit 1
done
