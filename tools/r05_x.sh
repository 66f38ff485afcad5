#!/bin/bash
# round 5: batched variance predictors (first convs as one GEMM, first LayerNorms grouped) vs
# per-predictor launches (TTS_VP_BATCH=0): acoustic GPU tests, batch-8 / 32 traces, C3 / C5 A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash tools/ac_trace.sh $T/trace "X=" "TTS_VP_BATCH=0" > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -E "==|one forward|conv_splitp|layernorm" $O/trace.txt
bash tools/ab_ac.sh $T/ab "X=" "TTS_VP_BATCH=0" 2>&1 | tail -5
echo r05x done
