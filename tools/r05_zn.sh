#!/bin/bash
# round 5: the fp32 split-K batch-invariance test and the rest of the acoustic / model / vocoder GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_model_gpu.py tests/test_vocoder_gpu.py > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
grep -E "split_k|passed|failed" $O/gputest.log | tail -3
