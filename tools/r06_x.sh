#!/bin/bash
# round 6: the decoder-extent read skipped on a capturing stream: the acoustic GPU tests
# (the new graph-capture test among them) and the model tests
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06x}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_model_gpu.py > $O/gputest.log 2>&1 || { grep -E "FAILED|Error|assert" $O/gputest.log | head -20; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
echo $T done
