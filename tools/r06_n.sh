#!/bin/bash
# round 6: C5 with the frame-count read enqueued before the first chunk (pinned copies + event) and
# no mel fill: model / service / config GPU tests, C5 p50 twice, one traced trial's timeline
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06n}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_service_gpu.py tests/test_configs_gpu.py tests/test_acoustic_gpu.py > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 python3 $R/tools/c5_trace.py > $O/c5_plain.$rep.txt 2>&1 || { tail -5 $O/c5_plain.$rep.txt; exit 1; }
  tail -1 $O/c5_plain.$rep.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c5 -o run -- python3 $R/tools/c5_trace.py > $O/c5_prof.log 2>&1 || { tail -5 $O/c5_prof.log; exit 1; }
python3 $R/tools/last_burst.py $O/c5/run_kernel_trace.csv > $O/c5_timeline.txt || exit 1
tail -1 $O/c5_timeline.txt
echo $T done
