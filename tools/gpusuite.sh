#!/bin/bash
# usage (GPU box): bash tools/gpusuite.sh <tag>
# The whole GPU suite (parity errors logged to gpurun_out/<tag>/parity_errors.json) and smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
PARITY_LOG=$O/parity_errors.json timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "$T gpusuite done"
