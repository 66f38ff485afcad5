#!/bin/bash
# round-5 evidence on the current code: GPU suite + smoke, then tools/evidence.sh (PMC traffic,
# bench line, rocprof stats, C2 breakdown, clock/MFMA) and the acoustic PMC tables
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
PARITY_LOG=$O/parity_errors.json timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash tools/evidence.sh $T > $O/evidence.log 2>&1 || { tail -20 $O/evidence.log; exit 1; }
tail -2 $O/evidence.log
bash tools/pmc_acoustic.sh $T/pmc_ac > $O/pmc_ac.log 2>&1 || { tail -20 $O/pmc_ac.log; exit 1; }
cat $O/bench.json
