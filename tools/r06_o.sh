#!/bin/bash
# round 6: C5 host-side split (tools/c5_host.py), twice
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06o}; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 python3 $R/tools/c5_host.py > $O/c5_host.$rep.txt 2>&1 || { tail -5 $O/c5_host.$rep.txt; exit 1; }
  cat $O/c5_host.$rep.txt | grep p50
done
echo $T done
