#!/bin/bash
# round 6: C2 split over 2 / 4 engines on as many streams vs one stream (tools/c2_overlap_probe.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06p}; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/tools/c2_overlap_probe.py > $O/c2_overlap.txt 2>&1 || { tail -5 $O/c2_overlap.txt; exit 1; }
grep -v amdgpu.ids $O/c2_overlap.txt
echo $T done
