#!/bin/bash
# round 6: GPU suite on the product library (fp32-split acoustic reverted), the C3 two-engine
# overlap probe, C1 generate(), and one C1 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06h}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/tools/c3_overlap_probe.py > $O/overlap.txt 2>&1 || { tail -20 $O/overlap.txt; exit 1; }
tail -1 $O/overlap.txt
timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1.txt 2>&1 || { tail -5 $O/c1.txt; exit 1; }
tail -1 $O/c1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1 -o run -- python3 $R/tools/c1_prof.py > $O/c1_prof.log 2>&1 || { tail -5 $O/c1_prof.log; exit 1; }
python3 $R/tools/kernel_summary.py $O/c1/run_kernel_trace.csv --top 30 > $O/c1_kernels.txt || exit 1
head -24 $O/c1_kernels.txt
echo $T done
