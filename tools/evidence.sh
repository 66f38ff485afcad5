#!/bin/bash
# usage (on the GPU box): bash tools/evidence.sh <tag>
# Round evidence in one call: PMC traffic of the default C2 step -> profiles/<tag>_pmc_traffic_c2.json
# (read by bench.py for roofline.traffic), the default bench line, and the rocprofv3
# --kernel-trace --stats summary of the same bench command.  Everything lands in gpurun_out/<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
bash $R/tools/pmc_traffic.sh $T/pmc || exit 1
python3 $R/tools/pmc_traffic.py $O/pmc/FETCH_SIZE $O/pmc/WRITE_SIZE $O/${T}_pmc_traffic_c2.json > /dev/null || exit 1
cp $O/${T}_pmc_traffic_c2.json $R/profiles/
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o run -- python3 $R/bench.py > $O/rocprof_bench.json 2> $O/rocprof.err || { tail -5 $O/rocprof.err; exit 1; }
echo evidence done
