#!/bin/bash
# usage (on the GPU box): bash tools/evidence.sh <tag>
# Round evidence in one call, everything under gpurun_out/<tag>/:
#   1. PMC traffic of the default C2 step (separate FETCH_SIZE / WRITE_SIZE passes) ->
#      profiles/<tag>_pmc_traffic_c2.json (bench.py reads the file profiles/pmc_current.json names
#      for roofline.traffic: point it at the new tag), and of the
#      C3 vocoder (bf16, 864 frames) -> profiles/<tag>_pmc_traffic_c3voc_bf16.json
#      (full_pipeline.roofline.traffic);
#   2. the default bench line (bench.json);
#   3. the rocprofv3 --kernel-trace --stats summary of the same bench command, and the C2 step
#      breakdown from a C2-only trace;
#   4. GPU clock / MFMA-busy per C2 dispatch (one PMC pass).
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O
bash $R/tools/pmc_traffic.sh $T/pmc || exit 1
python3 $R/tools/pmc_traffic.py $O/pmc/FETCH_SIZE $O/pmc/WRITE_SIZE $O/${T}_pmc_traffic_c2.json > $O/pmc_traffic.txt || exit 1
cp $O/${T}_pmc_traffic_c2.json $R/profiles/
# the C3 vocoder (bf16, 864 frames): full_pipeline.roofline.traffic
bash $R/tools/pmc_traffic.sh $T/pmc_c3 --dtype bf16 --frames 864 || exit 1
python3 $R/tools/pmc_traffic.py $O/pmc_c3/FETCH_SIZE $O/pmc_c3/WRITE_SIZE $O/${T}_pmc_traffic_c3voc_bf16.json 32 864 > $O/pmc_traffic_c3.txt || exit 1
cp $O/${T}_pmc_traffic_c3voc_bf16.json $R/profiles/
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o run -- python3 $R/bench.py > $O/rocprof_bench.json 2> $O/rocprof.err || { tail -5 $O/rocprof.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/c2trace.log 2>&1 || exit 1
python3 $R/tools/step_breakdown.py $O/c2trace/run_kernel_trace.csv > $O/step_breakdown_c2.txt || exit 1
bash $R/tools/pmc_clock.sh $T/clock || exit 1
python3 $R/tools/pmc_clock.py $O/clock > $O/clock_mfma_c2.txt || exit 1
echo evidence done
