#!/bin/bash
# usage (on the GPU box): bash tools/pmc_traffic.sh <outdir> [bench.py args]
# FETCH_SIZE and WRITE_SIZE passes (separate runs, --kernel-trace only) over a short vocoder
# bench (default C2; e.g. "--dtype bf16 --frames 864" for the C3 vocoder), for tools/pmc_traffic.py.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  mkdir -p $O/$c
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 "$@" > $O/$c/bench.log 2>&1 || { echo "pass $c failed"; tail -5 $O/$c/bench.log; exit 1; }
done
echo pmc traffic done
