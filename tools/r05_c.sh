#!/bin/bash
# conv_mt probes (no-DMA / no-MFMA / no-fragment-read builds) + PMC + the hipBLASLt yardstick
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 120 python3 tools/gemm_ref.py > $O/gemm_ref.txt 2>&1 || { tail -5 $O/gemm_ref.txt; exit 1; }
cat $O/gemm_ref.txt
bash tools/mt_probe.sh $T/probe mtp1 mtp2 mtp3
