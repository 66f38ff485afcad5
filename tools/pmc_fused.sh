#!/bin/bash
# PMC passes over a short C2 bench (each pass its own run, --kernel-trace only)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1)); mkdir -p $O/pass$i
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pass$i -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-full --no-streaming --no-cpu-baseline --no-c1 > $O/pass$i/bench.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i/bench.log; exit 1; }
done
echo pmc done
