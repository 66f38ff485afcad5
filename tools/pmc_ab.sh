#!/bin/bash
# usage (on the GPU box): bash tools/pmc_ab.sh <tag> <lib.so> [more libs]
# Two PMC passes (--kernel-trace only, separate runs) over one C2 step per library build:
# (a) clock / MFMA-busy / wave states, (b) instruction mix and LDS; tools/pmc_ab.py reads them.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  case $L in /*) ;; *) L=$R/$L;; esac
  n=$(basename $L .so)
  TTS_LIB=$L timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/a_$n -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/a_$n.log 2>&1 || { tail -3 $O/a_$n.log; exit 1; }
  TTS_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/b_$n -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/b_$n.log 2>&1 || { tail -3 $O/b_$n.log; exit 1; }
done
echo pmc ab done
