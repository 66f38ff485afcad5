#!/bin/bash
# usage (on the GPU box): bash tools/pmc_acoustic.sh <tag>
# PMC evidence of the acoustic forward (bf16, exact encoder) at batch 32 (C3) and batch 8 (C5):
# four passes per batch (separate runs, --kernel-trace only): clock / MFMA-busy / wave states,
# FETCH_SIZE, WRITE_SIZE, instruction mix + LDS bank conflicts; tools/pmc_acoustic.py reads them.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for B in 32 8; do
  P=(
    "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES"
    "FETCH_SIZE"
    "WRITE_SIZE"
    "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
  )
  for i in 0 1 2 3; do
    d=$O/b${B}_p$i
    ACOUSTIC_PROF_B=$B timeout -s KILL 120 rocprofv3 --pmc ${P[$i]} --kernel-trace --output-format csv -d $d -o run -- python3 $R/tools/acoustic_prof.py > $d.log 2>&1 || { echo "pass $B/$i failed"; tail -3 $d.log; exit 1; }
  done
  python3 $R/tools/pmc_acoustic.py $O/b${B}_p0 $O/b${B}_p1 $O/b${B}_p2 $O/b${B}_p3 $B > $O/pmc_acoustic_b$B.txt || exit 1
done
echo pmc acoustic done
