#!/bin/bash
# usage (on the GPU box): bash tools/pmc_clock.sh <outdir>
# One PMC pass (--kernel-trace only) over one default C2 step: GPU clock cycles per dispatch
# (GRBM_GUI_ACTIVE) next to MFMA-busy and wave-state cycles, for tools/pmc_clock.py.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
echo pmc clock done
