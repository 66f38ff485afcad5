#!/bin/bash
# round 6: fp32 models on split-precision acoustic GEMMs + attention (C1): GPU suite, C1 against
# the round-5 library, the C3 two-engine overlap probe, and one C1 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06f}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 1000 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputest.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" $O/gputest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base new; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = base ] && L=$R/gonova-tts_amd/libtts_hip_base.so
    TTS_LIB=$L timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_$v.$rep.txt 2>&1 || { tail -5 $O/c1_$v.$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/c1_$v.$rep.txt)"
  done
done
timeout -k 10 400 python3 $R/tools/c3_overlap_probe.py > $O/overlap.txt 2>&1 || { tail -20 $O/overlap.txt; exit 1; }
tail -1 $O/overlap.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1 -o run -- python3 $R/tools/c1_prof.py > $O/c1_prof.log 2>&1 || { tail -5 $O/c1_prof.log; exit 1; }
python3 $R/tools/kernel_summary.py $O/c1/run_kernel_trace.csv --top 30 > $O/c1_kernels.txt || exit 1
head -24 $O/c1_kernels.txt
echo $T done
