#!/bin/bash
# round 6: split GEMMs on one accumulator (power-of-two weight scale) + 128-row tiles at batch 32:
# acoustic GPU tests on the new library, then same-box A/B against the round-5 library (base):
# per-launch acoustic trace at batch 32 and the C3 bench line, alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06b}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_model_gpu.py tests/test_service_gpu.py > $O/gputest_acoustic.log 2>&1 || { tail -30 $O/gputest_acoustic.log; exit 1; }
tail -2 $O/gputest_acoustic.log
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  L=$R/gonova-tts_amd/libtts_hip.so; [ $v = base ] && L=$R/gonova-tts_amd/libtts_hip_base.so
  TTS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ac_$v -o run -- python3 $R/tools/acoustic_prof.py > $O/ac_$v.log 2>&1 || { tail -5 $O/ac_$v.log; exit 1; }
  ACOUSTIC_PROF_LAUNCHES=1 python3 $R/tools/acoustic_prof.py --summarize $O/ac_$v/run_kernel_trace.csv > $O/ac_trace_$v.txt || exit 1
  head -8 $O/ac_trace_$v.txt
done
for rep in 1 2; do
  for v in base new; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = base ] && L=$R/gonova-tts_amd/libtts_hip_base.so
    TTS_LIB=$L timeout -k 10 300 python3 $R/bench.py --no-c4 --no-streaming --no-c1 --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { tail -5 $O/bench_$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); f=d['full_pipeline']; print('$v', $rep, d['ms_per_step'], f.get('ms_per_step'), f.get('acoustic_ms_per_step'))"
  done
done
echo $T done
