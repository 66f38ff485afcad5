#!/bin/bash
# round 6: (1) GPU tests of the acoustic / model / service paths on the new library (single-
# accumulator split GEMMs, 128-row tiles, /health device bytes); (2) same-box A/B against the
# round-5 library (base): batch-32 acoustic trace and the C3 line; (3) fp32 split-K slice cap
# (sk4 variant) at batch 1 / 8 / 32
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06c}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_model_gpu.py tests/test_service_gpu.py > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
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
    TTS_LIB=$L timeout -k 10 300 python3 $R/bench.py --no-c4 --no-c1 --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { tail -5 $O/bench_$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); f=d['full_pipeline']; s=d['streaming']; print('$v', $rep, 'C2', d['ms_per_step'], 'C3', f.get('ms_per_step'), 'ac', f.get('acoustic_ms_per_step'), 'C5', s.get('p50_first_audio_ms'))"
  done
done
for nb in 0 8 32; do
  for v in new sk4; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = sk4 ] && L=$R/gonova-tts_amd/libtts_hip_sk4.so
    C1_BATCH=$nb TTS_LIB=$L timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_${v}_$nb.txt 2>&1 || { tail -5 $O/c1_${v}_$nb.txt; exit 1; }
    echo "$v batch $nb: $(tail -1 $O/c1_${v}_$nb.txt)"
  done
done
echo $T done
