#!/bin/bash
# round 6: fp32 vocoder stages 2-3 (64 and 32 channels) on split-precision GEMMs (2-k-step ring slots):
# vocoder / model / service / config GPU tests, C1 generate() against the round-5 library, and the
# bench's C1 service first frame
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06j}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_vocoder_gpu.py tests/test_model_gpu.py tests/test_service_gpu.py tests/test_configs_gpu.py > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
cd /tmp
for rep in 1 2; do
  for v in base new; do
    L=$R/gonova-tts_amd/libtts_hip.so; [ $v = base ] && L=$R/gonova-tts_amd/libtts_hip_base.so
    TTS_LIB=$L timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_$v.$rep.txt 2>&1 || { tail -5 $O/c1_$v.$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/c1_$v.$rep.txt)"
  done
done
timeout -k 10 400 python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print('C1', d.get('c1'))"
echo $T done
