#!/bin/bash
# round 6: the fp32 decoder's FFN down-projections (K = 4,608) on the packed split-K form when the
# decoder rows leave pad rows (TTS_F32_DEC_PACKED): a one-utterance probe against the goldens
# first (serialized kernels, short limit), then the acoustic / model / service / config GPU tests,
# C1 generate() with and without it, and the bench's C1 service first frame
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06ac}; O=$R/gpurun_out/$T; mkdir -p $O; cd /tmp
AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 python3 -u $R/tools/f32split_probe.py > $O/probe.txt 2>&1 || { tail -8 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
cd $R
PARITY_LOG=$O/parity_errors.json timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_model_gpu.py tests/test_service_gpu.py tests/test_configs_gpu.py > $O/gputest.log 2>&1 || { grep -E "FAILED|Error|assert" $O/gputest.log | head -20; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
cd /tmp
for rep in 1 2; do
  for v in off on; do
    S=0; [ $v = on ] && S=1
    TTS_F32_DEC_PACKED=$S timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_$v.$rep.txt 2>&1 || { tail -5 $O/c1_$v.$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/c1_$v.$rep.txt)"
  done
done
timeout -k 10 400 python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print('C1', d.get('c1'))"
echo $T done
