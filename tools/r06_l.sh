#!/bin/bash
# round 6: fp32 attention in 128-key chunks + merge (C1's batch-1 decoder): acoustic / model /
# service GPU tests, C1 generate() with and without the chunks (TTS_ATTN_F32_KC=0), one C1 kernel
# trace, and the bench's C1 service first frame
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06l}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_acoustic_gpu.py tests/test_model_gpu.py tests/test_service_gpu.py > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in kc0 kc128; do
    K=0; [ $v = kc128 ] && K=128
    TTS_ATTN_F32_KC=$K timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_$v.$rep.txt 2>&1 || { tail -5 $O/c1_$v.$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/c1_$v.$rep.txt)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c1 -o run -- python3 $R/tools/c1_prof.py > $O/c1_prof.log 2>&1 || { tail -5 $O/c1_prof.log; exit 1; }
python3 $R/tools/kernel_summary.py $O/c1/run_kernel_trace.csv --top 30 > $O/c1_kernels.txt || exit 1
head -24 $O/c1_kernels.txt
timeout -k 10 400 python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print('C1', d.get('c1'))"
echo $T done
