#!/bin/bash
# round 6: C1 service path without wait_for hops (queue fast paths, a plain admission get, a plain
# sender get) and the waveform copied to the host through pinned memory: model / service GPU
# tests, C1 generate() twice, the bench's C1 service first frame twice
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06k}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_service_gpu.py > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
cd /tmp
for rep in 1 2; do
  timeout -k 10 300 python3 $R/tools/c1_prof.py > $O/c1_new.$rep.txt 2>&1 || { tail -5 $O/c1_new.$rep.txt; exit 1; }
  echo "new $rep: $(tail -1 $O/c1_new.$rep.txt)"
done
for rep in 1 2; do
  timeout -k 10 400 python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-streaming --no-cpu-baseline > $O/bench_c1.$rep.json 2> $O/bench_c1.$rep.err || { tail -5 $O/bench_c1.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_c1.$rep.json')); print('C1', d.get('c1'))"
done
echo $T done
