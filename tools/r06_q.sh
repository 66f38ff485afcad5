#!/bin/bash
# round 6: C4 with two engines per GPU taking the length buckets in turn (dist.py step 4) against
# one engine, same call (bench.py --workload c4 reports both), twice; the C4 GPU test
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r06q}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py -k c4 > $O/gputest.log 2>&1 || { grep -E "FAILED|Error" $O/gputest.log | head; tail -5 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for rep in 1 2; do
  timeout -k 10 400 python3 $R/bench.py --workload c4 --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_c4.$rep.json 2> $O/bench_c4.$rep.err || { tail -5 $O/bench_c4.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_c4.$rep.json')); print('C4', d['ms_per_step'], d.get('one_engine_ms_per_step'), d.get('two_engine_ms_per_step'), d['value'])"
done
echo $T done
