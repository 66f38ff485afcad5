#!/bin/bash
# Same-box A/B driver (GPU box).  Box-to-box clock differences (~5 %) exceed most single-change
# effects, so compare arms only within one call.
#
# usage: bash tools/ab.sh <tag> <workload> <arm> [<arm> ...]
#   workload  c2  bench.py headline (C2 vocoder step) + per-family times
#             c3  bench.py full pipeline (C3 step, acoustic ms) + C2
#             c5  bench.py streaming first audio (C5 p50, predicted and given durations)
#             c1  tools/c1_prof.py (fp32 generate() of the C1 sentence)
#             ac  acoustic forward at batch 32 and 8 under rocprofv3: per-kernel summary
#   arm       a library build (path ending in .so: python -m gonova_tts_amd.build --variant X -D...)
#             or runtime switches ("TTS_X=1 TTS_Y=0"; "-" = the defaults) on the product library
# The product library with default switches always runs first as arm "base".  Each arm runs twice,
# alternating (ac: once); results and logs go to gpurun_out/<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; W=$2; shift 2; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARMS=("-" "$@")
run_arm() {  # run_arm <arm> <label> <command...>: the arm's library / switches around one command
  local arm=$1 label=$2; shift 2
  local lib=$R/gonova-tts_amd/libtts_hip.so envs=()
  case $arm in
    *.so) case $arm in /*) lib=$arm;; *) lib=$R/$arm;; esac;;
    -) ;;
    *) read -ra envs <<< "$arm";;
  esac
  env TTS_LIB=$lib "${envs[@]}" timeout -k 10 400 "$@" > $O/$label.out 2> $O/$label.err || { tail -5 $O/$label.err; return 1; }
}
REPS=2; [ $W = ac ] && REPS=1
for rep in $(seq 1 $REPS); do
  i=0
  for arm in "${ARMS[@]}"; do
    lbl=arm$i.$rep; i=$((i + 1))
    case $W in
      c2) run_arm "$arm" $lbl python3 $R/bench.py --no-full --no-c4 --no-streaming --no-cpu-baseline --no-c1 || exit 1
          python3 -c "import json; d=json.load(open('$O/$lbl.out')); k=d['roofline']['kernels']; print('$arm', $rep, 'C2', d['ms_per_step'], {a: b['ms_per_step'] for a, b in k.items()})";;
      c3) run_arm "$arm" $lbl python3 $R/bench.py --no-c4 --no-streaming --no-cpu-baseline --no-c1 || exit 1
          python3 -c "import json; d=json.load(open('$O/$lbl.out')); f=d['full_pipeline']; print('$arm', $rep, 'C2', d['ms_per_step'], 'C3', f['ms_per_step'], 'acoustic', f['acoustic_ms_per_step'])";;
      c5) run_arm "$arm" $lbl python3 $R/bench.py --steps 3 --warmup 1 --no-full --no-c4 --no-cpu-baseline --no-c1 || exit 1
          python3 -c "import json; d=json.load(open('$O/$lbl.out')); s=d['streaming']; print('$arm', $rep, 'C5', {k: v for k, v in s.items() if 'ms' in k and not isinstance(v, (list, dict))})";;
      c1) run_arm "$arm" $lbl python3 $R/tools/c1_prof.py || exit 1
          echo "$arm $rep $(tail -1 $O/$lbl.out)";;
      ac) for b in 32 8; do
            run_arm "$arm" $lbl.b$b env ACOUSTIC_PROF_B=$b rocprofv3 --kernel-trace --output-format csv -d $O/$lbl.b$b -o run -- python3 $R/tools/acoustic_prof.py || exit 1
            python3 $R/tools/acoustic_prof.py --summarize $O/$lbl.b$b/run_kernel_trace.csv > $O/$lbl.b$b.txt || exit 1
            echo "== $arm batch $b"; head -12 $O/$lbl.b$b.txt
          done;;
      *) echo "unknown workload $W"; exit 2;;
    esac
  done
done
echo "ab $T done"
