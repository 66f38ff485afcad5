#!/bin/bash
# round 6: in-kernel clock (s_memtime / s_memrealtime, after >= 3 s of back-to-back forwards) of the
# batch-32 acoustic GEMMs -- conv_xres (decoder, 16-bit) and conv_splitp (exact encoder) -- plus a
# same-box baseline bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06a; mkdir -p $O; cd $R
V=$R/gonova-tts_amd/libtts_hip_stamp.so
for t in ffn_up ffn_down qkv E_ffn_up E_ffn_down E_qkv; do
  STAMP_WARM_S=3 TTS_LIB=$V timeout -k 10 120 python3 -u tools/xres_stamps.py $t > $O/stamp_$t.txt 2>&1 || { tail -20 $O/stamp_$t.txt; exit 1; }
  head -3 $O/stamp_$t.txt
done
cd /tmp
timeout -k 10 400 python3 $R/bench.py --no-c4 --no-cpu-baseline --no-c1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); f=d['full_pipeline']; print(d['ms_per_step'], d['roofline']['frac'], f.get('acoustic_ms_per_step'), d.get('streaming',{}).get('p50_ms'))"
echo r06a done
