#!/bin/bash
# usage (GPU box): bash tools/mt_probe.sh <tag> [variant ...]
# tools/mt_bench.py with the product library and each variant build (libtts_hip_<variant>.so), then
# PMC passes (MFMA busy / clock / waits; LDS instruction mix and bank conflicts) on the product's
# FFN up-projection.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "== product"; timeout -k 10 120 python3 $R/tools/mt_bench.py || exit 1
for v in "$@"; do
  echo "== $v"; TTS_LIB=$R/gonova-tts_amd/libtts_hip_$v.so timeout -k 10 120 python3 $R/tools/mt_bench.py ffn_up ffn_down qkv || exit 1
done
P=("GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
   "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE")
for i in 0 1; do
  MT_ITERS=5 timeout -s KILL 60 rocprofv3 --pmc ${P[$i]} --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/mt_bench.py ffn_up > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, sys
from collections import defaultdict
O = sys.argv[1]
for i in (0, 1):
    per = defaultdict(lambda: defaultdict(float)); name = {}
    for r in csv.DictReader(open(f"{O}/p{i}/run_counter_collection.csv")):
        d = int(r["Dispatch_Id"]); per[d][r["Counter_Name"]] += float(r["Counter_Value"]); name[d] = r["Kernel_Name"]
    dur = {int(r["Dispatch_Id"]): (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
           for r in csv.DictReader(open(f"{O}/p{i}/run_kernel_trace.csv"))}
    ds = [d for d in per if "conv_mt" in name[d]][-3:]
    for d in ds:
        c = per[d]; t = dur[d]
        if i == 0:
            clk = c["GRBM_GUI_ACTIVE"] / 8 / t
            # SQ_VALU_MFMA_BUSY_CYCLES is summed over SIMDs (1024 of them)
            print(f"dispatch {d}: {t*1e6:.1f} us clock {clk/1e9:.2f} GHz  mfma busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * clk * t):.3f}"
                  f"  wait_any {c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES']:.3f} wait_inst {c['SQ_WAIT_INST_ANY']/c['SQ_WAVE_CYCLES']:.3f}")
        else:
            print(f"dispatch {d}: valu/mfma {c['SQ_INSTS_VALU']/c['SQ_INSTS_MFMA']:.2f} lds/mfma {c['SQ_INSTS_LDS']/c['SQ_INSTS_MFMA']:.2f}"
                  f" bank-conflict cyc/lds-inst {c['SQ_LDS_BANK_CONFLICT']/c['SQ_INSTS_LDS']:.2f}  lds idx active/lds inst {c['SQ_LDS_IDX_ACTIVE']/c['SQ_INSTS_LDS']:.2f}"
                  f" wait_inst_lds {c['SQ_WAIT_INST_LDS']/c['SQ_WAVE_CYCLES']:.3f}")
PY
