#!/bin/bash
# Dev (GPU box, repo root): where the biquad kernel's wave time goes.
# Two --pmc passes over tools/dev/bq_load.py (config-4 biquad stage).
#   tools/pmc_bq.sh <tag> [libxm_audio.so]
set -o pipefail
TAG=${1:-bq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$2" ] && export XM_AUDIO_LIB=$2
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_IFETCH"
for k in 1 2; do
  eval C=\$P$k
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/p$k -o run --output-format csv -- python3 tools/dev/bq_load.py > $OUT/p$k.log 2>&1 || { tail -5 $OUT/p$k.log; exit 1; }
  python3 - $OUT/p$k/run_counter_collection.csv <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "biquad" in r["Kernel_Name"]:
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(per.items()):
    print(f"{c:24s} {sum(v.values()) / len(v):.5g}")
PY
done
