#!/bin/bash
# Dev (GPU box, repo root): where the generic resample kernel's time goes, on
# one headline-shaped variant of tools/bench_configs.py.  Two --pmc passes.
#   tools/pmc_generic.sh <tag> [config=up]
set -o pipefail
TAG=${1:-gen}; CFG=${2:-up}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE"
for k in 1 2; do
  eval C=\$P$k
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/p$k -o run --output-format csv -- python3 tools/bench_configs.py $CFG --steps 1 --warmup 0 > $OUT/p$k.log 2>&1 || { tail -5 $OUT/p$k.log; exit 1; }
  python3 - $OUT/p$k/run_counter_collection.csv <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "generic" in r["Kernel_Name"]:
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(per.items()):
    print(f"{c:24s} {sum(v.values()) / len(v):.5g}")
PY
done
