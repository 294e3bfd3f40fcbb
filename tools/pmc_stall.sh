#!/bin/bash
# Dev (GPU box, repo root): where the headline kernel's wave time goes.
# One --pmc pass (SQ cycle buckets + GRBM clock) over a short bench run.
#   tools/pmc_stall.sh <tag> [bench args]
set -o pipefail
TAG=${1:-stall}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu --no-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-trace -d $OUT/p -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p.log 2>&1 || { tail -5 $OUT/p.log; exit 1; }
python3 - $OUT/p/run_counter_collection.csv <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs147" in r["Kernel_Name"]:
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(per.items()):
    print(f"{c:24s} {sum(v.values()) / len(v):.5g}")
PY
