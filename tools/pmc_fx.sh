#!/bin/bash
# Dev (GPU box, repo root): PMC passes over one config line of
# tools/bench_configs.py (fir, bq, up, ...; "bench": the headline bench.py
# command): where the kernel's wave time goes and its
# HBM bytes (FETCH_SIZE and WRITE_SIZE in passes of their own, never with a
# tracing domain).  Per-launch averages of the kernels whose name matches.
#   tools/pmc_fx.sh <tag> <fir|bq|up|...|bench> <kernel-name-substring>
set -o pipefail
TAG=${1:-fx}; CFG=${2:-fir}; KN=${3:-k_fir_rb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for k in 1 2 3 4; do
  eval C=\$P$k
  if [ "$CFG" = bench ]; then
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/p$k -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-check > $OUT/p$k.log 2>&1 || { tail -5 $OUT/p$k.log; exit 1; }
  else
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/p$k -o run --output-format csv -- python3 tools/bench_configs.py $CFG --steps 2 --warmup 1 --no-check > $OUT/p$k.log 2>&1 || { tail -5 $OUT/p$k.log; exit 1; }
  fi
  python3 - $OUT/p$k/run_counter_collection.csv "$KN" <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(per.items()):
    print(f"{c:24s} {sum(v.values()) / len(v):.5g}   ({len(v)} launches)")
PY
done
