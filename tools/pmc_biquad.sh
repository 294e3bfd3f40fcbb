#!/bin/bash
# PMC issue/stall counters for the config-4 biquad kernel alone (dev; GPU box,
# repo root).  One --pmc pass per set, each under its own limit.
OUT=gpurun_out/pmc_bq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/dev/bq_load.py > $OUT/plain.log 2>&1 || { tail -5 $OUT/plain.log; exit 1; }
grep pass $OUT/plain.log
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
  "SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_IFETCH SQ_INSTS_BRANCH" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/dev/bq_load.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
for f in $OUT/p*/run_counter_collection.csv; do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "biquad" not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc):
    print(f"{k:28s} {acc[k] / max(1, len({1})):.4g}  (summed over {n[k]} rows)")
PY
done
