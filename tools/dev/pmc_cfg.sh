#!/bin/bash
# Dev (GPU box, repo root): one config line's per-kernel HBM traffic and SQ
# counters, each counter group a --pmc pass of its own (no tracing), over
# STEPS timed calls + 1 warm-up of tools/bench_configs.py <config> (the
# --calls division includes the warm-up).
#   tools/dev/pmc_cfg.sh <tag> <config> [steps]
set -o pipefail
TAG=${1:?tag}; CFG=${2:?config}; STEPS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="WRITE_SIZE"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P4="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR SQ_INSTS_BRANCH"
P5="GRBM_GUI_ACTIVE GRBM_COUNT"
for k in 1 2 3 4 5; do
  eval C=\$P$k
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/p$k -o run --output-format csv -- python3 tools/bench_configs.py $CFG --steps $STEPS --warmup 1 --no-check --no-box > $OUT/p$k.log 2>&1 || { tail -5 $OUT/p$k.log; exit 1; }
done
python3 tools/dev/pmc_kernels.py --calls $((STEPS + 1)) --out $OUT/${CFG}_pmc.json --source "tools/dev/pmc_cfg.sh $CFG: $((STEPS + 1)) calls per pass" $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 $OUT/p5
