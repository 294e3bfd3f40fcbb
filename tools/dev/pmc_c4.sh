#!/bin/bash
# Dev (GPU box, repo root): config 4's per-kernel HBM traffic and SQ counters,
# each counter group a --pmc pass of its own (no tracing), over 2 timed calls
# of tools/bench_configs.py c4 (+1 warm-up, which the --calls division
# includes: 3 calls per pass).
#   tools/dev/pmc_c4.sh <tag>
set -o pipefail
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="WRITE_SIZE"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for k in 1 2 3; do
  eval C=\$P$k
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/p$k -o run --output-format csv -- python3 tools/bench_configs.py c4 --steps 2 --warmup 1 --no-check --no-box > $OUT/p$k.log 2>&1 || { tail -5 $OUT/p$k.log; exit 1; }
done
python3 tools/dev/pmc_kernels.py --calls 3 --out $OUT/c4_pmc.json --source "tools/dev/pmc_c4.sh: 3 config-4 calls per pass" $OUT/p1 $OUT/p2 $OUT/p3
