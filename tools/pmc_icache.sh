#!/bin/bash
# Dev (GPU box): instruction-cache counters of the headline kernel (SQ block,
# 8 counters = one pass; never combined with tracing).
#   tools/pmc_icache.sh <tag> [bench args...]
TAG=${1:-ic}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_INPUT_VALID_READYB SQ_IFETCH SQ_IFETCH_LEVEL \
    -d $OUT/p1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p1.log 2>&1 || { echo "icache pass failed rc=$?"; tail -5 $OUT/p1.log; exit 1; }
python3 tools/prof_summary.py $OUT k_rs147
