#!/bin/bash
# Dev (GPU box, repo root): per config line one rocprofv3 --pmc pass of
# WRITE_SIZE and the L2's 64-B write requests to memory, over
# tools/bench_configs.py <line> --steps 2 --warmup 1 (3 calls).
#   tools/dev/write_survey.sh <tag> <line> ...
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $OUT/$L -o run --output-format csv -- python3 tools/bench_configs.py $L --steps 2 --warmup 1 --no-check --no-box > $OUT/$L.log 2>&1 || { tail -5 $OUT/$L.log; exit 1; }
  echo "$L done"
done
