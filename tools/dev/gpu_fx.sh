#!/bin/bash
# Dev GPU pass for the effects kernels: effects tests, the fir / bq / c4
# config lines, and a kernel-trace profile of the bq and fir lines.
set -o pipefail
OUT=gpurun_out/${1:-fx}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "biquad or fir or effects or eq or chain" > $OUT/pytest_fx.log 2>&1 || { tail -30 $OUT/pytest_fx.log; exit 1; }
tail -2 $OUT/pytest_fx.log
timeout -k 10 300 python3 -u tools/bench_configs.py fir bq c4 > $OUT/cfg.log 2>&1 || { tail -5 $OUT/cfg.log; exit 1; }
grep '^{' $OUT/cfg.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o fx -- python3 tools/bench_configs.py fir bq --no-check > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -8
