#!/bin/bash
# Round 5, first box pass: GPU tests, then the headline ablation A/B and the
# product's SQ stall buckets.  Every GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest_gpu.txt 2>&1 || { tail -20 gpurun_out/r5a/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/r5a/pytest_gpu.txt
tools/ab_libs.sh 2 lib lib_abnowait lib_abnodma lib_abnotaps lib_abnolgk lib_abnobar lib_abprio1 lib_abprio2 2>&1 | tee gpurun_out/r5a/ab.txt || exit 1
tools/pmc_stall.sh r5a/stall 2>&1 | tee gpurun_out/r5a/stall.txt
