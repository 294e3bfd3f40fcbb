#!/bin/bash
# Round 5, box pass b: the DMA-pattern microbenchmark, the rest of the
# headline ablation A/B, and the product's SQ stall buckets.
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 300 tools/ubench/bin/dma_pattern > gpurun_out/r5b/dma_pattern.txt 2>&1 || { cat gpurun_out/r5b/dma_pattern.txt; exit 1; }
cat gpurun_out/r5b/dma_pattern.txt
tools/ab_libs.sh 1 lib lib_abnobar lib_abprio1 lib_abprio2 lib_abnotaps 2>&1 | tee gpurun_out/r5b/ab.txt || exit 1
tools/pmc_stall.sh r5b/stall 2>&1 | tee gpurun_out/r5b/stall.txt
