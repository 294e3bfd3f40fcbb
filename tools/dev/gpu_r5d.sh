#!/bin/bash
# Round 5, box pass d: output-store forms beside the fused kernel's DMA stream.
set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 300 tools/ubench/bin/dma_pattern stores > gpurun_out/r5d/dma_stores.txt 2>&1 || { cat gpurun_out/r5d/dma_stores.txt; exit 1; }
cat gpurun_out/r5d/dma_stores.txt
