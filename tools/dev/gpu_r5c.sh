#!/bin/bash
# Round 5, box pass c: what the product's other traffic does to its DMA stream
# (microbenchmark modes), and the store ablations of the fused kernel.
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_edges.py tests/test_gpu_fast_multisp.py -x -v -q --timeout 120 --timeout-method thread > gpurun_out/r5c/pytest_edges.txt 2>&1 || { tail -30 gpurun_out/r5c/pytest_edges.txt; exit 1; }
tail -2 gpurun_out/r5c/pytest_edges.txt
timeout -k 10 300 tools/ubench/bin/dma_pattern modes > gpurun_out/r5c/dma_modes.txt 2>&1 || { cat gpurun_out/r5c/dma_modes.txt; exit 1; }
cat gpurun_out/r5c/dma_modes.txt
tools/ab_libs.sh 1 lib lib_abnt lib_abntns lib_abntnw lib_abntnb lib_abntne lib_abntnc lib_abntp8 lib_abntall lib_abp8 lib_abnodma 2>&1 | tee gpurun_out/r5c/ab.txt || exit 1
timeout -k 10 300 python3 tools/bench_configs.py c4 --steps 10 --warmup 3 > gpurun_out/r5c/c4.txt 2>&1 || { tail -5 gpurun_out/r5c/c4.txt; exit 1; }
tail -3 gpurun_out/r5c/c4.txt
tools/dev/pmc_c4.sh r5c/c4 > gpurun_out/r5c/c4_pmc.txt 2>&1 || { tail -5 gpurun_out/r5c/c4_pmc.txt; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5c/c4/c4_pmc.json')); [print(k, round(v.get('launches',0),1), round(v.get('fetch_GB',0),3), round(v.get('write_GB',0),3)) for k,v in d['per_call'].items()]; print(d['per_call_total'])"
