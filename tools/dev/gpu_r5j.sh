#!/bin/bash
# Round 5, box pass j: the whole GPU suite on the current tree, then config 2
# with box identifiers and the clocks sampled during its timed loop.
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r5j/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r5j/pytest_gpu.txt
timeout -k 10 600 python3 tools/bench_configs.py c2 --steps 400 --warmup 5 > gpurun_out/r5j/c2.jsonl 2>&1 || { tail -5 gpurun_out/r5j/c2.jsonl; exit 1; }
grep '^{' gpurun_out/r5j/c2.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); b=d.get('box',{}); print(d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'), d.get('clocks_during'), {k:v for k,v in b.items() if 'serial' in k.lower() or 'unique' in k.lower() or 'partition' in k.lower() or 'bus' in k.lower()})"
