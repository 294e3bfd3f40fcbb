#!/bin/bash
# Round 5, box pass i: the 147/320 two-phase kernel (tests, bench line).
set -o pipefail
mkdir -p gpurun_out/r5i
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast_d2.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5i/pytest.txt 2>&1 || { tail -40 gpurun_out/r5i/pytest.txt; exit 1; }
tail -3 gpurun_out/r5i/pytest.txt
timeout -k 10 600 python3 tools/bench_configs.py r96to44 --steps 10 --warmup 3 > gpurun_out/r5i/configs.jsonl 2>&1 || { tail -5 gpurun_out/r5i/configs.jsonl; exit 1; }
grep '^{' gpurun_out/r5i/configs.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('kernel'), d.get('parity_check'))"
