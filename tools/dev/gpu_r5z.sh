#!/bin/bash
# Round 5 final-tree pass: tools/gpu_check.sh (GPU tests, smoke, the driver's
# bench line, the kernel-trace summary, FETCH/WRITE/SQ PMC passes), then every
# config line (box identifiers and clocks in each) for BASELINE.md.
set -o pipefail
TAG=${1:-r5z}
bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 900 python3 -u tools/bench_configs.py c2 c3 c4 c5 c1s16 mono1 mono8 odd ptrs up s16rs conv planar oconv stream r32to48 r48to32 r96to48 r24to48 r16to48 r96to44 r44to96 r22to48 s16rs3 planar2 conv2 m22to48 s22to48 m44to96 m24to48 m16to48 s24to48 s96to44 c1odd --steps 15 --warmup 3 > gpurun_out/$TAG/configs.jsonl 2> gpurun_out/$TAG/configs.err || { tail -5 gpurun_out/$TAG/configs.err; exit 1; }
grep '^{' gpurun_out/$TAG/configs.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d.get('kernel'), d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))"
